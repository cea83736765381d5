#!/usr/bin/env python3
"""bench.py -- headline benchmark: batched forward NTT/s (N = 2^16, L = 8, batch = 1024) on MI355X.

Workload (BASELINE.json configs[2], the N = 2^16 configuration the metric is quoted on):
  one step = one batched forward negacyclic NTT (phantom convention, mfhe_ntt_fwd) over a
  [1024][8][65536] u64 residue batch (4 GiB) resident in HBM.  Secondary line items:
  inverse NTT and encode+CRT ops/s (RNS decompose + wide CRT compose -> f64) on the same shape.

Multi-GPU: one process per GPU, residue-batch sharding -- every rank transforms its own batch (weak
scaling), no data-path collective; barrier + max-over-ranks timing.  Under a launcher (torchrun sets
WORLD_SIZE, which must equal --gpus) this process is one rank; `python bench.py --gpus N` with no
launcher starts the N ranks itself (launch_ranks) before anything touches the GPU.

Run: python bench.py [--gpus N --steps K --warmup W]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import traceback
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "matrix-fhe-gpu_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (/opt/skills/guides/MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log-n", type=int, default=16)
    ap.add_argument("--limbs", type=int, default=8)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--arith", type=int, default=0, help="0 auto, 1 f64, 2 u64")
    ap.add_argument("--ntt-wg", type=int, default=None, help="MFHE_OPT_NTT_WG_PER_CU override (tuning)")
    ap.add_argument("--ntt-prefetch", type=int, default=None, help="MFHE_OPT_NTT_PREFETCH override (tuning)")
    ap.add_argument("--ntt-chunk", type=int, default=None, help="MFHE_OPT_NTT_CHUNK_BYTES override (tuning)")
    ap.add_argument("--ntt-pack", type=int, default=None, help="MFHE_OPT_NTT_PACK override (tuning)")
    ap.add_argument("--ntt-plan", type=int, default=None, help="MFHE_OPT_NTT_PLAN override (tuning)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="skip the reference-geometry pipeline and other-config NTT lines (N=1 only)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-c5", action="store_true", help="skip the BASELINE C5 residue-shard line")
    ap.add_argument("--only", default="all", help="all | ntt | crt | recombine | c4 | c5 | u64 (profiling)")
    ap.add_argument("--recombine-batch", type=int, default=256,
                    help="polys per step for the residue-shard INTT + CRT recombine line (0 = skip)")
    ap.add_argument("--secondary-timeout", type=float, default=300.0,
                    help="seconds the lines after the headline may take before the watchdog prints the headline and exits")
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--hang-check", type=float, default=0.0, help=argparse.SUPPRESS)
    return ap.parse_args()


def gen_moduli(bits, m, count):
    """Largest `count` primes q < 2^bits with q = 1 mod m (deterministic; same as the oracle's)."""
    out = []
    c = ((2 ** bits - 2) // m) * m + 1
    while len(out) < count:
        if is_prime(c):
            out.append(c)
        c -= m
    return out


def is_prime(n):
    if n < 2:
        return False
    for p in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def pmc_traffic(N, L, batch):
    """HBM-side bytes per forward transform from the committed rocprofv3 FETCH_SIZE/WRITE_SIZE passes
    (tools/pmc_run.sh + tools/pmc_summary.py -> profiles/*pmc_ntt_traffic.json), if one was measured on
    this exact shape; counters cannot be read from inside a timed run."""
    import glob
    best = None
    for f in sorted(glob.glob(str(ROOT / "profiles" / "*pmc_ntt_traffic*.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        c = d.get("config", {})
        if (c.get("N"), c.get("limbs"), c.get("batch")) == (N, L, batch) and "fwd_traffic_bytes_per_transform" in d:
            best = (d["fwd_traffic_bytes_per_transform"], Path(f).name)
    return best


def prof_trace(N, L, batch):
    """The committed rocprofv3 kernel trace of the bench command (tools/prof_agree.py ->
    profiles/*ntt_rocprof_vs_event*.json) for this shape: the latest round's file wins."""
    import glob
    best = None
    for f in sorted(glob.glob(str(ROOT / "profiles" / "*ntt_rocprof_vs_event*.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        sh = d.get("shape", {})
        if (sh.get("N"), sh.get("limbs"), sh.get("batch")) == (N, L, batch) and "rocprof_kernel_ms_per_transform" in d:
            best = dict(d, file=Path(f).name)
    return best


def _warm(fn, min_s=0.05, max_calls=2000):
    """Untimed calls of fn for at least min_s of wall time (synchronised): the clock ramps over the first ~30 ms of
    work (profiles/r02_bench_steps.txt).  Single-rank lines only -- a rank-dependent call count would desynchronise
    the collectives of a multi-rank line."""
    import torch
    t_end = time.perf_counter() + min_s
    for n in range(1, max_calls + 1):
        fn()
        if n % 4 == 0:
            torch.cuda.synchronize()
            if time.perf_counter() >= t_end:
                break
    torch.cuda.synchronize()


def other_configs_line(reps=10):
    """The other BASELINE.json NTT shapes on this one GPU (parity cases, not the headline): C2 whole, and the
    per-GPU residue shard of C4 (4 GPUs) and C5 (8 GPUs).  Forward and inverse NTT/s, HIP events.

    C2's 128 MiB batch fits the 256 MiB Infinity Cache, so re-transforming one buffer measures the cache, not
    HBM: C2 is timed both ways -- one resident buffer ("cache_resident") and 8 rotating
    buffers of 128 MiB (1 GiB, each evicted before its next use: the HBM figure, which is the one `frac_fwd`
    is quoted on)."""
    import torch
    import mfhe
    res = {}
    for name, log_n, L, lg, batch, nbuf in (("C2: N=2^14 L=4 batch 256", 14, 4, 4, 256, 8),
                                           ("C4 shard: N=2^16 L=16 (4 of 16 limbs) batch 1024", 16, 16, 4, 1024, 1),
                                           ("C5 shard: N=2^17 L=32 (4 of 32 limbs) batch 4096", 17, 32, 4, 4096, 1)):
        N = 1 << log_n
        moduli = gen_moduli(50, 1 << (log_n + 2), L)
        ctx = mfhe.Context(moduli, log_n, mfhe.CONV_PHANTOM)
        qt = torch.tensor(moduli[:lg], dtype=torch.int64, device="cuda").repeat_interleave(N).repeat(batch)
        bufs = []
        for _ in range(nbuf):
            d = torch.empty(batch * lg * N, dtype=torch.int64, device="cuda")
            d.random_(0, 2 ** 62).remainder_(qt)
            bufs.append(d)
        del qt

        def rate(fn, nb):
            # warm up for >= 50 ms of calls, not a fixed count: the clock ramps over the first ~30 ms of work
            # (profiles/r02_bench_steps.txt), which a C2 call (~80 us) would otherwise spend inside the timed loop
            t_end = time.perf_counter() + 0.05
            k = 0
            while True:
                fn(bufs[k % nb], batch=batch, start_limb=0, nlimbs=lg)
                k += 1
                if k % nb == 0:
                    torch.cuda.synchronize()
                    if time.perf_counter() >= t_end:
                        break
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            n = reps * nb
            for k in range(n):
                fn(bufs[k % nb], batch=batch, start_limb=0, nlimbs=lg)
            e1.record()
            torch.cuda.synchronize()
            return batch * lg / (e0.elapsed_time(e1) / n * 1e-3)

        out = {}
        for kind, fn in (("fwd", ctx.ntt_fwd), ("inv", ctx.ntt_inv)):
            r = rate(fn, nbuf)
            out[f"{kind}_NTT_per_s"] = round(r)
            out[f"{kind}_alg_GBps"] = round(16.0 * N * r / 1e9, 1)
            if nbuf > 1:
                rc = rate(fn, 1)
                out[f"cache_resident_{kind}_NTT_per_s"] = round(rc)
                out[f"cache_resident_{kind}_alg_GBps"] = round(16.0 * N * rc / 1e9, 1)
        out["frac_fwd"] = round(out["fwd_alg_GBps"] / HBM_PEAK_GBS, 4)
        out["working_set_GiB"] = round(batch * lg * N * 8 / 2 ** 30, 3)
        if nbuf > 1:
            out["rotating_buffers"] = f"{nbuf} x {out['working_set_GiB']} GiB (HBM figure; cache_resident_*: one buffer)"
        res[name] = out
        del bufs
        ctx.close()
    return res


def pipeline_line(reps=10):
    """src/main.cu:31-157 flow at the reference geometry (n = 64, 512 W-lanes, the 11 reference moduli):
    encode -> encrypt_pair -> decrypt_and_decode, HIP-event timed, with main.cu's 1e-4 check."""
    import numpy as np
    import torch
    import mfhe
    ctx = mfhe.Context(mfhe.RNS_MODULI, 6, mfhe.CONV_PHANTOM | mfhe.CONV_WCRT)
    ctx.reserve_workspace()
    n2 = 64 * 64
    ell, i = np.meshgrid(np.arange(512), np.arange(n2), indexing="ij")
    msg = ((ell + i * 1e-5) + 1j * (ell - i * 1e-5)).ravel()          # main.cu:62-69
    mt = torch.from_numpy(msg.view(np.float64).copy()).cuda()
    words = 512 * 11 * n2
    sk = torch.empty(512 * 11 * 64, dtype=torch.int64, device="cuda")
    re_, im_ = (torch.empty(words, dtype=torch.int64, device="cuda") for _ in range(2))
    cre, cim = (torch.empty(2 * words, dtype=torch.int64, device="cuda") for _ in range(2))
    res = torch.empty_like(mt)
    ctx.keygen(sk)

    def run():
        ctx.encode(mt, re_, im_)
        ctx.encrypt_pair(re_, im_, sk, cre, cim)
        ctx.decrypt_and_decode(cre, cim, sk, res)
    _warm(run)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    err = float(np.max(np.abs(res.cpu().numpy().view(np.complex128) - msg)))
    ms = e0.elapsed_time(e1) / reps
    ctx.close()
    return {"workload": "encode->encrypt_pair->decrypt_and_decode, n=64 x 512 W-lanes x L=11 (reference geometry)",
            "ms": round(ms, 3), "messages_per_s": round(512 * n2 / (ms * 1e-3)), "max_err": err,
            "main_cu_check_1e-4": err < 1e-4}


def trace_line(reps=10):
    """Batched trace GEMM (batched_trace.cu:37-197) at the reference geometry: 512 matrices x L = 11 x
    n = 64: map B -> B', C = n A B'^T (complex mod q), rescale.  FP64-VALU bound: 4 exact modmuls per complex
    MAC, 512 * 11 * 64^3 complex MACs per call."""
    import numpy as np
    import torch
    import mfhe
    n, L, batch = 64, 11, 512
    ctx = mfhe.Context(mfhe.RNS_MODULI, 1, mfhe.CONV_PHANTOM)
    q = np.array(mfhe.RNS_MODULI, np.uint64)[None, :, None]
    rng = np.random.default_rng(5)
    planes = [mfhe.to_device_u64((rng.integers(0, 2 ** 63, (batch, L, n * n), dtype=np.uint64) % q).ravel())
              for _ in range(4)]
    bp = [torch.empty_like(planes[0]) for _ in range(2)]
    c = [torch.empty_like(planes[0]) for _ in range(2)]
    inv = [pow(2 ** 35, -1, int(m)) for m in mfhe.RNS_MODULI[:3]] + [0] * (L - 3)

    def gemm():
        ctx.trace_gemm(planes[0], planes[1], bp[0], bp[1], c[0], c[1], n, L, batch)

    def full():
        ctx.trace_map_bprime(planes[2], planes[3], bp[0], bp[1], n, L, batch)
        gemm()
        ctx.trace_rescale(c[0], c[1], n, L, batch, inv)
    _warm(full)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(9)]
    e[0].record()
    for _ in range(reps):
        gemm()
    e[1].record()
    for _ in range(reps):
        full()
    e[2].record()
    ctx.set_option(mfhe.OPT_TRACE_SPLIT, 0)
    gemm()
    e[3].record()
    for _ in range(reps):
        gemm()
    e[4].record()
    ctx.set_option(mfhe.OPT_TRACE_SPLIT, 1)
    gemm()
    e[5].record()
    for _ in range(reps):
        gemm()
    e[6].record()
    torch.cuda.synchronize()
    ctx.set_option(mfhe.OPT_TRACE_SPLIT, 2)
    x_ms = e[5].elapsed_time(e[6]) / reps

    def fused():
        ctx.trace_product(planes[0], planes[1], planes[2], planes[3], c[0], c[1], n, L, batch, inv)
    fused()
    e[7].record()
    for _ in range(reps):
        fused()
    e[8].record()
    torch.cuda.synchronize()
    p_ms = e[7].elapsed_time(e[8]) / reps
    g_ms, f_ms = e[0].elapsed_time(e[1]) / reps, e[1].elapsed_time(e[2]) / reps
    m_ms = e[3].elapsed_time(e[4]) / reps
    macs = batch * L * n ** 3
    ctx.close()
    return {"workload": "batched trace GEMM, 512 matrices x L=11 x n=64 complex mod q (reference geometry)",
            "gemm_ms": round(g_ms, 3), "map_gemm_rescale_ms": round(f_ms, 3),
            "fused_product_ms": round(p_ms, 3),
            "complex_modmac_per_s": round(macs / (g_ms * 1e-3)),
            "kernel": "split-digit product on v_mfma_f64_16x16x4 (16 MFMA per 16x16x4 complex block-step, exact)",
            "fp64_tflops": round(macs * 16 * 2 / (g_ms * 1e-3) / 1e12, 1), "fp64_peak_tflops": 78.6,
            "modmul_kernel_gemm_ms": round(m_ms, 3), "split_valu_kernel_gemm_ms": round(x_ms, 3)}


def profile_figures(N, L, batch, alg_bytes, world):
    """Roofline fields from the committed single-GPU profiles of the default command (rocprofv3 kernel trace via
    tools/prof_agree.py, FETCH_SIZE / WRITE_SIZE passes via tools/pmc_summary.py).  At N = 1 they are this
    command's own figures and go into `roofline` directly; at N > 1 they describe another run, so they are
    returned only under `profile_1gpu`, labelled (tests/test_bench_cli.py checks both forms)."""
    prof = {}
    tr = pmc_traffic(N, L, batch)
    if tr:
        prof["traffic"] = tr[0]
        prof["traffic_source"] = f"profiles/{tr[1]}"
        prof["traffic_over_algorithmic"] = round(tr[0] / alg_bytes, 3)
    tr = prof_trace(N, L, batch)
    if tr:
        # per-kernel averages of a committed rocprofv3 --kernel-trace run of this same command: the roofline
        # recomputed from the trace alone
        prof["kernel_ms_per_transform"] = round(tr["rocprof_kernel_ms_per_transform"], 4)
        prof["kernel_trace_frac"] = round(
            alg_bytes / (tr["rocprof_kernel_ms_per_transform"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        prof["kernel_trace_source"] = f"profiles/{tr['file']}"
        prof["kernel_trace_per_kernel_avg_us"] = {
            k.split("(")[0].split("<")[0].replace("void mfhe::", ""): round(v["avg_us"], 2)
            for k, v in tr["per_kernel"].items()}
    if world == 1 or not prof:
        return prof
    prof["note"] = ("from the committed single-GPU profiles of the N = 1 command, not measured in this "
                    f"{world}-rank run (per-GPU work is the same: weak scaling)")
    return {"profile_1gpu": prof}


def c4_line(world, rank, comm, barrier, reps=5):
    """BASELINE C4: encode -> encrypt_pair -> decrypt_and_decode with wide CRT at the reference geometry (n = 64,
    512 W-lanes), L = 16 moduli q = 1 mod 2^8 * 771, residues sharded across the ranks: rank g runs every
    per-limb stage (W-CRT, samplers, X-NTT ring products, W-INTT) on limbs [g*16/G, (g+1)*16/G) and the decode's
    wide CRT is the RCCL recombine (mfhe_decrypt_and_decode_sharded).  All ranks work on ONE batch (strong
    scaling inside this line).  Input and check: test_encode_encrypt_decrypt_decode_wcrt.cu:44-52,109."""
    import numpy as np
    import torch
    import mfhe
    L, G = 16, world
    if L % G or 512 % G:
        return {"skipped": f"world {G} does not divide 16 limbs / 512 lanes"}
    moduli = gen_moduli(35, 197376, L)
    lg = L // G
    ctx = mfhe.Context(moduli[rank * lg:(rank + 1) * lg], 6, mfhe.CONV_PHANTOM | mfhe.CONV_WCRT)
    ctx.set_limb_shard(rank * lg, L)
    ctx.reserve_workspace()
    c_all = mfhe.Context(moduli, 6, mfhe.CONV_PHANTOM)
    n2 = 4096
    msg = (np.arange(512)[:, None] * np.ones((1, n2)) + 0.001j).ravel()
    mt = torch.from_numpy(msg.view(np.float64).copy()).cuda()
    words = 512 * lg * n2
    re_, im_ = (torch.empty(words, dtype=torch.int64, device="cuda") for _ in range(2))
    cre, cim = (torch.empty(2 * words, dtype=torch.int64, device="cuda") for _ in range(2))
    sk = torch.empty(512 * lg * 64, dtype=torch.int64, device="cuda")
    res = torch.empty_like(mt)
    ctx.keygen(sk)
    out = {}
    for mode in ("allgather", "alltoall"):
        ctx.decrypt_and_decode_sharded(c_all, comm, mode, cre, cim, sk, res)   # grows the receive buffer

        def run():
            ctx.encode(mt, re_, im_)
            ctx.encrypt_pair(re_, im_, sk, cre, cim)
            ctx.decrypt_and_decode_sharded(c_all, comm, mode, cre, cim, sk, res)
        for _ in range(5):   # a fixed count on every rank (collectives inside)
            run()
        barrier()
        # HIP events on the stream every call of run() is ordered on (the RCCL exchange included), plus the
        # host wall clock around the same loop; max over ranks of both
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / reps
        barrier()
        t = torch.tensor([e0.elapsed_time(e1) / reps * 1e-3, wall], dtype=torch.float64, device="cuda")
        if world > 1:
            import torch.distributed as dist
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t[0].item()
        err = float(np.max(np.abs(res.cpu().numpy().view(np.complex128) - msg)))
        out[mode] = {"ms": round(dt * 1e3, 3), "wall_ms": round(t[1].item() * 1e3, 3),
                     "messages_per_s": round(512 * n2 / dt), "max_err": err, "check_1e-3": err < 1e-3}
    ctx.close()
    c_all.close()
    return {"workload": f"C4: encode->encrypt_pair->decrypt_and_decode, n=64 x 512 W-lanes, L=16 x 35-bit moduli, "
                        f"limbs sharded over {G} GPU(s) ({lg} per GPU), RCCL recombine in decode",
            "scaling": "strong (one batch for all ranks)",
            "exchange": ("1-rank communicator: the sharded code path with no data exchanged" if G == 1 else
                         f"RCCL across {G} ranks"), **out}


def c5_line(world, rank, barrier, timed, backend, reps=2, recv_gib=2.0):
    """BASELINE C5: N = 2^17, L = 32 x 50-bit primes (bootstrapping depth), batch 4096, residues sharded over
    the G ranks: rank g owns limbs [g*32/G, (g+1)*32/G) of every polynomial (16 GiB per GPU at G = 8, the
    whole 128 GiB at G = 1).  Strong scaling: the problem is fixed, G divides it.  One step =
      * forward + inverse NTT of the shard (no communication);
      * the CRT recombine of the whole batch: RCCL exchange + sharded wide-CRT compose -> f64/delta of this
        rank's polys, chunked over polys so the receive buffer stays <= recv_gib (mfhe.dist.chunk_plan).
    The shard holds the residues of real messages (|z| < 1, delta = 2^35), as a decode does.
    Curves: NTT alone, NTT + recombine by all-to-all (each rank receives only its polys' missing limbs,
    (G-1)/G^2 of the set), NTT + recombine by all-gather (every rank receives (G-1)/G of the set, 112 GiB at
    G = 8: run chunk by chunk, never as one buffer).  G = 1: the compose is local (no exchange)."""
    import torch
    import mfhe
    from mfhe import dist as mdist
    log_n, L, batch = 17, 32, 4096
    N = 1 << log_n
    if L % world or batch % world:
        return {"skipped": f"world {world} does not divide 32 limbs / 4096 polys"}
    if world > 1 and backend != "nccl":
        # decided before anything is allocated (the shard is 128/G GiB per rank)
        return {"skipped": f"world {world}: the C5 recombine needs the RCCL communicator (backend {backend})"}
    moduli = gen_moduli(50, 1 << (log_n + 2), L)
    s0, lg = mdist.limb_range(L, world, rank)
    ctx = mfhe.Context(moduli[s0:s0 + lg], log_n, mfhe.CONV_PHANTOM)   # this rank's limbs: NTT tables
    ctx_all = mfhe.Context(moduli, log_n, mfhe.CONV_PHANTOM)           # all 32: the CRT tables
    dev = torch.device("cuda", torch.cuda.current_device())
    stream = torch.cuda.current_stream()
    shard = torch.empty(batch * lg * N, dtype=torch.int64, device=dev)
    g = torch.Generator(device=dev).manual_seed(0x4D46484500000005)
    cpg = 256                                    # decompose in 256-poly pieces (same messages on every rank)
    z = torch.empty(cpg * N, dtype=torch.float64, device=dev)
    for p0 in range(0, batch, cpg):
        z.uniform_(-1.0, 1.0, generator=g)
        ctx.rns_decompose(z, shard[p0 * lg * N:(p0 + cpg) * lg * N], cpg, N, stream=stream)
    del z
    out = torch.empty(batch // world * N, dtype=torch.float64, device=dev)
    if world > 1:
        comm = mfhe.Comm.create()
        modes = ("alltoall", "allgather")
    else:
        # N = 1: the local compose, and the same native chunked call over a 1-rank communicator, which exchanges
        # nothing and composes straight from the shard (dist.cpp world-1 path): it must cost what the local compose does
        comm = mfhe.Comm.from_id(mfhe.Comm.unique_id(), 1, 0)
        modes = ("local", "alltoall")
    # chunk so one receive half holds <= recv_gib / 2 (two halves, exchange k + 1 beside compose k): all-to-all
    # receives cp/G polys x 32 limbs per chunk, all-gather cp x 32
    per_poly = L * N * 8
    half = recv_gib / 2 * 2 ** 30
    chunks = {"alltoall": int(half // per_poly) * world, "allgather": int(half // per_poly), "local": batch}
    for m in modes:
        if m != "local":
            ctx_all.crt_recombine_chunked_reserve(comm, m, chunks[m], N)

    def ntt():
        ctx.ntt_fwd(shard, batch=batch, stream=stream)
        ctx.ntt_inv(shard, batch=batch, stream=stream)

    def check(m):
        """Every output row against its regenerated message: |err| <= 2^-36 (llround to delta = 2^35, exact
        CRT).  Row r of this rank holds poly owned_polys(...)[r] (chunk order)."""
        own = torch.tensor(mdist.owned_polys(batch, world, rank, chunks[m]) if m != "local" else list(range(batch)),
                           dtype=torch.int64, device=dev)
        rows = torch.arange(own.numel(), device=dev)
        g.manual_seed(0x4D46484500000005)
        zz = torch.empty(cpg * N, dtype=torch.float64, device=dev)
        err = 0.0
        for p0 in range(0, batch, cpg):
            zz.uniform_(-1.0, 1.0, generator=g)
            sel = (own >= p0) & (own < p0 + cpg)
            r, p = rows[sel], own[sel] - p0
            if r.numel():
                err = max(err, float((out.view(-1, N)[r] - zz.view(-1, N)[p]).abs().nan_to_num(nan=float("inf")).max()))
        return err

    res = {}
    w, _ = timed(ntt, reps, 1)
    t_ntt = w / reps
    res["ntt_fwd_inv_ms"] = round(t_ntt * 1e3, 3)
    res["ntt_NTT_per_s"] = round(2 * batch * L / t_ntt)     # both directions, all ranks
    for m in modes:
        def step(m=m):
            ntt()
            if m == "local":
                ctx_all.crt_compose_f64(shard, out, batch, N, stream=stream)
            else:
                mdist.crt_recombine_chunked(ctx_all, shard, batch, N, m, chunks[m], out, stream=stream, comm=comm)
        out.fill_(float("nan"))
        w, _ = timed(step, reps, 1)
        t = w / reps
        recv = (world - 1) / world * batch * per_poly / (world if m == "alltoall" else 1)
        err = check(m)
        res[m] = {"ms": round(t * 1e3, 3), "recombine_ms": round((t - t_ntt) * 1e3, 3),
                  "polys_per_s": round(batch / t), "chunk_polys": min(batch, chunks[m]),
                  "recv_GiB_per_gpu": round(recv / 2 ** 30, 2),
                  "recv_GBps_per_gpu": round(recv / max(t - t_ntt, 1e-9) / 1e9, 1),
                  "max_err_all_rows": err, "check_2^-36": err <= 2.0 ** -36}
        if m != "local":
            res[m]["path"] = ("mfhe_crt_recombine_chunked: RCCL exchange of chunk k+1 on the communicator's stream "
                              "beside the compose of chunk k, two receive halves" if world > 1 else
                              "mfhe_crt_recombine_chunked on a 1-rank communicator: no exchange, one compose from the shard")
            # the recombine call alone, then the same call with the composes skipped (MFHE_RECOMBINE_EXCHANGE_ONLY) and
            # with the exchanges skipped (MFHE_RECOMBINE_COMPOSE_ONLY: the composes out of the halves the last call
            # filled, real values).  overlap_frac = 1 - (recombine - max(x, c)) / min(x, c): 1 when the shorter of
            # exchange and compose hides entirely under the longer, 0 when they run back to back
            def rec(fl=0, m=m, o=None):
                ctx_all.crt_recombine_chunked(comm, m, shard, batch, N, chunks[m], o, stream=stream, flags=fl)
            w_r, _ = timed(lambda: rec(o=out), reps, 1)
            w_x, _ = timed(lambda: rec(mfhe.RECOMBINE_EXCHANGE_ONLY), reps, 1)
            w_c, _ = timed(lambda: rec(mfhe.RECOMBINE_COMPOSE_ONLY, o=out), reps, 1)
            r_ms, x_ms, c_ms = (w / reps * 1e3 for w in (w_r, w_x, w_c))
            res[m]["recombine_only_ms"] = round(r_ms, 3)
            res[m]["exchange_only_ms"] = round(x_ms, 3)
            res[m]["compose_only_ms"] = round(c_ms, 3)
            lo, hi = min(x_ms, c_ms), max(x_ms, c_ms)
            res[m]["overlap_frac"] = round(1.0 - (r_ms - hi) / lo, 3) if lo > 0.01 * hi else None
            if res[m]["overlap_frac"] is None:
                res[m]["overlap_note"] = "no exchange to overlap (world 1)" if world == 1 else "exchange or compose ~0"
    if comm is not None:
        comm.close()
    ctx.close()
    ctx_all.close()
    return {"workload": f"C5: N=2^17, L=32 x 50-bit primes, batch 4096, limbs sharded over {world} GPU(s) "
                        f"({lg} per GPU): fwd+inv NTT of the shard, then chunked RCCL recombine + wide-CRT "
                        f"compose -> f64 of this rank's 4096/{world} polys",
            "scaling": "strong (one problem for all ranks)", **res}


def cpu_quota():
    """CPUs this process may use per the cgroup CPU quota (cpu.max / cfs_quota_us), or None if unlimited."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, int(q) // int(p))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, q // p)
    except (OSError, ValueError):
        pass
    return None


def cpu_baseline(log_n, moduli, seconds):
    """The reference's CPU path restated (oracle/, test infrastructure; the reference itself has no runnable
    CPU path), timed on this box's host cores on bounded samples of each workload:
      * phantom forward NTT (Harvey/Shoup, fnwt_1d semantics) at the headline shape, all cores and 1 core;
      * encode+CRT ops (RNS decompose batched_encoder.cu:125-152 + wide CRT compose encoder.cu:191-230 +
        big -> f64 HE.cu:1007-1027) on the same shape, all cores and 1 core;
      * the reference's own GL NTT (ntt_core.cu:462-481) at its geometry (n = 64, L = 11, 512 x 64 polys);
      * the C1 (N = 2^12, L = 1, single poly) and C2 (N = 2^14, L = 4, batch 256) forward NTT.

    Cores.  `cores` = the OpenMP threads of the all-core figures, set explicitly: the CPUs this process may
    use, i.e. min(affinity mask, cgroup quota, the harness's per-GPU CPU share).  On the GPU box nproc and the
    affinity mask count the whole host (256) while one GPU's job is given a 16-CPU share (OMP_NUM_THREADS=16
    there, and its worker-pool rule): 256 threads on 16 CPUs would time the scheduler, not the oracle.  All
    three numbers are printed with the reason."""
    import numpy as np
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle
    aff = len(os.sched_getaffinity(0))
    quota = cpu_quota()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    threads = min(x for x in (aff, quota, share) if x)
    reason = ("affinity mask" if threads == aff else "cgroup CPU quota" if threads == quota
              else "per-GPU CPU share (OMP_NUM_THREADS set by the harness; affinity counts the whole host)")
    oracle.L.orc_set_threads(threads)
    N, L = 1 << log_n, len(moduli)
    per = max(0.5, seconds / 8)          # seconds per measured figure
    rng = np.random.default_rng(0)

    def rate(fn, units):
        fn()                               # warm (tables, thread pool)
        done, dt = 0, 0.0
        while dt < per:
            t0 = time.perf_counter()
            fn()
            dt += time.perf_counter() - t0
            done += units
        return done / dt

    def residues(b, L_, n, mods):
        q = np.array(mods, np.uint64)[None, :, None]
        return (rng.integers(0, 2 ** 63, (b, L_, n), dtype=np.uint64) % q).ravel()

    m64 = np.array(moduli, np.uint64)
    b = 64
    x = residues(b, L, N, moduli)
    ntt_all = rate(lambda: oracle.L.orc_phantom_fwd(oracle.P(x), b, L, log_n, oracle.P(m64)), b * L)
    x1 = x[: 2 * L * N].copy()
    ntt_1 = rate(lambda: oracle.L.orc_phantom_fwd_1t(oracle.P(x1), 2, L, log_n, oracle.P(m64)), 2 * L)

    # encode+CRT: one op = one real poly of N coefficients decomposed to L residues and composed back to f64
    W = oracle.crt_words(moduli)
    delta = 2.0 ** 35

    def enc_crt(npoly, one):
        z = rng.random(npoly * N) * 2 - 1
        r = np.zeros(npoly * L * N, np.uint64)
        mag = np.zeros(npoly * N * W, np.uint64)
        neg = np.zeros(npoly * N, np.uint8)
        out = np.zeros(npoly * N, np.float64)
        dec = oracle.L.orc_rns_decompose_1t if one else oracle.L.orc_rns_decompose
        com = oracle.L.orc_crt_compose_1t if one else oracle.L.orc_crt_compose

        def f():
            dec(oracle.P(z), 1, npoly, N, L, oracle.P(m64), delta, oracle.P(r))
            com(oracle.P(r), npoly, L, N, oracle.P(m64), W, oracle.P(mag), oracle.P(neg))
            oracle.L.orc_big_to_f64(oracle.P(mag), oracle.P(neg), npoly * N, W, delta, oracle.P(out), 1)
        return rate(f, npoly)
    crt_all, crt_1 = enc_crt(64, False), enc_crt(2, True)

    # reference GL NTT at the reference geometry: n = 64, the 11 reference moduli, 512 x 64 polys
    import mfhe
    rm = mfhe.RNS_MODULI
    g = residues(512 * 64, 11, 64, rm)
    gl = rate(lambda: oracle.gl_fwd(g, 11, 64, rm), 512 * 64 * 11)
    # C1 / C2 shapes
    m12 = oracle.gen_primes(50, 1 << 14, 1)
    c1 = residues(1, 1, 1 << 12, m12)
    c1r = rate(lambda: oracle.phantom_fwd(c1, 1, 12, m12), 1)
    m14 = oracle.gen_primes(50, 1 << 16, 4)
    c2 = residues(256, 4, 1 << 14, m14)
    c2r = rate(lambda: oracle.phantom_fwd(c2, 4, 14, m14), 256 * 4)
    return {"value": ntt_all, "unit": "NTT/s", "cores": threads, "kind": "port",
            "nproc": os.cpu_count(), "affinity_cores": aff, "cgroup_quota_cores": quota,
            "omp_num_threads_env": share, "cores_reason": reason,
            "sample": f"forward NTT N=2^{log_n} x L={L} (oracle phantom Harvey NTT, OpenMP {threads} threads), "
                      f"~{per:.1f} s per figure; the headline workload is 1024 polys x {L} limbs, sampled at "
                      f"{b} polys ({b * L} NTTs) per call",
            "one_core_NTT_per_s": ntt_1,
            "encode_crt_ops_per_s": {"all_cores": crt_all, "one_core": crt_1,
                                     "op": f"decompose + wide CRT compose + f64 of one N=2^{log_n} poly, L={L}, W={W}"},
            "gl_ntt_reference_geometry_NTT_per_s": gl,
            "C1_fwd_NTT_per_s": c1r, "C2_fwd_NTT_per_s": c2r}


def u64_line(reps=20, warm=3):
    """C3 forward and inverse NTT on the 64-bit integer path: 60-bit primes, which the FP64 path cannot take
    (q < 2^50), and the headline's 50-bit primes forced onto U64 for comparison.  Every q < 2^60 here, so both
    directions run the lazy U60 schedules (ArithU60); the Harvey schedule (ArithU64, OPT_NTT_U60 0) beside them."""
    import torch
    import mfhe
    log_n, L, batch = 16, 8, 1024
    N = 1 << log_n
    res = {}
    for name, bits, arith in (("60-bit primes (auto -> u64)", 60, 0), ("50-bit primes, u64 forced", 50, mfhe.ARITH_U64)):
        moduli = gen_moduli(bits, 1 << (log_n + 2), L)
        ctx = mfhe.Context(moduli, log_n, mfhe.CONV_PHANTOM)
        if arith:
            ctx.set_arith(arith)
        d = torch.empty(batch * L * N, dtype=torch.int64, device="cuda")
        qt = torch.tensor(moduli, dtype=torch.int64, device="cuda").repeat_interleave(N).repeat(batch)
        d.random_(0, 2 ** 62).remainder_(qt)
        del qt
        out = {}

        def rate(fn):
            for _ in range(warm):
                fn(d, batch=batch)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn(d, batch=batch)
            e1.record()
            torch.cuda.synchronize()
            return batch * L / (e0.elapsed_time(e1) / reps * 1e-3)
        for kind, fn in (("fwd", ctx.ntt_fwd), ("inv", ctx.ntt_inv)):
            r = rate(fn)
            out[f"{kind}_NTT_per_s"] = round(r)
            out[f"{kind}_alg_GBps"] = round(16.0 * N * r / 1e9, 1)
        out["frac_fwd"] = round(out["fwd_alg_GBps"] / HBM_PEAK_GBS, 4)
        out["arith"] = "u64" if ctx.info().arith == mfhe.ARITH_U64 else "f64"
        if out["arith"] == "u64":   # schedule of both directions: lazy U60 (every q < 2^60) or Harvey
            out["schedule"] = "u60" if ctx.get_option(mfhe.OPT_NTT_U60) else "harvey"
            if out["schedule"] == "u60":   # the same box's Harvey schedule, for the A/B (MFHE_OPT_NTT_U60 0)
                ctx.set_option(mfhe.OPT_NTT_U60, 0)
                out["harvey_fwd_NTT_per_s"] = round(rate(ctx.ntt_fwd))
                out["harvey_inv_NTT_per_s"] = round(rate(ctx.ntt_inv))
                ctx.set_option(mfhe.OPT_NTT_U60, 1)
        out["max_modulus_bits"] = max(moduli).bit_length()
        res[name] = out
        del d
        ctx.close()
    return res


WATCHDOG_EXIT = 3   # exit status of a run whose secondary lines the watchdog stopped (the headline is printed)


def start_watchdog(out: dict, rank: int, seconds: float):
    """After `seconds`, rank 0 prints `out` (the finished headline plus whatever secondary lines completed) with a
    note, and every rank exits WATCHDOG_EXIT without waiting for the GPU work or collectives in flight: a hang in a
    multi-rank line fails the run visibly (non-zero status, passed through by launch_ranks) while the headline
    measured before it is still on stdout."""
    import threading

    def bail():
        if rank == 0:
            out["secondary_lines"] = (f"stopped by the {seconds:.0f} s watchdog (exit status {WATCHDOG_EXIT}); "
                                      f"lines finished before it are included")
            print(json.dumps(out), flush=True)
        sys.stderr.write(f"bench.py rank {rank}: secondary lines exceeded {seconds} s, exiting {WATCHDOG_EXIT}\n")
        sys.stderr.flush()
        os._exit(WATCHDOG_EXIT)
    wd = threading.Timer(seconds, bail)
    wd.daemon = True
    wd.start()
    return wd


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` with no launcher around it: start N rank processes (torch.distributed.run, one per
    GPU, rendezvous on 127.0.0.1) and wait for them.  This parent never touches the GPU (it does not even import
    torch): it forwards the ranks' output line by line to stderr and re-prints rank 0's one JSON line on stdout,
    then exits with the ranks' exit status (non-zero also when no JSON line came back)."""
    import subprocess
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(Path(__file__).resolve()), *sys.argv[1:]]
    print(f"bench.py: --gpus {n} without WORLD_SIZE -> launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    env = dict(os.environ, MFHE_BENCH_LAUNCHED="1")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    line = None
    for ln in p.stdout:
        s = ln.strip()
        if s.startswith("{") and '"metric"' in s:
            try:
                json.loads(s)
                line = s
                continue
            except ValueError:
                pass
        sys.stderr.write(ln)
        sys.stderr.flush()
    rc = p.wait()
    if line is not None:
        print(line, flush=True)
        # torch.distributed.run reports any failed rank as 1: restore the watchdog's own status
        if rc != 0 and "watchdog" in str(json.loads(line).get("secondary_lines", "")):
            return WATCHDOG_EXIT
    if rc == 0 and line is None:
        print("bench.py: the ranks exited 0 but printed no JSON line", file=sys.stderr)
        return 1
    return rc


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={env_world} from the launcher but --gpus {args.gpus}: they must agree "
                 f"(n_gpus is reported from the ranks that actually run)")
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    import torch
    import torch.distributed as dist

    if args.launch_check:
        # CPU rehearsal of the launcher (tests/test_bench_cli.py): the ranks meet over gloo, no GPU
        w = int(os.environ.get("WORLD_SIZE", "1"))
        if w > 1:
            dist.init_process_group("gloo")
        t = torch.ones(1)
        if w > 1:
            dist.all_reduce(t)
        out = {"metric": "launch-check", "n_gpus": w, "value": t.item(),
               "launched_by_bench": os.environ.get("MFHE_BENCH_LAUNCHED") == "1"}
        wd = start_watchdog(out, int(os.environ.get("RANK", "0")), args.secondary_timeout)
        if args.hang_check:
            time.sleep(args.hang_check)   # a secondary line that never returns (tests/test_bench_cli.py)
        wd.cancel()
        if int(os.environ.get("RANK", "0")) == 0:
            print(json.dumps(out), flush=True)
        if w > 1:
            dist.destroy_process_group()
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (never set by the driver): MFHE_BENCH_BACKEND=gloo + MFHE_BENCH_SAME_DEVICE=1 run the
    # N > 1 code path with every rank on cuda:0 of a one-GPU box (RCCL refuses two ranks on one GPU)
    backend = os.environ.get("MFHE_BENCH_BACKEND", "nccl")
    if os.environ.get("MFHE_BENCH_SAME_DEVICE") == "1":
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import mfhe

    log_n, L, batch = args.log_n, args.limbs, args.batch
    N = 1 << log_n
    moduli = gen_moduli(50, 1 << (log_n + 2), L)
    ctx = mfhe.Context(moduli, log_n, mfhe.CONV_PHANTOM)
    if args.arith:
        ctx.set_arith(args.arith)
    for opt, val in ((4, args.ntt_wg), (5, args.ntt_prefetch), (mfhe.OPT_NTT_CHUNK_BYTES, args.ntt_chunk),
                     (mfhe.OPT_NTT_PACK, args.ntt_pack), (mfhe.OPT_NTT_PLAN, args.ntt_plan)):
        if val is not None:
            ctx.set_option(opt, val)
    stream = torch.cuda.current_stream()

    # synthetic residues uniform in [0, q_l), generated on device
    g = torch.Generator(device=dev).manual_seed(0x4D46484500000000 % (2 ** 63) + 3 + rank)
    data = torch.empty(batch * L * N, dtype=torch.int64, device=dev)
    qt = torch.tensor(moduli, dtype=torch.int64, device=dev).repeat_interleave(N).repeat(batch)
    data.random_(0, 2 ** 62, generator=g)
    data.remainder_(qt)
    del qt

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def timed(fn, steps, warmup):
        for _ in range(warmup):
            fn()
        barrier()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        for _ in range(steps):
            fn()
        ev1.record(stream)
        barrier()
        wall = time.perf_counter() - t0
        ev_ms = ev0.elapsed_time(ev1)
        t = torch.tensor([wall], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.item(), ev_ms / steps

    res = {}
    if args.only in ("all", "ntt"):
        wall, ev_ms = timed(lambda: ctx.ntt_fwd(data, batch=batch, stream=stream), args.steps, args.warmup)
        res["fwd_wall"], res["fwd_ev_ms"] = wall, ev_ms
        # the inverse with exactly the forward's steps and warm-up (the first ~30 ms of calls run in the clock
        # ramp, profiles/r02_bench_steps.txt, so fewer steps would understate it)
        wall_i, ev_i = timed(lambda: ctx.ntt_inv(data, batch=batch, stream=stream), args.steps, args.warmup)
        res["inv_ev_ms"], res["inv_wall"] = ev_i, wall_i
    if args.only in ("all", "crt"):
        # encode+CRT op = one real poly of N coefficients: decompose (f64 -> L residues) + compose (-> f64/delta)
        cb = max(1, batch // 4)
        z = torch.rand(cb * N, dtype=torch.float64, device=dev, generator=g) * 2 - 1
        r = data[: cb * L * N]
        zo = torch.empty_like(z)

        def enc_crt():
            ctx.rns_decompose(z, r, cb, N, stream=stream)
            ctx.crt_compose_f64(r, zo, cb, N, stream=stream)

        # ~0.5 ms per call: 100 warm-up calls (a fixed count, the same on every rank) keep the clock ramp of the first
        # ~30 ms of work out of the timed calls (profiles/r02_bench_steps.txt)
        wall_c, ev_c = timed(enc_crt, max(1, args.steps), 100)
        res["crt_ev_ms"], res["crt_batch"] = ev_c, cb

    out = {}
    if rank == 0:
        ntts = batch * L * world
        out.update({
            "metric": "forward-NTT/s (N=2^16, L RNS limbs)",
            "unit": "NTT/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic uniform residues in [0, q_l), device-resident",
            "config": {"workload": f"batched forward negacyclic NTT (phantom convention), N=2^{log_n}, "
                                   f"L={L} x 50-bit primes, batch={batch} per GPU",
                       "N": N, "limbs": L, "batch_per_gpu": batch,
                       "arith": "f64" if ctx.info().arith == mfhe.ARITH_F64 else "u64",
                       "parallelism": f"residue-batch shard x{world} (no collective)"},
        })
        if "fwd_wall" in res:
            step_s = res["fwd_wall"] / args.steps
            out["value"] = ntts / step_s
            out["ms_per_step"] = step_s * 1e3
            alg_bytes = 16.0 * N * batch * L       # 8N read + 8N write per NTT
            ach = alg_bytes / (res["fwd_ev_ms"] * 1e-3) / 1e9
            chunk_polys = max(1, ctx.get_option(mfhe.OPT_NTT_CHUNK_BYTES) // (L * N * 8))
            nchunks = -(-batch // chunk_polys) if log_n >= 14 else 1
            kname = (f"mfhe_ntt_fwd call = {nchunks} chunks x (column pass ntt_col_db_kernel + block pass "
                     f"ntt_pass_kernel) launches" if log_n >= 14 else
                     "mfhe_ntt_fwd call = 1 single-pass ntt_pass_kernel launch")
            out["roofline"] = {"bound": "hbm", "kernel": kname,
                               "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                               "traffic_unit": "bytes per transform (FETCH_SIZE x2 + WRITE_SIZE, L2<->fabric)",
                               "algorithmic_bytes_per_launch": alg_bytes,
                               "hbm_read_frac": round(ach / 2 / HBM_PEAK_GBS, 4),
                               "event_ms_per_transform": round(res["fwd_ev_ms"], 4)}
            out["roofline"].update(profile_figures(N, L, batch, alg_bytes, world))
            out["inverse_NTT_per_s"] = ntts / (res["inv_wall"] / args.steps)
            out["inverse_over_forward"] = round(out["inverse_NTT_per_s"] / out["value"], 4)
        if "crt_ev_ms" in res:
            cb = res["crt_batch"]
            out["encode_crt_ops_per_s"] = cb / (res["crt_ev_ms"] * 1e-3) * world
            out["encode_crt_GBps"] = 16.0 * (L + 1) * N * cb / (res["crt_ev_ms"] * 1e-3) / 1e9

    # The headline is measured and complete.  The secondary lines below run collectives that have never executed
    # on more than one real GPU (RCCL communicators of libmfhe beside torch's): a watchdog on every rank bounds
    # them, so a hang there still leaves the headline line printed (rank 0); the stopped run then exits with
    # WATCHDOG_EXIT (3), so the driver sees that the secondary lines did not finish.
    wd = start_watchdog(out, rank, args.secondary_timeout)

    if args.only in ("all", "recombine") and args.recombine_batch and L % world == 0:
        try:
            # residue sharding: rank g owns limbs [g*L/G, (g+1)*L/G) of every poly.  One step =
            # forward + inverse NTT of the shard (a computation round trip) + RCCL exchange + sharded CRT
            # compose of this rank's batch slice -> f64.  The shard holds RNS residues of real messages
            # (|z| < 1 scaled by delta), as a decode does.
            from mfhe import dist as mdist
            rb = max(world, args.recombine_batch // world * world)
            s0, lg = mdist.limb_range(L, world, rank)
            full = torch.empty(rb * L * N, dtype=torch.int64, device=dev)
            zr = torch.rand(rb * N, dtype=torch.float64, device=dev, generator=g) * 2 - 1
            ctx.rns_decompose(zr, full, rb, N, stream=stream)
            shard = full.view(rb, L, N)[:, s0:s0 + lg, :].contiguous().view(-1)
            del full, zr
            rout = torch.empty(rb // world * N, dtype=torch.float64, device=dev)
            # multi-GPU: the recombine is the native RCCL call (mfhe_crt_recombine_sharded) on a communicator
            # owned by libmfhe, receive buffers reserved here, outside the timed steps
            comm = None
            if world > 1 and backend == "nccl":
                comm = mfhe.Comm.create()
                for mode in ("allgather", "alltoall"):
                    ctx.crt_recombine_reserve(comm, mode, rb, N)
            rc = {}
            nrep = max(1, args.steps // 4)
            modes = ("allgather", "alltoall") if world > 1 else ("local",)
            for mode in modes:
                def step(mode=mode):
                    ctx.ntt_fwd(shard, batch=rb, start_limb=s0, nlimbs=lg, stream=stream)
                    ctx.ntt_inv(shard, batch=rb, start_limb=s0, nlimbs=lg, stream=stream)
                    if mode == "local":
                        ctx.crt_compose_f64(shard, rout, rb, N, stream=stream)
                    else:
                        mdist.crt_recombine(ctx, shard, rb, N, mode, out=rout, stream=stream, comm=comm)
                w_r, _ = timed(step, nrep, 1)
                rc[mode] = w_r / nrep

            def ntt_rt():
                ctx.ntt_fwd(shard, batch=rb, start_limb=s0, nlimbs=lg, stream=stream)
                ctx.ntt_inv(shard, batch=rb, start_limb=s0, nlimbs=lg, stream=stream)
            w_n, _ = timed(ntt_rt, nrep, 1)
            if comm is not None:
                comm.close()
            res["recombine"] = {"batch": rb, "limbs_per_gpu": lg, "ntt_roundtrip_only_ms": w_n / nrep * 1e3,
                                "exchange": ("none (1 GPU: local compose)" if world == 1 else "native RCCL (mfhe_crt_recombine_sharded)")
                                            if comm is not None or world == 1
                                            else "torch.distributed " + backend,
                                **{f"{m}_ms": t * 1e3 for m, t in rc.items()},
                                **{f"{m}_polys_per_s": rb / t for m, t in rc.items()}}
        except Exception as e:   # a secondary line must not cost the headline line
            traceback.print_exc()
            res["recombine"] = {"error": repr(e)[:300]}
        out["residue_shard_ntt_roundtrip_crt_recombine"] = res["recombine"]

    c4 = None
    if args.only in ("all", "c4") and not args.no_pipeline:
        if world > 1 and backend == "nccl":
            c4comm = mfhe.Comm.create()
        else:
            c4comm = mfhe.Comm.from_id(mfhe.Comm.unique_id(), 1, 0) if world == 1 else None
        if c4comm is None:
            c4 = {"skipped": f"world {world}: the C4 decode recombine needs the RCCL communicator (backend {backend})"}
        else:
            try:
                c4 = c4_line(world, rank, c4comm, barrier)
            except Exception as e:   # a secondary line must not cost the headline line
                traceback.print_exc()
                c4 = {"error": repr(e)[:300]}
            c4comm.close()
        out["c4_sharded_pipeline"] = c4

    c5 = None
    if args.only in ("all", "c5") and not args.no_c5:
        try:
            c5 = c5_line(world, rank, barrier, timed, backend)
        except Exception as e:   # a secondary line must not cost the headline line
            traceback.print_exc()
            c5 = {"error": repr(e)[:300]}
        torch.cuda.empty_cache()
        out["c5_residue_shard"] = c5

    if rank == 0:
        if world == 1 and not args.no_pipeline and args.only == "all":
            out["reference_geometry_pipeline"] = pipeline_line()
            out["other_ntt_configs"] = other_configs_line()
            out["trace_gemm_reference_geometry"] = trace_line()
            out["u64_path_c3_forward_ntt"] = u64_line()
        if world == 1 and args.only == "u64":
            out["u64_path_c3_forward_ntt"] = u64_line()
        if world == 1 and not args.no_cpu_baseline and args.only == "all":
            try:
                out["cpu_baseline"] = cpu_baseline(log_n, moduli, args.cpu_seconds)
            except Exception as e:  # reported, never fatal
                out["cpu_baseline"] = {"error": str(e)}
        wd.cancel()
        print(json.dumps(out), flush=True)
    wd.cancel()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
