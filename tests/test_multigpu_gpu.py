"""G-process, G-GPU runs (G = 2, 4, 8; each skipped with fewer visible GPUs) of the native RCCL residue-shard paths.

Rank g runs on cuda:g with an RCCL communicator owned by libmfhe (mfhe_comm_*), holds limbs [g*L/2, (g+1)*L/2)
and calls the sharded entry points for real:
  * mfhe_decrypt_and_decode_sharded in both exchange modes (BASELINE C4 flow at L = 16) must equal the unsharded
    mfhe_decrypt_and_decode of the same ciphertext bit for bit (the rank computes the unsharded result itself);
  * mfhe_crt_recombine_sharded must equal the unsharded mfhe_crt_compose_f64 of its poly slice;
  * mfhe_crt_recombine_chunked (both modes, ragged last chunk, rows compact / global, repeated calls, an injected
    local failure on one rank with and without the status agreement) must equal it too;
  * a rank with bad arguments must fail on EVERY rank (the verdict exchange), not leave its peers in a collective.
The one-GPU box of the round-end tests skips this; the 1-rank communicator tests in test_c4_gpu.py /
test_dist_gpu.py run the same code paths there.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ngpus():
    try:
        import torch
        return torch.cuda.device_count()   # does not initialise the GPU
    except Exception:
        return 0


def _rank(rank, world, uidq, resq):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root / "matrix-fhe-gpu_amd"), str(root / "tests")]
    try:
        import torch
        torch.cuda.set_device(rank)
        import mfhe
        import oracle as O
        if rank == 0:
            uid = mfhe.Comm.unique_id()
            for _ in range(world - 1):
                uidq.put(uid)
        else:
            uid = uidq.get(timeout=60)
        comm = mfhe.Comm.from_id(uid, world, rank)
        ok = {}
        # ---- C4 decrypt + decode, L = 16, n = 64 (reference geometry) ----
        L, nlog, phi = 16, 6, 512
        moduli = O.gen_primes(35, 197376, L)
        n2 = 1 << (2 * nlog)
        full = mfhe.Context(moduli, nlog, mfhe.CONV_PHANTOM | mfhe.CONV_WCRT)
        msg = (np.arange(phi)[:, None] * np.ones((1, n2)) + 0.001j).ravel()
        mt = torch.from_numpy(msg.view(np.float64).copy()).cuda()
        words = phi * L * n2
        re_, im_ = (torch.empty(words, dtype=torch.int64, device="cuda") for _ in range(2))
        full.encode(mt, re_, im_)
        sk = torch.empty(phi * L * (1 << nlog), dtype=torch.int64, device="cuda")
        full.keygen(sk)
        cre, cim = (torch.empty(2 * words, dtype=torch.int64, device="cuda") for _ in range(2))
        full.encrypt_pair(re_, im_, sk, cre, cim)
        want = torch.empty_like(mt)
        full.decrypt_and_decode(cre, cim, sk, want)
        lg = L // world
        lo, hi = rank * lg, (rank + 1) * lg

        def limbs(t, inner):
            return t.view(-1, L, inner)[:, lo:hi, :].reshape(-1).contiguous()

        wl = phi * L * n2
        my_cre = torch.cat([limbs(cre[:wl], n2), limbs(cre[wl:], n2)])
        my_cim = torch.cat([limbs(cim[:wl], n2), limbs(cim[wl:], n2)])
        my_sk = limbs(sk, 1 << nlog)
        shard = mfhe.Context(moduli[lo:hi], nlog, mfhe.CONV_PHANTOM | mfhe.CONV_WCRT)
        shard.set_limb_shard(lo, L)
        c_all = mfhe.Context(moduli, nlog, mfhe.CONV_PHANTOM)
        for mode in ("allgather", "alltoall"):
            got = torch.empty_like(mt)
            shard.decrypt_and_decode_sharded(c_all, comm, mode, my_cre, my_cim, my_sk, got)
            torch.cuda.synchronize()
            ok[f"c4_{mode}"] = bool(torch.equal(got, want))
        # ---- raw recombine: 8 x 50-bit limbs, 2 G polys of 4096 ----
        m8 = O.gen_primes(50, 1 << 18, 8)
        ctx8 = mfhe.Context(m8, 16)
        rng = np.random.default_rng(3)
        npr = 2 * world
        v = rng.integers(-(1 << 40), 1 << 40, (npr, 4096), dtype=np.int64)
        res = np.stack([(v.astype(object) % int(m)).astype(np.uint64) for m in m8], axis=1)
        d = mfhe.to_device_u64(res.ravel())
        ref = torch.empty(npr * 4096, dtype=torch.float64, device="cuda")
        ctx8.crt_compose_f64(d, ref, npr, 4096)
        s0, lg8 = rank * (8 // world), 8 // world
        my = mfhe.to_device_u64(res[:, s0:s0 + lg8, :].ravel())
        bs = npr // world
        for mode in ("allgather", "alltoall"):
            out = torch.empty(bs * 4096, dtype=torch.float64, device="cuda")
            ctx8.crt_recombine_sharded(comm, mode, my, npr, 4096, out)
            torch.cuda.synchronize()
            ok[f"recombine_{mode}"] = bool(torch.equal(out, ref[rank * bs * 4096:(rank + 1) * bs * 4096]))
        # ---- chunked, pipelined recombine (mfhe_crt_recombine_chunked, the C5 / sharded-decode path; VERDICT r04
        # #3): both modes, 7 G polys in chunks of 2 G (3 full chunks + a ragged one of G), rows compact and global,
        # every call twice on the same communicator (the second call's exchanges wait on the first call's composes
        # of the same receive halves) -- bit-exact against the unsharded compose ----
        from mfhe import dist as mdist
        npc, cpc = 7 * world, 2 * world
        v2 = rng.integers(-(1 << 40), 1 << 40, (npc, 4096), dtype=np.int64)
        res2 = np.stack([(v2.astype(object) % int(m)).astype(np.uint64) for m in m8], axis=1)
        ref2 = torch.empty(npc * 4096, dtype=torch.float64, device="cuda")
        ctx8.crt_compose_f64(mfhe.to_device_u64(res2.ravel()), ref2, npc, 4096)
        ref2 = ref2.view(npc, 4096)
        my2 = mfhe.to_device_u64(res2[:, s0:s0 + lg8, :].ravel())
        own = torch.tensor(mdist.owned_polys(npc, world, rank, cpc), dtype=torch.int64, device="cuda")
        for mode in ("allgather", "alltoall"):
            ctx8.crt_recombine_chunked_reserve(comm, mode, cpc, 4096)
            for rows_global in (False, True):
                good = True
                for _ in range(2):
                    out = torch.full((npc if rows_global else npc // world, 4096), float("nan"),
                                     dtype=torch.float64, device="cuda")
                    ctx8.crt_recombine_chunked(comm, mode, my2, npc, 4096, cpc, out.view(-1), rows_global=rows_global)
                    torch.cuda.synchronize()
                    got = out[own] if rows_global else out
                    good &= bool(torch.equal(got, ref2[own]))
                    if rows_global:   # other ranks' rows untouched
                        mask = torch.ones(npc, dtype=torch.bool, device="cuda")
                        mask[own] = False
                        good &= bool(torch.isnan(out[mask]).all())
                ok[f"chunked_{mode}_{'global' if rows_global else 'compact'}"] = good
            # a local failure on the last rank only (its compose of chunk 1): it gets the error, every rank leaves
            # the call (no peer left in a collective), and the next call is bit-exact on every rank
            out = torch.empty(npc // world, 4096, dtype=torch.float64, device="cuda")
            fl = mfhe.RECOMBINE_DEBUG_FAIL if rank == world - 1 else 0
            try:
                ctx8.crt_recombine_chunked(comm, mode, my2, npc, 4096, cpc, out.view(-1), flags=fl)
                raised = False
            except mfhe.MfheError:
                raised = True
            torch.cuda.synchronize()
            ok[f"chunked_{mode}_injected_fail_local"] = raised == (rank == world - 1)
            # the same with MFHE_RECOMBINE_AGREE on every rank: every rank gets the error
            try:
                ctx8.crt_recombine_chunked(comm, mode, my2, npc, 4096, cpc, out.view(-1),
                                           flags=fl | mfhe.RECOMBINE_AGREE)
                raised = False
            except mfhe.MfheError:
                raised = True
            ok[f"chunked_{mode}_injected_fail_agreed"] = raised
            out.fill_(float("nan"))
            ctx8.crt_recombine_chunked(comm, mode, my2, npc, 4096, cpc, out.view(-1))
            torch.cuda.synchronize()
            ok[f"chunked_{mode}_after_failure"] = bool(torch.equal(out, ref2[own]))
        # ---- rank 1 passes a ctx_all with another scale: every rank must get an error, none may hang ----
        bad = mfhe.Context(moduli, nlog, mfhe.CONV_PHANTOM, delta=2.0 ** 30) if rank == 1 else c_all
        try:
            shard.decrypt_and_decode_sharded(bad, comm, "allgather", my_cre, my_cim, my_sk, torch.empty_like(mt))
            ok["bad_args_fail_everywhere"] = False
        except mfhe.MfheError:
            ok["bad_args_fail_everywhere"] = True
        comm.close()
        resq.put((rank, ok))
    except Exception as e:   # reported, so the parent never waits forever
        resq.put((rank, {"exception": repr(e)}))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_rccl_sharded_paths_equal_unsharded(world):
    if _ngpus() < world:
        pytest.skip(f"needs {world} visible GPUs (the round-end box has one)")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    uidq, resq = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, uidq, resq)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(resq.get(timeout=600) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert res[r] and all(res[r].values()), res
