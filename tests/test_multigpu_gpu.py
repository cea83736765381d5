"""Two-process, two-GPU run of the native RCCL residue-shard paths (skipped with fewer than 2 visible GPUs).

Rank g runs on cuda:g with an RCCL communicator owned by libmfhe (mfhe_comm_*), holds limbs [g*L/2, (g+1)*L/2)
and calls the sharded entry points for real:
  * mfhe_decrypt_and_decode_sharded in both exchange modes (BASELINE C4 flow at L = 16) must equal the unsharded
    mfhe_decrypt_and_decode of the same ciphertext bit for bit (the rank computes the unsharded result itself);
  * mfhe_crt_recombine_sharded must equal the unsharded mfhe_crt_compose_f64 of its poly slice;
  * a rank with bad arguments must fail on BOTH ranks (the verdict exchange), not leave its peer in a collective.
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
        # ---- raw recombine: 8 x 50-bit limbs, 6 polys of 4096 ----
        m8 = O.gen_primes(50, 1 << 18, 8)
        ctx8 = mfhe.Context(m8, 16)
        rng = np.random.default_rng(3)
        v = rng.integers(-(1 << 40), 1 << 40, (6, 4096), dtype=np.int64)
        res = np.stack([(v.astype(object) % int(m)).astype(np.uint64) for m in m8], axis=1)
        d = mfhe.to_device_u64(res.ravel())
        ref = torch.empty(6 * 4096, dtype=torch.float64, device="cuda")
        ctx8.crt_compose_f64(d, ref, 6, 4096)
        s0, lg8 = rank * (8 // world), 8 // world
        my = mfhe.to_device_u64(res[:, s0:s0 + lg8, :].ravel())
        bs = 6 // world
        for mode in ("allgather", "alltoall"):
            out = torch.empty(bs * 4096, dtype=torch.float64, device="cuda")
            ctx8.crt_recombine_sharded(comm, mode, my, 6, 4096, out)
            torch.cuda.synchronize()
            ok[f"recombine_{mode}"] = bool(torch.equal(out, ref[rank * bs * 4096:(rank + 1) * bs * 4096]))
        # ---- rank 1 passes a ctx_all with another scale: both ranks must get an error, neither may hang ----
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


@pytest.mark.skipif(_ngpus() < 2, reason="needs 2 visible GPUs (the round-end box has one)")
def test_two_rank_rccl_sharded_paths_equal_unsharded():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    uidq, resq = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, uidq, resq)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(resq.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert res[r] and all(res[r].values()), res
