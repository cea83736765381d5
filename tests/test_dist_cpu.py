"""World-size-2 gloo tests of the multi-GPU residue-sharding exchange (mfhe/dist.py).

Each rank owns limbs [g*L/2, (g+1)*L/2) of every polynomial.  The exchange must hand each rank
the residues of its batch slice as `world` shards at (offset, shard_stride) -- the layout
mfhe_crt_compose_f64_sharded reads in place.  The CRT result of that layout is checked with the
oracle (the GPU test of the same kernel is in test_crt_gpu.py).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

RNS = [17592186435073, 17182765057, 17184541441, 17186120449]
B, N = 4, 16


def _full():
    rng = np.random.default_rng(11)
    q = np.array(RNS, np.uint64)[None, :, None]
    return rng.integers(0, 2 ** 63, (B, len(RNS), N), dtype=np.uint64) % q


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, mode, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root / "matrix-fhe-gpu_amd"), str(root / "tests")]
    import torch.distributed as dist
    from mfhe import dist as mdist
    import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = _full()
        L = len(RNS)
        s0, lg = mdist.limb_range(L, world, rank)
        shard = torch.from_numpy(full[:, s0:s0 + lg, :].astype(np.int64).copy())
        buf, off, stride, bs = mdist.exchange_residues(shard, B, lg, N, mode)
        b = buf.numpy().view(np.uint64)
        # rebuild [bs][L][N] from the sharded layout exactly as the kernel addresses it
        view = np.stack([b[off + s * stride: off + s * stride + bs * lg * N].reshape(bs, lg, N)
                         for s in range(world)], axis=1).reshape(bs, L, N)
        mine = full[rank * bs:(rank + 1) * bs]
        ok = np.array_equal(view, mine)
        mag, neg = O.crt_compose(view.ravel(), bs, L, N, RNS)
        want, wneg = O.crt_compose(mine.ravel(), bs, L, N, RNS)
        ok = ok and np.array_equal(mag, want) and np.array_equal(neg, wneg)
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("mode", ["allgather", "alltoall"])
def test_residue_shard_exchange(mode, world):
    """world 2 and 4 (the C4 config shards 16 limbs over 4 GPUs; here 4 limbs, one per rank)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


def test_limb_range_rejects_uneven():
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "matrix-fhe-gpu_amd"))
    from mfhe import dist as mdist
    assert mdist.limb_range(8, 4, 3) == (6, 2)
    with pytest.raises(ValueError):
        mdist.limb_range(6, 4, 0)


def _c4_rank(rank, world, port, mode, q):
    """BASELINE C4 decode exchange: 16 limbs over `world` ranks, every rank composes its lane slice and an
    all-gather of the f64 slices gives every rank the whole batch (mfhe_decode_sharded's data flow)."""
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root / "matrix-fhe-gpu_amd"), str(root / "tests")]
    import torch.distributed as dist
    from mfhe import dist as mdist
    import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        moduli = O.gen_primes(35, 197376, 16)
        lanes, n2 = 8, 16
        rng = np.random.default_rng(5)
        v = rng.integers(-(1 << 40), 1 << 40, (lanes, n2))
        full = np.stack([(v.astype(object) % m).astype(np.uint64) for m in moduli], axis=1)   # [lanes][16][n2]
        s0, lg = mdist.limb_range(16, world, rank)
        shard = torch.from_numpy(full[:, s0:s0 + lg, :].astype(np.int64).copy())
        buf, off, stride, bs = mdist.exchange_residues(shard, lanes, lg, n2, mode)
        b = buf.numpy().view(np.uint64)
        view = np.stack([b[off + s * stride: off + s * stride + bs * lg * n2].reshape(bs, lg, n2)
                         for s in range(world)], axis=1).reshape(bs, 16, n2)
        W = O.crt_words(moduli)
        mag, neg = O.crt_compose(view.ravel(), bs, 16, n2, moduli, W)
        mine = torch.from_numpy(O.big_to_f64(mag, neg, W, 2.0 ** 35))
        slices = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(slices, mine)
        got = torch.cat(slices).numpy()
        q.put((rank, bool(np.array_equal(got, v.ravel().astype(np.float64) / 2.0 ** 35))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("mode", ["allgather", "alltoall"])
def test_c4_decode_exchange(mode, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c4_rank, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}
