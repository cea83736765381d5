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
    """BASELINE C4 decode exchange: 16 limbs over `world` ranks, the chunked recombine writes every rank's lanes of
    each chunk at their lane index and one in-place all-gather per chunk gives every rank the whole batch
    (mfhe_decode_sharded's data flow, he.hip decode_sharded_impl, restated by mfhe.dist.decode_recombine)."""
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
        lanes, n2 = 16, 8
        rng = np.random.default_rng(5)
        v = rng.integers(-(1 << 40), 1 << 40, (lanes, n2))
        full = np.stack([(v.astype(object) % m).astype(np.uint64) for m in moduli], axis=1)   # [lanes][16][n2]
        s0, lg = mdist.limb_range(16, world, rank)
        shard = torch.from_numpy(full[:, s0:s0 + lg, :].astype(np.int64).copy()).view(-1)
        ok = True
        for chunk in (lanes // 4, lanes, 3 * world):   # 4 chunks (as the decode), one chunk, a ragged last chunk
            out = torch.full((lanes * n2,), np.nan, dtype=torch.float64)
            mdist.decode_recombine(_OracleShardCtx(moduli, 2.0 ** 35), shard, lanes, n2, mode, chunk, out)
            ok = ok and np.array_equal(out.numpy(), v.ravel().astype(np.float64) / 2.0 ** 35)
        q.put((rank, bool(ok)))
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


class _OracleShardCtx:
    """Stands in for an mfhe.Context in crt_recombine's torch.distributed path on CPU: info().num_limbs and
    crt_compose_f64_sharded, the latter restated with the oracle over the sharded layout exactly as
    crt_compose_f64_kernel addresses it (limb k = s * Lg + j at src_offset + s * shard_stride + (p * Lg + j) * n)."""

    class _Info:
        def __init__(self, L):
            self.num_limbs = L

    def __init__(self, moduli, delta):
        self.moduli, self.delta = moduli, delta

    def info(self):
        return self._Info(len(self.moduli))

    def crt_compose_f64_sharded(self, src, out, nshards, shard_stride, npoly, ncoeff, out_stride=1, stream=None,
                                src_offset=0):
        import oracle as O
        L = len(self.moduli)
        lg = L // nshards
        b = src.numpy().view(np.uint64)
        res = np.empty((npoly, L, ncoeff), np.uint64)
        for k in range(L):
            s, j = divmod(k, lg)
            for p in range(npoly):
                base = src_offset + s * shard_stride + (p * lg + j) * ncoeff
                res[p, k] = b[base:base + ncoeff]
        W = O.crt_words(self.moduli)
        mag, neg = O.crt_compose(res.ravel(), npoly, L, ncoeff, self.moduli, W)
        out.view(-1)[::out_stride][:npoly * ncoeff] = torch.from_numpy(O.big_to_f64(mag, neg, W, self.delta))
        return out


def _c5_rank(rank, world, port, mode, chunk, q):
    """BASELINE C5's exchange at small N: L = 32 limbs sharded over `world` ranks, the recombine chunked over
    polys (mfhe.dist.crt_recombine_chunked, the bench's c5 line), every rank's output rows = the composed
    values of the polys owned_polys says it owns."""
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
        L, batch, n, delta = 32, 16, 8, 2.0 ** 35
        moduli = O.gen_primes(50, 1 << 10, L)
        rng = np.random.default_rng(7)
        v = rng.integers(-(1 << 52), 1 << 52, (batch, n))
        full = np.stack([(v.astype(object) % m).astype(np.uint64) for m in moduli], axis=1)   # [batch][L][n]
        s0, lg = mdist.limb_range(L, world, rank)
        shard = torch.from_numpy(full[:, s0:s0 + lg, :].astype(np.int64).copy()).view(-1)
        out = torch.full((batch // world * n,), np.nan, dtype=torch.float64)
        mdist.crt_recombine_chunked(_OracleShardCtx(moduli, delta), shard, batch, n, mode, chunk, out)
        own = mdist.owned_polys(batch, world, rank, chunk)
        want = v[own].ravel().astype(np.float64) / delta
        ok = len(own) == batch // world and np.array_equal(out.numpy(), want)
        # every poly is owned by exactly one rank
        allown = [None] * world
        dist.all_gather_object(allown, own)
        ok = ok and sorted(sum(allown, [])) == list(range(batch))
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["allgather", "alltoall"])
@pytest.mark.parametrize("world,chunk", [(8, 8), (8, 16), (4, 12), (2, 4)])
def test_c5_chunked_recombine_layout(mode, world, chunk):
    """C5 is 8 GPUs: world 8 (one chunk and two chunks of polys), plus 4 and 2 ranks with ragged chunking."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c5_rank, args=(r, world, port, mode, chunk, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


def test_chunk_plan_bounds():
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "matrix-fhe-gpu_amd"))
    from mfhe import dist as mdist
    assert mdist.chunk_plan(4096, 8, 512) == [(p, 512, p // 8) for p in range(0, 4096, 512)]
    assert mdist.chunk_plan(20, 4, 6) == [(0, 4, 0), (4, 4, 1), (8, 4, 2), (12, 4, 3), (16, 4, 4)]
    assert mdist.chunk_plan(12, 2, 8) == [(0, 8, 0), (8, 4, 4)]
    with pytest.raises(ValueError):
        mdist.chunk_plan(10, 4, 8)
