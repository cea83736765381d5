"""Native multi-GPU recombine (include/mfhe.h mfhe_comm_* / mfhe_crt_recombine_sharded) on one GPU.

At world 1 the recombine composes straight from the shard (no exchange, r06). The chunked tests pass
MFHE_RECOMBINE_SELF_EXCHANGE, so a 1-rank RCCL communicator still runs the real exchange code path: ncclAllGather /
ncclAllToAll into the communicator-owned receive halves, the exchange stream and its events, then the sharded
compose. Every result must equal the unsharded mfhe_crt_compose_f64 bit for bit.  RCCL refuses two ranks on one GPU, so the G > 1 layout is pinned by the
gloo tests in test_dist_cpu.py (same offsets and strides) and by the sharded-compose kernel test below,
which feeds it G shards laid out exactly as the G-rank exchanges deliver them.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SX = 32   # mfhe.RECOMBINE_SELF_EXCHANGE: world 1 runs the exchange pipeline anyway (tests of the multi-rank machinery)


def _residues(rng, npoly, moduli, ncoeff, delta):
    """RNS residues of centred values |v| < 2^40 (the decode regime), [npoly][L][ncoeff]."""
    v = rng.integers(-(1 << 40), 1 << 40, (npoly, ncoeff), dtype=np.int64)
    q = np.array(moduli, dtype=object)
    return np.stack([(v.astype(object) % int(m)).astype(np.uint64) for m in q], axis=1), v


@pytest.mark.parametrize("mode", ["allgather", "alltoall"])
def test_recombine_one_rank_equals_unsharded(mfhe, orc, mode):
    import torch
    moduli = orc.gen_primes(50, 1 << 18, 8)
    ctx = mfhe.Context(moduli, 16)
    npoly, ncoeff = 6, 1 << 12
    rng = np.random.default_rng(3)
    res, v = _residues(rng, npoly, moduli, ncoeff, ctx.info().delta)
    d = mfhe.to_device_u64(res.ravel())
    comm = mfhe.Comm.from_id(mfhe.Comm.unique_id(), 1, 0)
    try:
        ctx.crt_recombine_reserve(comm, mode, npoly, ncoeff)
        out = torch.empty(npoly * ncoeff, dtype=torch.float64, device="cuda")
        ctx.crt_recombine_sharded(comm, mode, d, npoly, ncoeff, out)
        ref = torch.empty_like(out)
        ctx.crt_compose_f64(d, ref, npoly, ncoeff)
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
        np.testing.assert_array_equal(out.cpu().numpy(), v.ravel().astype(np.float64) / ctx.info().delta)
        # raw exchange: a 1-rank all-gather is a copy
        recv = torch.empty_like(d)
        comm.allgather_limbs(d, recv)
        torch.cuda.synchronize()
        assert torch.equal(recv, d)
    finally:
        comm.close()
        ctx.close()


def test_recombine_rejects_bad_shapes(mfhe, orc):
    import torch
    moduli = orc.gen_primes(50, 1 << 14, 3)
    ctx = mfhe.Context(moduli, 12)
    comm = mfhe.Comm.from_id(mfhe.Comm.unique_id(), 1, 0)
    try:
        d = torch.zeros(4 * 3 * 16, dtype=torch.int64, device="cuda")
        out = torch.zeros(4 * 16, dtype=torch.float64, device="cuda")
        with pytest.raises(mfhe.MfheError):
            ctx.crt_recombine_sharded(comm, 7, d, 4, 16, out)
        with pytest.raises(ValueError):   # undersized shard caught on the host
            ctx.crt_recombine_sharded(comm, "allgather", d[:10], 4, 16, out)
    finally:
        comm.close()
        ctx.close()


@pytest.mark.parametrize("G,mode", [(2, "allgather"), (4, "allgather"), (2, "alltoall"), (4, "alltoall")])
def test_sharded_compose_layout_of_g_rank_exchange(mfhe, orc, G, mode):
    """What rank g composes after a G-rank exchange, built on one GPU in the exact receive layout the
    native call uses (all-gather: [G][B][L/G][n] at offset g*B/G; all-to-all: [G][B/G][L/G][n])."""
    import torch
    L, B, n = 8, 8, 256
    moduli = orc.gen_primes(50, 1 << 14, L)
    ctx = mfhe.Context(moduli, 12)
    rng = np.random.default_rng(G)
    res, _ = _residues(rng, B, moduli, n, ctx.info().delta)
    lg, bs = L // G, B // G
    shards = [res[:, g * lg:(g + 1) * lg, :] for g in range(G)]          # rank g's [B][L/G][n]
    ref = torch.empty(B * n, dtype=torch.float64, device="cuda")
    ctx.crt_compose_f64(mfhe.to_device_u64(res.ravel()), ref, B, n)
    for g in range(G):
        if mode == "allgather":
            recv = np.concatenate([s.ravel() for s in shards])
            off, stride = g * bs * lg * n, B * lg * n
        else:
            recv = np.concatenate([s[g * bs:(g + 1) * bs].ravel() for s in shards])
            off, stride = 0, bs * lg * n
        out = torch.empty(bs * n, dtype=torch.float64, device="cuda")
        ctx.crt_compose_f64_sharded(mfhe.to_device_u64(recv), out, G, stride, bs, n, src_offset=off)
        torch.cuda.synchronize()
        assert torch.equal(out, ref[g * bs * n:(g + 1) * bs * n])
    ctx.close()


@pytest.mark.parametrize("mode", ["allgather", "alltoall"])
@pytest.mark.parametrize("rows_global", [False, True])
def test_chunked_recombine_one_rank_equals_unsharded(mfhe, orc, mode, rows_global):
    """mfhe_crt_recombine_chunked: several chunks, a ragged last chunk (11 polys in chunks of
    4: 4 + 4 + 3), the exchange on the communicator's stream beside the compose -- bit-identical to the unsharded
    compose.  Called twice back to back (the second call's first exchanges wait on the first call's composes of
    the same receive halves), and once more with a chunk as large as the batch."""
    import torch
    moduli = orc.gen_primes(50, 1 << 18, 8)
    ctx = mfhe.Context(moduli, 16)
    npoly, ncoeff = 11, 1 << 12
    rng = np.random.default_rng(5)
    res, v = _residues(rng, npoly, moduli, ncoeff, ctx.info().delta)
    d = mfhe.to_device_u64(res.ravel())
    ref = torch.empty(npoly * ncoeff, dtype=torch.float64, device="cuda")
    ctx.crt_compose_f64(d, ref, npoly, ncoeff)
    comm = mfhe.Comm.from_id(mfhe.Comm.unique_id(), 1, 0)
    try:
        ctx.crt_recombine_chunked_reserve(comm, mode, 4, ncoeff)
        for chunk in (4, 4, 64, 1):
            out = torch.full((npoly * ncoeff,), float("nan"), dtype=torch.float64, device="cuda")
            ctx.crt_recombine_chunked(comm, mode, d, npoly, ncoeff, chunk, out, rows_global=rows_global, flags=SX)
            torch.cuda.synchronize()
            assert torch.equal(out, ref), chunk
        # strided output (the decode writes re / im interleaved)
        out2 = torch.full((2 * npoly * ncoeff,), float("nan"), dtype=torch.float64, device="cuda")
        ctx.crt_recombine_chunked(comm, mode, d, npoly, ncoeff, 3, out2[1:], out_stride=2, rows_global=rows_global,
                                  flags=SX)
        torch.cuda.synchronize()
        assert torch.equal(out2[1::2], ref) and torch.isnan(out2[0::2]).all()
        np.testing.assert_array_equal(ref.cpu().numpy(), v.ravel().astype(np.float64) / ctx.info().delta)
    finally:
        comm.close()
        ctx.close()


def test_chunked_recombine_rejects_bad_arguments(mfhe, orc):
    import torch
    moduli = orc.gen_primes(50, 1 << 14, 3)
    ctx = mfhe.Context(moduli, 12)
    comm = mfhe.Comm.from_id(mfhe.Comm.unique_id(), 1, 0)
    try:
        d = torch.zeros(4 * 3 * 16, dtype=torch.int64, device="cuda")
        out = torch.zeros(4 * 16, dtype=torch.float64, device="cuda")
        with pytest.raises(mfhe.MfheError):
            ctx.crt_recombine_chunked(comm, 7, d, 4, 16, 2, out)
        with pytest.raises(mfhe.MfheError):   # unknown flag bits
            mfhe.check(mfhe.lib.mfhe_crt_recombine_chunked(ctx.handle, comm._h, 0, d.data_ptr(), 4, 16, 2,
                                                           out.data_ptr(), 1, 64, None))
        with pytest.raises(ValueError):   # undersized output caught on the host
            ctx.crt_recombine_chunked(comm, "alltoall", d, 4, 16, 2, out[:10])
    finally:
        comm.close()
        ctx.close()


@pytest.mark.parametrize("agree", [False, True])
def test_chunked_recombine_injected_failure_keeps_communicator_usable(mfhe, orc, agree):
    """a local failure after the exchanges started (MFHE_RECOMBINE_DEBUG_FAIL fails the compose of
    chunk 1) returns an error once every remaining exchange was still issued -- no return in the middle of the
    chunk loop -- and the communicator stays usable: the next call on it is bit-exact.  With
    MFHE_RECOMBINE_AGREE the error also goes through the all-rank status agreement."""
    import torch
    moduli = orc.gen_primes(50, 1 << 18, 8)
    ctx = mfhe.Context(moduli, 16)
    npoly, ncoeff = 11, 1 << 12
    rng = np.random.default_rng(7)
    res, _ = _residues(rng, npoly, moduli, ncoeff, ctx.info().delta)
    d = mfhe.to_device_u64(res.ravel())
    ref = torch.empty(npoly * ncoeff, dtype=torch.float64, device="cuda")
    ctx.crt_compose_f64(d, ref, npoly, ncoeff)
    comm = mfhe.Comm.from_id(mfhe.Comm.unique_id(), 1, 0)
    try:
        ctx.crt_recombine_chunked_reserve(comm, "alltoall", 4, ncoeff)
        out = torch.full((npoly * ncoeff,), float("nan"), dtype=torch.float64, device="cuda")
        flags = mfhe.RECOMBINE_DEBUG_FAIL | (mfhe.RECOMBINE_AGREE if agree else 0) | SX
        with pytest.raises(mfhe.MfheError, match="injected"):
            ctx.crt_recombine_chunked(comm, "alltoall", d, npoly, ncoeff, 4, out, flags=flags)
        torch.cuda.synchronize()
        o = out.view(npoly, ncoeff)
        assert torch.equal(o[:4], ref.view(npoly, ncoeff)[:4])   # chunk 0 composed before the failure
        assert torch.isnan(o[4:]).all()                          # chunks 1, 2: exchanged, not composed
        for _ in range(2):   # the communicator and its receive halves are usable afterwards
            out.fill_(float("nan"))
            ctx.crt_recombine_chunked(comm, "alltoall", d, npoly, ncoeff, 4, out, flags=SX)
            torch.cuda.synchronize()
            assert torch.equal(out, ref)
    finally:
        comm.close()
        ctx.close()


def test_chunked_recombine_exchange_only_and_after_prev(mfhe, orc):
    """MFHE_RECOMBINE_EXCHANGE_ONLY (bench.py's exchange_only_ms) leaves the output untouched and accepts a null
    one; MFHE_RECOMBINE_AFTER_PREV (the decode's im call right after its re call) gives the same result as a
    plain call when the shard was ready at the previous call."""
    import torch
    moduli = orc.gen_primes(50, 1 << 18, 8)
    ctx = mfhe.Context(moduli, 16)
    npoly, ncoeff = 9, 1 << 12
    rng = np.random.default_rng(9)
    res, _ = _residues(rng, npoly, moduli, ncoeff, ctx.info().delta)
    d = mfhe.to_device_u64(res.ravel())
    d2 = mfhe.to_device_u64(res[::-1].copy().ravel())
    ref = torch.empty(npoly * ncoeff, dtype=torch.float64, device="cuda")
    ref2 = torch.empty_like(ref)
    ctx.crt_compose_f64(d, ref, npoly, ncoeff)
    ctx.crt_compose_f64(d2, ref2, npoly, ncoeff)
    comm = mfhe.Comm.from_id(mfhe.Comm.unique_id(), 1, 0)
    try:
        ctx.crt_recombine_chunked_reserve(comm, "allgather", 2, ncoeff)
        out = torch.full((npoly * ncoeff,), float("nan"), dtype=torch.float64, device="cuda")
        ctx.crt_recombine_chunked(comm, "allgather", d, npoly, ncoeff, 2, out, flags=mfhe.RECOMBINE_EXCHANGE_ONLY | SX)
        ctx.crt_recombine_chunked(comm, "allgather", d, npoly, ncoeff, 2, None, flags=mfhe.RECOMBINE_EXCHANGE_ONLY | SX)
        torch.cuda.synchronize()
        assert torch.isnan(out).all()
        out2 = torch.full_like(out, float("nan"))
        ctx.crt_recombine_chunked(comm, "allgather", d, npoly, ncoeff, 2, out, flags=SX)
        ctx.crt_recombine_chunked(comm, "allgather", d2, npoly, ncoeff, 2, out2, flags=mfhe.RECOMBINE_AFTER_PREV | SX)
        torch.cuda.synchronize()
        assert torch.equal(out, ref) and torch.equal(out2, ref2)
    finally:
        comm.close()
        ctx.close()


@pytest.mark.parametrize("mode", ["allgather", "alltoall"])
def test_world1_recombine_composes_from_the_shard(mfhe, orc, mode):
    """at world 1 the chunked recombine exchanges nothing and composes straight from the shard -- bit
    for bit the unsharded compose, for every chunk size and both row orders. EXCHANGE_ONLY then does nothing, and
    DEBUG_FAIL still fails. COMPOSE_ONLY composes. No receive buffer is needed (no reserve is called here)."""
    import torch
    moduli = orc.gen_primes(50, 1 << 18, 8)
    ctx = mfhe.Context(moduli, 16)
    npoly, ncoeff = 11, 1 << 12
    res, v = _residues(np.random.default_rng(21), npoly, moduli, ncoeff, ctx.info().delta)
    d = mfhe.to_device_u64(res.ravel())
    ref = torch.empty(npoly * ncoeff, dtype=torch.float64, device="cuda")
    ctx.crt_compose_f64(d, ref, npoly, ncoeff)
    comm = mfhe.Comm.from_id(mfhe.Comm.unique_id(), 1, 0)
    try:
        for chunk in (1, 4, 64):
            for rows_global in (False, True):
                for fl in (0, mfhe.RECOMBINE_COMPOSE_ONLY, mfhe.RECOMBINE_AFTER_PREV | mfhe.RECOMBINE_AGREE):
                    out = torch.full((npoly * ncoeff,), float("nan"), dtype=torch.float64, device="cuda")
                    ctx.crt_recombine_chunked(comm, mode, d, npoly, ncoeff, chunk, out, rows_global=rows_global,
                                              flags=fl)
                    torch.cuda.synchronize()
                    assert torch.equal(out, ref), (chunk, rows_global, fl)
        out = torch.full((npoly * ncoeff,), float("nan"), dtype=torch.float64, device="cuda")
        ctx.crt_recombine_chunked(comm, mode, d, npoly, ncoeff, 4, out, flags=mfhe.RECOMBINE_EXCHANGE_ONLY)
        ctx.crt_recombine_chunked(comm, mode, d, npoly, ncoeff, 4, None, flags=mfhe.RECOMBINE_EXCHANGE_ONLY)
        torch.cuda.synchronize()
        assert torch.isnan(out).all()
        with pytest.raises(mfhe.MfheError, match="injected"):
            ctx.crt_recombine_chunked(comm, mode, d, npoly, ncoeff, 4, out, flags=mfhe.RECOMBINE_DEBUG_FAIL)
        with pytest.raises(mfhe.MfheError):   # the two measurement flags exclude each other
            ctx.crt_recombine_chunked(comm, mode, d, npoly, ncoeff, 4, out,
                                      flags=mfhe.RECOMBINE_EXCHANGE_ONLY | mfhe.RECOMBINE_COMPOSE_ONLY)
        out.zero_()
        ctx.crt_recombine_sharded(comm, mode, d, npoly - 0, ncoeff, out)   # the one-shot form: also no exchange
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
        np.testing.assert_array_equal(ref.cpu().numpy(), v.ravel().astype(np.float64) / ctx.info().delta)
    finally:
        comm.close()
        ctx.close()


def test_compose_only_recomposes_the_halves(mfhe, orc):
    """MFHE_RECOMBINE_COMPOSE_ONLY (bench.py compose_only_ms) through the exchange pipeline (self-exchange): with two
    chunks, the halves hold exactly chunks 0 and 1 after a normal call, so a compose-only call reproduces its output
    bit for bit without exchanging. A later AFTER_PREV call must not rely on a compose-only call's (absent)
    exchanges: it still equals the plain result."""
    import torch
    moduli = orc.gen_primes(50, 1 << 18, 8)
    ctx = mfhe.Context(moduli, 16)
    npoly, ncoeff = 8, 1 << 12
    res, _ = _residues(np.random.default_rng(23), npoly, moduli, ncoeff, ctx.info().delta)
    d = mfhe.to_device_u64(res.ravel())
    ref = torch.empty(npoly * ncoeff, dtype=torch.float64, device="cuda")
    ctx.crt_compose_f64(d, ref, npoly, ncoeff)
    comm = mfhe.Comm.from_id(mfhe.Comm.unique_id(), 1, 0)
    try:
        for mode in ("allgather", "alltoall"):
            ctx.crt_recombine_chunked_reserve(comm, mode, 4, ncoeff)
            out = torch.full((npoly * ncoeff,), float("nan"), dtype=torch.float64, device="cuda")
            ctx.crt_recombine_chunked(comm, mode, d, npoly, ncoeff, 4, out, flags=SX)
            out2 = torch.full_like(out, float("nan"))
            ctx.crt_recombine_chunked(comm, mode, d, npoly, ncoeff, 4, out2, flags=SX | mfhe.RECOMBINE_COMPOSE_ONLY)
            torch.cuda.synchronize()
            assert torch.equal(out, ref) and torch.equal(out2, ref), mode
            # after a reserve no exchange is tracked: AFTER_PREV is ignored (the exchanges wait for the stream)
            ctx.crt_recombine_chunked_reserve(comm, mode, 4, ncoeff)
            out3 = torch.full_like(out, float("nan"))
            ctx.crt_recombine_chunked(comm, mode, d, npoly, ncoeff, 4, out3, flags=SX | mfhe.RECOMBINE_AFTER_PREV)
            torch.cuda.synchronize()
            assert torch.equal(out3, ref), mode
    finally:
        comm.close()
        ctx.close()
