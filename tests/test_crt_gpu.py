"""GPU parity: RNS decompose and wide CRT compose / centre-lift / f64 vs the CPU oracle, bit-exact.

Reference: quantize_coeff_to_rns_kernel (batched_encoder.cu:125-152),
crt_compose_centerlift_big_kernel (encoder.cu:191-230), compose_big_pair_to_complex_by_delta
(HE.cu:1007-1027), dequantize_exact_kernel (encoder.cu:112-150).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RNS = [17592186435073, 17182765057, 17184541441, 17186120449, 17186515201, 17186909953,
       17188883713, 17190462721, 17190857473, 17191844353, 17192831233]


def _param_sets(orc):
    return [
        ("reference", RNS, 6),
        ("C1-like L=1", orc.gen_primes(50, 1 << 14, 1), 12),
        ("C3 L=8 50-bit", orc.gen_primes(50, 1 << 18, 8), 16),
        ("C4 L=16", orc.gen_primes(50, 1 << 18, 16), 16),
        ("C5 L=32", orc.gen_primes(50, 1 << 19, 32), 17),
        ("60-bit L=5", orc.gen_primes(61, 1 << 10, 5), 8),
    ]


def _values(rng, count, delta):
    z = rng.uniform(-1.0, 1.0, count)
    z[:8] = [0.0, 0.5 / delta, -0.5 / delta, 1.5 / delta, -2.5 / delta, 1.0, -1.0, 2.0 ** 27 / delta]
    return z


def test_rns_decompose_matches_oracle(mfhe, orc):
    import torch
    rng = np.random.default_rng(0)
    for name, moduli, log_n in _param_sets(orc):
        for delta in (2.0 ** 35, 2.0 ** 40 + 3.0):
            ctx = mfhe.Context(moduli, log_n, mfhe.CONV_PHANTOM, delta=delta)
            npoly, nc = 3, 4096
            z = _values(rng, npoly * nc, delta) * 1000.0
            zt = torch.from_numpy(z).cuda()
            out = torch.zeros(npoly * len(moduli) * nc, dtype=torch.int64, device="cuda")
            ctx.rns_decompose(zt, out, npoly, nc)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(mfhe.to_host_u64(out), orc.rns_decompose(z, npoly, nc, moduli, delta),
                                          err_msg=name)
            # strided (complex interleaved) input, as the encoder uses for re / im
            zc = torch.from_numpy(np.stack([z, -z], 1).ravel().copy()).cuda()
            ctx.rns_decompose(zc[1:], out, npoly, nc, in_stride=2)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(mfhe.to_host_u64(out), orc.rns_decompose(-z, npoly, nc, moduli, delta))


def test_crt_compose_and_f64_match_oracle(mfhe, orc):
    import torch
    rng = np.random.default_rng(1)
    for name, moduli, log_n in _param_sets(orc):
        ctx = mfhe.Context(moduli, log_n)
        W = ctx.crt_words
        assert W == orc.crt_words(moduli)
        npoly, nc = 2, 3000
        q = np.array(moduli, np.uint64)[None, :, None]
        data = (rng.integers(0, 2 ** 63, (npoly, len(moduli), nc), dtype=np.uint64) % q)
        # small centred values too (the decode regime): v in [-2^40, 2^40]
        small = rng.integers(-(1 << 40), 1 << 40, nc)
        data[1] = np.array([[int(v) % int(m) for v in small] for m in moduli], np.uint64)
        data[1, :, :3] = np.array([[0, 1, int(m) - 1] for m in moduli], np.uint64)
        data = data.ravel()
        d = mfhe.to_device_u64(data)
        mag = torch.zeros(npoly * nc * W, dtype=torch.int64, device="cuda")
        neg = torch.zeros(npoly * nc, dtype=torch.uint8, device="cuda")
        ctx.crt_compose(d, mag, neg, npoly, nc)
        torch.cuda.synchronize()
        omag, oneg = orc.crt_compose(data, npoly, len(moduli), nc, moduli, W)
        np.testing.assert_array_equal(mfhe.to_host_u64(mag).reshape(-1, W), omag, err_msg=name)
        np.testing.assert_array_equal(neg.cpu().numpy(), oneg, err_msg=name)
        ref = orc.big_to_f64(omag, oneg, W, ctx.delta)
        f = torch.zeros(npoly * nc, dtype=torch.float64, device="cuda")
        ctx.crt_to_f64(mag, neg, f, npoly * nc)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(f.cpu().numpy(), ref, err_msg=name)
        f2 = torch.zeros(2 * npoly * nc, dtype=torch.float64, device="cuda")
        ctx.crt_compose_f64(d, f2, npoly, nc, out_stride=2)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(f2.cpu().numpy()[::2], ref, err_msg=name)
        # truncating int64 centre lift (crt_compose_centerlift_kernel, encoder.cu:152-189): random residues
        # (wide values, truncated to the low word) and the small-value decode regime
        i64 = torch.zeros(npoly * nc, dtype=torch.int64, device="cuda")
        ctx.crt_compose_i64(d, i64, npoly, nc)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(i64.cpu().numpy(), orc.crt_compose_i64(data, npoly, len(moduli), nc, moduli, W),
                                      err_msg=name)
        np.testing.assert_array_equal(i64.cpu().numpy()[nc + 3:], small[3:], err_msg=name)


@pytest.mark.parametrize("nc", [4096, 3001])
def test_vector_and_scalar_kernels_agree(mfhe, orc, nc):
    """Even ncoeff with unit stride and 16-B aligned buffers runs the two-coefficient decompose kernel (16-B
    loads/stores), odd ncoeff or a misaligned output the one-coefficient kernel: both bit-exact against the
    oracle.  The compose then mixes fast and slow paths in one launch (random residues fail the fast-path
    check, small values take it), at unit and non-unit output strides."""
    import torch
    rng = np.random.default_rng(nc)
    for moduli, log_n in ((orc.gen_primes(50, 1 << 18, 8), 16), (orc.gen_primes(50, 1 << 18, 16), 16), (RNS, 6)):
        ctx = mfhe.Context(moduli, log_n)
        L, npoly = len(moduli), 3
        z = _values(rng, npoly * nc, ctx.delta)
        z[1::7] = rng.uniform(-1e6, 1e6, z[1::7].size)
        zt = torch.from_numpy(z).cuda()
        expect_r = orc.rns_decompose(z, npoly, nc, moduli, ctx.delta)
        for off in (0, 1):   # off = 1: an 8-B aligned (not 16-B) output view
            buf = torch.zeros(npoly * L * nc + 1, dtype=torch.int64, device="cuda")
            r = buf[off:off + npoly * L * nc]
            ctx.rns_decompose(zt, r, npoly, nc)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(mfhe.to_host_u64(r), expect_r)
        q = np.array(moduli, np.uint64)[None, :, None]
        res = expect_r.reshape(npoly, L, nc).copy()
        res[2] = rng.integers(0, 2 ** 63, (L, nc), dtype=np.uint64) % q[0]   # slow path
        res = res.ravel()
        omag, oneg = orc.crt_compose(res, npoly, L, nc, moduli, ctx.crt_words)
        ref = orc.big_to_f64(omag, oneg, ctx.crt_words, ctx.delta)
        d = mfhe.to_device_u64(res)
        for stride in (1, 3):
            f = torch.zeros(npoly * nc * stride, dtype=torch.float64, device="cuda")
            ctx.crt_compose_f64(d, f, npoly, nc, out_stride=stride)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(f.cpu().numpy()[::stride], ref)


def test_decompose_compose_roundtrip_full_size(mfhe):
    """Size-independent property at C3 scale: compose_f64(decompose(z)) == round(z*delta)/delta."""
    import torch
    import oracle
    moduli = oracle.gen_primes(50, 1 << 18, 8)
    ctx = mfhe.Context(moduli, 16)
    npoly, nc = 64, 1 << 16
    g = torch.Generator(device="cuda").manual_seed(3)
    z = torch.rand(npoly * nc, dtype=torch.float64, device="cuda", generator=g) * 2 - 1
    r = torch.empty(npoly * 8 * nc, dtype=torch.int64, device="cuda")
    ctx.rns_decompose(z, r, npoly, nc)
    out = torch.empty_like(z)
    ctx.crt_compose_f64(r, out, npoly, nc)
    torch.cuda.synchronize()
    zd = z * ctx.delta                     # exact (delta = 2^35)
    expect = torch.trunc(zd + torch.copysign(torch.full_like(zd, 0.5), zd)) / ctx.delta   # llround: ties away
    assert (torch.round(zd) != torch.trunc(zd + torch.copysign(torch.full_like(zd, 0.5), zd))).any()
    assert torch.equal(out, expect)


@pytest.mark.parametrize("small", [False, True])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_crt_compose_f64_sharded_matches_unsharded(mfhe, orc, world, small):
    """mfhe_crt_compose_f64_sharded reads the all-gather / all-to-all receive layouts in place, on random
    residues (full multi-word path) and on residues of small centred values (FP64 fast path)."""
    import torch
    moduli = orc.gen_primes(50, 1 << 18, 16)
    ctx = mfhe.Context(moduli, 16, mfhe.CONV_PHANTOM)
    B, L, N = 2 * world, 16, 2048
    lg, bs = L // world, 2
    rng = np.random.default_rng(world)
    qv = np.array(moduli, np.uint64)[None, :, None]
    if small:
        v = rng.integers(-(2 ** 61), 2 ** 61, (B, 1, N), dtype=np.int64)
        full = np.where(v < 0, (qv - (np.abs(v).astype(np.uint64) % qv)) % qv, v.astype(np.uint64) % qv)
    else:
        full = rng.integers(0, 2 ** 63, (B, L, N), dtype=np.uint64) % qv
    ref = torch.empty(bs * N, dtype=torch.float64, device="cuda")
    got = torch.empty_like(ref)
    # all-gather layout: [world][B][lg][N]; rank r composes polys [r*bs, (r+1)*bs)
    gathered = np.concatenate([full[:, g * lg:(g + 1) * lg, :].ravel() for g in range(world)])
    dg = mfhe.to_device_u64(gathered)
    # all-to-all layout for rank r: [world][bs][lg][N]
    for r in (0, world - 1):
        mine = mfhe.to_device_u64(full[r * bs:(r + 1) * bs].ravel())
        ctx.crt_compose_f64(mine, ref, bs, N)
        ctx.crt_compose_f64_sharded(dg, got, world, B * lg * N, bs, N, src_offset=r * bs * lg * N)
        torch.cuda.synchronize()
        assert torch.equal(got, ref)
        a2a = np.concatenate([full[r * bs:(r + 1) * bs, g * lg:(g + 1) * lg, :].ravel() for g in range(world)])
        ctx.crt_compose_f64_sharded(mfhe.to_device_u64(a2a), got, world, bs * lg * N, bs, N)
        torch.cuda.synchronize()
        assert torch.equal(got, ref)


@pytest.mark.parametrize("L,W", [(1, None), (1, 7), (2, None), (8, None), (9, None), (11, 7), (16, None), (24, None),
                                 (32, None), (40, None)])
def test_crt_compose_small_value_fast_path_boundaries(mfhe, orc, L, W):
    """Centred values around the fast path's limits (|X| near 2^62, near Q/2 for small Q) must match the
    full multi-word compose bit-exactly (oracle), whichever path the kernel takes.  r06: from 11 words of Q the fast
    path holds 32 residues in registers (crt.hip crt_fast_ch): L = 16, 24, 32 in one round, L = 40 in two with the
    check re-reading them."""
    import torch
    moduli = RNS[:L] if L == 11 else orc.gen_primes(50, 1 << 18, L)
    Q = 1
    for q in moduli:
        Q *= q
    vals = [0, 1, -1, 2 ** 35, -(2 ** 35) - 7, 2 ** 52 + 1, -(2 ** 53), 2 ** 62 - 1, -(2 ** 62 - 1), 2 ** 62, -(2 ** 62),
            2 ** 63 - 1, -(2 ** 63 - 1), 2 ** 64 + 3, -(2 ** 70)]
    half = (Q - 1) // 2
    vals += [half, -half, half - 1, -(half - 1)]
    vals = [v for v in vals if abs(v) <= half]
    nc = len(vals)
    res = np.array([[v % q for v in vals] for q in moduli], dtype=np.uint64).ravel()
    ctx = mfhe.Context(moduli, 6, mfhe.CONV_PHANTOM)
    if W:
        ctx.set_option(mfhe.OPT_CRT_WORDS, W)
    Wc = ctx.info().crt_words
    d = mfhe.to_device_u64(res)
    mag = torch.empty(nc * Wc, dtype=torch.int64, device="cuda")
    neg = torch.empty(nc, dtype=torch.uint8, device="cuda")
    ctx.crt_compose(d, mag, neg, 1, nc)
    f = torch.empty(nc, dtype=torch.float64, device="cuda")
    ctx.crt_compose_f64(d, f, 1, nc)
    torch.cuda.synchronize()
    m_ref, n_ref = orc.crt_compose(res, 1, L, nc, moduli, W=Wc)
    np.testing.assert_array_equal(mfhe.to_host_u64(mag).reshape(nc, Wc), m_ref)
    np.testing.assert_array_equal(neg.cpu().numpy(), n_ref)
    np.testing.assert_array_equal(f.cpu().numpy(), orc.big_to_f64(m_ref, n_ref, Wc, 2.0 ** 35))
    for i, v in enumerate(vals):   # and the value itself
        got = sum(int(w) << (64 * j) for j, w in enumerate(m_ref[i]))
        assert (-got if n_ref[i] else got) == v
