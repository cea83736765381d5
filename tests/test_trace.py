"""Trace GEMM (src/core/batched_trace.cu:37-197, src/core/trace.cu:30-161): B -> B', C = n A B'^T and the
rescale, [batch][L][n][n] planes.

The reference has no test for this stage, so parity is anchored on the oracle restatement
(orc_trace_*, the reference's exact add_mod / sub_mod / mul_mod_u128 sequence), itself checked here
against an independent Python-integer computation of the same linear algebra.  Parity with reference
outputs is unpinned (no reference run is possible here).  Integer work: bit-exact.
"""
import numpy as np
import pytest

RNS = [17592186435073, 17182765057, 17184541441, 17186120449, 17186515201, 17186909953,
       17188883713, 17190462721, 17190857473, 17191844353, 17192831233]


def _rand(rng, batch, L, n, moduli):
    q = np.array(moduli[:L], np.uint64)[None, :, None]
    return (rng.integers(0, 2 ** 63, (batch, L, n * n), dtype=np.uint64) % q).ravel()


def _py_trace(ar, ai, br, bi, n, L, batch, moduli):
    """Independent restatement with Python integers: map B -> B', then C = n A B'^T (complex mod q)."""
    shp = (batch, L, n, n)
    ar, ai, br, bi = (x.reshape(shp).astype(object) for x in (ar, ai, br, bi))
    cr = np.zeros(shp, dtype=object)
    ci = np.zeros(shp, dtype=object)
    for b in range(batch):
        for l in range(L):
            q = int(moduli[l])
            # B'(X) = conj(B)(X^-1) with X^n = i: row j -> -j, times -i for j != 0
            pr = np.zeros((n, n), dtype=object)
            pi = np.zeros((n, n), dtype=object)
            for j in range(n):
                re, im = br[b, l, j], (-bi[b, l, j]) % q
                if j:
                    re, im = im, (-br[b, l, j]) % q      # (-i)(re + i im) = im - i re
                pr[(-j) % n], pi[(-j) % n] = re, im
            A_r, A_i = ar[b, l], ai[b, l]
            cr[b, l] = (n * (A_r.dot(pr.T) - A_i.dot(pi.T))) % q
            ci[b, l] = (n * (A_r.dot(pi.T) + A_i.dot(pr.T))) % q
    return cr.ravel().astype(np.uint64), ci.ravel().astype(np.uint64)


def test_oracle_trace_matches_python_integers(orc):
    rng = np.random.default_rng(7)
    n, L, batch = 8, 3, 2
    ar, ai, br, bi = (_rand(rng, batch, L, n, RNS) for _ in range(4))
    bpr, bpi = orc.trace_map_bprime(br, bi, n, L, batch, RNS)
    cr, ci = orc.trace_gemm(ar, ai, bpr, bpi, n, L, batch, RNS)
    er, ei = _py_trace(ar, ai, br, bi, n, L, batch, RNS)
    np.testing.assert_array_equal(cr, er)
    np.testing.assert_array_equal(ci, ei)
    # rescale: the reference's (inv0, inv1, inv2) call leaves limbs >= 3 multiplied by 0
    inv = [orc.L.orc_invmod(2 ** 35 % q, q) for q in RNS[:L]]
    sr, si = orc.trace_rescale(cr, ci, n, L, batch, RNS, inv)
    for l in range(L):
        q = RNS[l]
        v = cr.reshape(batch, L, -1)[:, l].astype(object) * inv[l] % q
        np.testing.assert_array_equal(sr.reshape(batch, L, -1)[:, l], v.astype(np.uint64))


def _gpu_case(mfhe, orc, moduli, log_n_ctx, n, L, batch, seed, split=1):
    import torch
    ctx = mfhe.Context(moduli, log_n_ctx, mfhe.CONV_PHANTOM)
    ctx.set_option(mfhe.OPT_TRACE_SPLIT, split)
    rng = np.random.default_rng(seed)
    ar, ai, br, bi = (_rand(rng, batch, L, n, moduli) for _ in range(4))
    d = [mfhe.to_device_u64(x) for x in (ar, ai, br, bi)]
    bp = [torch.empty_like(d[0]), torch.empty_like(d[0])]
    c = [torch.empty_like(d[0]), torch.empty_like(d[0])]
    ctx.trace_map_bprime(d[2], d[3], bp[0], bp[1], n, L, batch)
    ctx.trace_gemm(d[0], d[1], bp[0], bp[1], c[0], c[1], n, L, batch)
    torch.cuda.synchronize()
    obpr, obpi = orc.trace_map_bprime(br, bi, n, L, batch, moduli)
    np.testing.assert_array_equal(mfhe.to_host_u64(bp[0]), obpr)
    np.testing.assert_array_equal(mfhe.to_host_u64(bp[1]), obpi)
    ocr, oci = orc.trace_gemm(ar, ai, obpr, obpi, n, L, batch, moduli)
    np.testing.assert_array_equal(mfhe.to_host_u64(c[0]), ocr)
    np.testing.assert_array_equal(mfhe.to_host_u64(c[1]), oci)
    inv = [orc.L.orc_invmod(2 ** 35 % q, q) for q in moduli[:3]] + [0] * (L - 3) if L > 3 else \
        [orc.L.orc_invmod(2 ** 35 % q, q) for q in moduli[:L]]
    ctx.trace_rescale(c[0], c[1], n, L, batch, inv)
    torch.cuda.synchronize()
    osr, osi = orc.trace_rescale(ocr, oci, n, L, batch, moduli, inv)
    np.testing.assert_array_equal(mfhe.to_host_u64(c[0]), osr)
    np.testing.assert_array_equal(mfhe.to_host_u64(c[1]), osi)


@pytest.mark.gpu
@pytest.mark.parametrize("split", [2, 1, 0])
@pytest.mark.parametrize("n,L,batch", [(64, 11, 16), (64, 3, 1), (128, 2, 3), (256, 1, 1), (8, 11, 4), (2, 1, 5)])
def test_trace_reference_moduli_vs_oracle(mfhe, orc, n, L, batch, split):
    """n = 64 / 128 / 256: the split-digit kernel on the FP64 matrix cores (split = 2) or as VALU FMAs
    (split = 1; n > 64 crosses their 64-k reductions), or the modmul tile kernel (split = 0, KR = 16);
    n = 8 / 2: the u128 kernel."""
    _gpu_case(mfhe, orc, RNS, 6, n, L, batch, n * 100 + L, split)


@pytest.mark.gpu
def test_trace_split_extreme_operands(mfhe, orc):
    """Split kernel at its digit bounds: every operand q - 1 or (q - 1) / 2 (largest centred magnitudes)."""
    import torch
    n, L, batch = 128, 11, 2
    ctx = mfhe.Context(RNS, 6, mfhe.CONV_PHANTOM)
    q = np.array(RNS, np.uint64)[None, :, None]
    hi = np.broadcast_to(q - 1, (batch, L, n * n)).ravel().copy()
    half = np.broadcast_to((q - 1) // 2, (batch, L, n * n)).ravel().copy()
    for split, (ar, ai, br, bi) in [(m, x) for m in (1, 2)
                                    for x in ((hi, hi, hi, hi), (half, half, half, half), (hi, half, half, hi))]:
        ctx.set_option(mfhe.OPT_TRACE_SPLIT, split)
        d = [mfhe.to_device_u64(x) for x in (ar, ai, br, bi)]
        c = [torch.empty_like(d[0]), torch.empty_like(d[0])]
        ctx.trace_gemm(d[0], d[1], d[2], d[3], c[0], c[1], n, L, batch)
        torch.cuda.synchronize()
        ocr, oci = orc.trace_gemm(ar, ai, br, bi, n, L, batch, RNS)
        np.testing.assert_array_equal(mfhe.to_host_u64(c[0]), ocr)
        np.testing.assert_array_equal(mfhe.to_host_u64(c[1]), oci)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [40, 45, 49, 58])
@pytest.mark.parametrize("split", [2, 1])
def test_trace_wide_moduli_vs_oracle(mfhe, orc, bits, split):
    """40 / 45-bit primes: split kernels (S = 20 / 23); 49-bit: modmul kernel with KR = 2; 58-bit: u128."""
    moduli = orc.gen_primes(bits, 1 << 8, 4)
    _gpu_case(mfhe, orc, moduli, 6, 128, 4, 3, bits, split)


@pytest.mark.gpu
def test_trace_invalid_arguments(mfhe):
    import torch
    ctx = mfhe.Context(RNS, 6, mfhe.CONV_PHANTOM)
    t = torch.zeros(64 * 64, dtype=torch.int64, device="cuda")
    with pytest.raises(mfhe.MfheError):
        ctx.trace_gemm(t, t, t, t, t, t, 48, 1, 1)        # n not a power of two
    big = [torch.zeros(12 * 64 * 64, dtype=torch.int64, device="cuda") for _ in range(6)]
    with pytest.raises(mfhe.MfheError):
        ctx.trace_gemm(*big, 64, 12, 1)                   # more limbs than the context
    with pytest.raises(mfhe.MfheError):
        ctx.trace_map_bprime(t, t, t, t, 64, 1, 1)        # aliasing output


@pytest.mark.gpu
@pytest.mark.parametrize("n,L,batch,rescale", [(64, 11, 8, True), (64, 11, 3, False), (128, 3, 2, True),
                                               (256, 1, 1, True)])
def test_trace_product_fused_vs_oracle(mfhe, orc, n, L, batch, rescale):
    """mfhe_trace_product (map + GEMM + rescale in one launch) == the oracle's three stages."""
    import torch
    ctx = mfhe.Context(RNS, 6, mfhe.CONV_PHANTOM)
    rng = np.random.default_rng(n + L)
    ar, ai, br, bi = (_rand(rng, batch, L, n, RNS) for _ in range(4))
    d = [mfhe.to_device_u64(x) for x in (ar, ai, br, bi)]
    c = [torch.empty_like(d[0]), torch.empty_like(d[0])]
    inv = ([orc.L.orc_invmod(2 ** 35 % q, q) for q in RNS[:min(L, 3)]] + [0] * max(0, L - 3)) if rescale else None
    ctx.trace_product(d[0], d[1], d[2], d[3], c[0], c[1], n, L, batch, inv)
    torch.cuda.synchronize()
    obpr, obpi = orc.trace_map_bprime(br, bi, n, L, batch, RNS)
    ocr, oci = orc.trace_gemm(ar, ai, obpr, obpi, n, L, batch, RNS)
    if rescale:
        ocr, oci = orc.trace_rescale(ocr, oci, n, L, batch, RNS, inv)
    np.testing.assert_array_equal(mfhe.to_host_u64(c[0]), ocr)
    np.testing.assert_array_equal(mfhe.to_host_u64(c[1]), oci)


@pytest.mark.gpu
def test_trace_product_unsupported_shapes(mfhe, orc):
    import torch
    t = torch.zeros(2 * 64 * 64, dtype=torch.int64, device="cuda")
    o = torch.zeros_like(t)
    ctx = mfhe.Context(orc.gen_primes(58, 1 << 8, 2), 6, mfhe.CONV_PHANTOM)
    with pytest.raises(mfhe.MfheError) as e:
        ctx.trace_product(t, t, t, t, o, o, 64, 2, 1)
    assert e.value.code == mfhe.EUNSUPPORTED
    ctx2 = mfhe.Context(RNS, 6, mfhe.CONV_PHANTOM)
    with pytest.raises(mfhe.MfheError):
        ctx2.trace_product(t, t, t, t, o, o, 32, 2, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("split", [2, 1])
@pytest.mark.parametrize("case", ["real", "imag"])
def test_trace_split_accumulator_bound_45bit(mfhe, orc, split, case):
    """Split-digit accumulators near their < 2^53 bound: 45-bit primes, operands +-(q-1)/2 with signs that make
    every digit product of the real (or imaginary) accumulators the same sign, n = 1024 (16 reduction
    intervals).  Constant planes give the exact answer analytically: C[i][j] = n * n * a * b'_j mod q."""
    import torch
    moduli = orc.gen_primes(45, 4, 2)
    ctx = mfhe.Context(moduli, 1, mfhe.CONV_PHANTOM)
    ctx.set_option(mfhe.OPT_TRACE_SPLIT, split)
    n, L, batch = 1024, 2, 1

    def plane(vals):   # vals[l] -> one constant per limb, as canonical residues
        return np.concatenate([np.full(n * n, v % q, dtype=np.uint64) for v, q in zip(vals, moduli)])
    X = [(q - 1) // 2 for q in moduli]
    a = [(x, -x) for x in X] if case == "real" else [(x, x) for x in X]
    bp = [(x, x) for x in X]
    d = [mfhe.to_device_u64(plane([v[i] for v in vals])) for vals in (a, bp) for i in (0, 1)]
    c = [torch.empty_like(d[0]), torch.empty_like(d[0])]
    ctx.trace_gemm(d[0], d[1], d[2], d[3], c[0], c[1], n, L, batch)
    torch.cuda.synchronize()
    for l, q in enumerate(moduli):
        (ar, ai), (br, bi) = a[l], bp[l]
        er, ei = n * n * (ar * br - ai * bi) % q, n * n * (ar * bi + ai * br) % q
        assert np.all(mfhe.to_host_u64(c[0]).reshape(L, -1)[l] == er)
        assert np.all(mfhe.to_host_u64(c[1]).reshape(L, -1)[l] == ei)
    # the fused product maps B -> B' itself: B' row 0 = conj(b), rows j != 0 = -i conj(b) = (-b_im, -b_re)
    if split == 2:
        b = a     # take B = a's constants; B' then has the mixed signs of the map
        db = [mfhe.to_device_u64(plane([v[i] for v in b])) for i in (0, 1)]
        ctx.trace_product(d[0], d[1], db[0], db[1], c[0], c[1], n, L, batch)
        torch.cuda.synchronize()
        for l, q in enumerate(moduli):
            (ar, ai), (br, bi) = a[l], b[l]
            hr = mfhe.to_host_u64(c[0]).reshape(L, n, n)[l]
            hi = mfhe.to_host_u64(c[1]).reshape(L, n, n)[l]
            for j, (pr, pi) in ((0, (br, -bi)), (1, (-bi, -br)), (n - 1, (-bi, -br))):
                assert np.all(hr[:, j] == n * n * (ar * pr - ai * pi) % q)
                assert np.all(hi[:, j] == n * n * (ar * pi + ai * pr) % q)
    ctx.close()


@pytest.mark.gpu
def test_trace_alternating_n_on_side_stream(mfhe, orc):
    """Calls with different n (hence different per-limb epilogue constants) queued back to back on a side
    stream with no synchronisation in between: each result must match the oracle (the constants travel in the
    kernel arguments, no shared device table is rewritten between launches)."""
    import torch
    ctx = mfhe.Context(RNS, 6, mfhe.CONV_PHANTOM)
    L, batch = 3, 2
    rng = np.random.default_rng(11)
    st = torch.cuda.Stream()
    jobs = []
    with torch.cuda.stream(st):
        for n in (64, 128, 64, 128):
            ar, ai, br, bi = (_rand(rng, batch, L, n, RNS) for _ in range(4))
            d = [mfhe.to_device_u64(x) for x in (ar, ai, br, bi)]
            c = [torch.empty_like(d[0]), torch.empty_like(d[0])]
            ctx.trace_gemm(d[0], d[1], d[2], d[3], c[0], c[1], n, L, batch, stream=st)
            jobs.append((n, (ar, ai, br, bi), c, d))
    st.synchronize()
    for n, (ar, ai, br, bi), c, _ in jobs:
        ocr, oci = orc.trace_gemm(ar, ai, br, bi, n, L, batch, RNS)
        np.testing.assert_array_equal(mfhe.to_host_u64(c[0]), ocr)
        np.testing.assert_array_equal(mfhe.to_host_u64(c[1]), oci)
    ctx.close()


@pytest.mark.gpu
def test_trace_rejects_aliasing_and_short_planes(mfhe):
    import torch
    ctx = mfhe.Context(RNS, 6, mfhe.CONV_PHANTOM)
    n, L, batch = 64, 2, 1
    p = [torch.zeros(batch * L * n * n, dtype=torch.int64, device="cuda") for _ in range(6)]
    with pytest.raises(mfhe.MfheError):      # C == A: other tiles still read A
        ctx.trace_gemm(p[0], p[1], p[2], p[3], p[0], p[5], n, L, batch)
    with pytest.raises(mfhe.MfheError):
        ctx.trace_product(p[0], p[1], p[2], p[3], p[4], p[1], n, L, batch)
    with pytest.raises(ValueError):          # undersized plane caught on the host
        ctx.trace_gemm(p[0][:100], p[1], p[2], p[3], p[4], p[5], n, L, batch)
    ctx.close()
