"""GPU parity for the W axis, the XY encoder transforms and the encode/encrypt/decrypt/decode pipelines.

Integer stages are bit-exact against the oracle (W-CRT HE.cu:716-781,1029-1114,1245-1270; samplers
HE.cu:564-627,690-713; decrypt HE.cu:1553-1601).  FP64 stages (W-DFT, XY DFT, HE.cu:1147-1172,
encoder.cu:318-326,460-501) are compared within a stated tolerance -- the reference's own FP
results depend on nvcc FMA contraction, so bit-exactness is not defined there.
End-to-end checks are the reference's own: decode(encode(x)) within 1e-3 (test_encode_decode_wcrt.cu:115),
encrypt/decrypt within 1e-3 / 1e-4 (test_encode_encrypt_decrypt_decode_wcrt.cu:109, main.cu:150).
"""
import numpy as np
import pytest

from oracle import P, U64

pytestmark = pytest.mark.gpu

RNS = [17592186435073, 17182765057, 17184541441, 17186120449, 17186515201, 17186909953,
       17188883713, 17190462721, 17190857473, 17191844353, 17192831233]
CONV = 1 | 4   # PHANTOM | WCRT
FP_TOL = 1e-9  # relative, FP64 dense transforms (K = 512 complex MACs)


@pytest.fixture(scope="module")
def small(mfhe, orc):
    n = 8
    ctx = mfhe.Context(RNS, 3, CONV)
    h = orc.HE(n, RNS, 2.0 ** 35)
    return n, ctx, h


def _dev(mfhe, a):
    return mfhe.to_device_u64(a)


def _rand_mat(rng, n, L=11):
    q = np.array(RNS[:L], np.uint64)[None, :, None]
    return (rng.integers(0, 2 ** 63, (512, L, n * n), dtype=np.uint64) % q).ravel()


def test_wcrt_fwd_inv_vector_bit_exact(mfhe, orc, small):
    import torch
    n, ctx, h = small
    rng = np.random.default_rng(0)
    x = _rand_mat(rng, n)
    out = torch.empty(x.size, dtype=torch.int64, device="cuda")
    ctx.wcrt_fwd(_dev(mfhe, x), out)
    ref = np.zeros_like(x)
    orc.L.orc_wntt_forward_matrix(P(x), P(ref), n, 11, 512, P(U64(RNS)), orc.L.orc_he_V(h.h))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mfhe.to_host_u64(out), ref)
    # inverse: poly-major eval -> matrix-major coeff; must also invert the forward exactly
    back = torch.empty_like(out)
    ctx.wcrt_inv(out, back)
    ref2 = np.zeros_like(x)
    orc.L.orc_wntt_inverse_matrix(P(ref), P(ref2), n, 11, 512, P(U64(RNS)), orc.L.orc_he_VinvT(h.h))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mfhe.to_host_u64(back), ref2)
    np.testing.assert_array_equal(ref2, x)
    # vector variant (secret-key layout)
    v = (rng.integers(0, 2 ** 63, (512, 11, n), dtype=np.uint64) % np.array(RNS, np.uint64)[None, :, None]).ravel()
    vo = torch.empty(v.size, dtype=torch.int64, device="cuda")
    ctx.wcrt_fwd_vector(_dev(mfhe, v), vo)
    vr = np.zeros_like(v)
    orc.L.orc_wntt_forward_vector(P(v), P(vr), n, 11, 512, P(U64(RNS)), orc.L.orc_he_V(h.h))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mfhe.to_host_u64(vo), vr)


def test_kat3_wcrt_basis_reference_geometry(mfhe, orc):
    """test_custom_ntt_roundtrip.cu:168-254 on the device at n = 64, L = 11."""
    import torch
    ctx = mfhe.Context(RNS, 6, CONV)
    n2 = 64 * 64
    inp = torch.zeros(512 * 11 * n2, dtype=torch.int64, device="cuda")
    inp[7 * 11 * n2] = 1
    out = torch.empty_like(inp)
    ctx.wcrt_fwd(inp, out)
    got = mfhe.to_host_u64(out)
    q = RNS[0]
    eta = orc.L.orc_find_eta(q)
    exp = orc.wcrt_exp()
    for w in range(8):
        assert int(got[((w * 64) * 11) * 64]) == pow(pow(eta, int(exp[w]), q), 7, q)


def test_wcrt_centered_matches_reference_semantics(mfhe, orc, small):
    import torch
    n, ctx, h = small
    w, y, x = np.meshgrid(np.arange(512), np.arange(n), np.arange(n), indexing="ij")
    coeff = (((w + x + y) % 17) - 8).astype(np.int64).ravel()
    ev = torch.empty(coeff.size, dtype=torch.int64, device="cuda")
    ctx.wcrt_fwd_centered(torch.from_numpy(coeff).cuda(), ev)
    ref = np.zeros_like(coeff)
    orc.L.orc_wntt_forward_centered(P(coeff), P(ref), n, 512, 11, P(U64(RNS)), orc.L.orc_he_V(h.h), h.W)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(ev.cpu().numpy(), ref)       # saturates, as the reference does
    rt = torch.empty_like(ev)
    ctx.wcrt_inv_centered(ev, rt)
    ref_rt = np.zeros_like(coeff)
    orc.L.orc_wntt_inverse_centered(P(ref), P(ref_rt), n, 512, P(U64(RNS)), orc.L.orc_he_VinvT(h.h))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(rt.cpu().numpy(), ref_rt)
    # intended semantics: exact round trip with a single limb (test_wcrt_roundtrip.cu:67-72)
    c1 = mfhe.Context(RNS[:1], 3, CONV)
    ev1 = torch.empty_like(ev)
    c1.wcrt_fwd_centered(torch.from_numpy(coeff).cuda(), ev1)
    rt1 = torch.empty_like(ev)
    c1.wcrt_inv_centered(ev1, rt1)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(rt1.cpu().numpy(), coeff)


@pytest.mark.parametrize("cgemm", [2, 3, 1, 0])
def test_wdft_and_xy_transforms_vs_oracle(mfhe, orc, small, cgemm):
    """W-DFT / XY transforms on the f64 MFMA complex GEMM with the W-DFT factored through 771 = 3 x 257 (2,
    default; 3: the XY products as two launches), dense (1), and the VALU kernel (0)."""
    n, ctx, h = small
    prev = ctx.get_option(mfhe.OPT_CGEMM_MFMA)
    ctx.set_option(mfhe.OPT_CGEMM_MFMA, cgemm)
    try:
        _wdft_and_xy_transforms(mfhe, orc, n, ctx)
    finally:
        ctx.set_option(mfhe.OPT_CGEMM_MFMA, prev)


@pytest.mark.parametrize("n", [4, 16, 64])
def test_cgemm_mfma_matches_valu(mfhe, n):
    """f64 MFMA complex GEMM (gemm.hip cgemm_mfma_kernel) vs the VALU kernel at tile-ragged and full sizes:
    XY-IDFT / XY-DFT (M = K = P = n per lane) and W-DFT / W-IDFT (M = K = 512, P = n^2), 1e-12 relative; the
    factored W-DFT (mode 2, default) too: its 256 x 256 zeta tables are single cos / sin values while the dense V
    (HE.cu:282-290) is a chain of products, so the two agree to rounding, not bit for bit.  At n = 64 mode 2 runs
    XY by 64-point FFTs (gemm.hip xy_fft_kernel, r06), equal to rounding; mode 3 runs both XY products of a lane
    in one launch (gemm.hip xy_fused_kernel): the same doubles as the two launches of mode 1, bit for bit."""
    import torch
    ctx = mfhe.Context(RNS[:2], n.bit_length() - 1, CONV)
    assert ctx.get_option(mfhe.OPT_CGEMM_MFMA) == 2
    n2 = n * n
    rng = np.random.default_rng(n)
    z = (rng.standard_normal(512 * n2) + 1j * rng.standard_normal(512 * n2)).astype(np.complex128)
    zt = torch.from_numpy(z.view(np.float64).copy()).cuda()
    outs = {}
    for mode in (2, 3, 1, 0):
        ctx.set_option(mfhe.OPT_CGEMM_MFMA, mode)
        assert ctx.get_option(mfhe.OPT_CGEMM_MFMA) == mode
        res = []
        for fn in (ctx.xy_idft, ctx.xy_dft):
            o = torch.empty_like(zt)
            fn(zt, o, 512)
            res.append(o)
        for fn in (ctx.wdft_fwd, ctx.wdft_inv):
            o = torch.empty_like(zt)
            fn(zt, o)
            res.append(o)
        torch.cuda.synchronize()
        outs[mode] = [r.cpu().numpy() for r in res]
    for mode in (2, 3, 1):
        for a, b in zip(outs[mode], outs[0]):
            assert np.max(np.abs(a - b)) <= 1e-12 * np.max(np.abs(b)), mode
    for i in range(2):
        if n == 64:   # XY: FFT (2) == GEMM (3) to rounding (the GEMMs' V is a chain of products, ~4e-14 per entry)
            assert np.max(np.abs(outs[2][i] - outs[3][i])) <= 1e-12 * np.max(np.abs(outs[3][i])), i
        else:
            np.testing.assert_array_equal(outs[2][i], outs[3][i])
        np.testing.assert_array_equal(outs[3][i], outs[1][i])   # one launch (3) == two launches (1)
    # mode 2 takes the factored W-DFT's 257-point DFTs by Rader's algorithm (gemm.hip wdft_rader_kernel and
    # wdft_rader_inv_kernel, r06), mode 3 by the GEMM: equal to rounding
    for i in range(2, 4):
        assert np.max(np.abs(outs[2][i] - outs[3][i])) <= 1e-13 * np.max(np.abs(outs[3][i])), i
    with pytest.raises(mfhe.MfheError):
        ctx.set_option(mfhe.OPT_CGEMM_MFMA, 4)


def _wdft_and_xy_transforms(mfhe, orc, n, ctx):
    import torch
    n2 = n * n
    rng = np.random.default_rng(2)
    z = (rng.standard_normal(512 * n2) + 1j * rng.standard_normal(512 * n2)).astype(np.complex128)
    zt = torch.from_numpy(z.view(np.float64).copy()).cuda()
    out = torch.empty_like(zt)
    V = np.zeros(512 * 512 * 2)
    Vi = np.zeros(512 * 512 * 2)
    assert orc.L.orc_wdft_tables(P(V), P(Vi)) == 0
    ctx.wdft_fwd(zt, out)
    ref = np.zeros(512 * n2 * 2)
    orc.L.orc_wdft_forward(P(np.ascontiguousarray(z.view(np.float64))), P(ref), P(V), n2, 512)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert np.max(np.abs(got - ref)) <= FP_TOL * np.max(np.abs(ref))
    ctx.wdft_inv(out, zt)
    torch.cuda.synchronize()
    back = zt.cpu().numpy().view(np.complex128)
    assert np.max(np.abs(back - z)) < 1e-8
    # XY: dft(idft(M)) == M, and idft == oracle Vinv M Vinv^T
    M = (rng.standard_normal(512 * n2) + 1j * rng.standard_normal(512 * n2)).astype(np.complex128)
    mt = torch.from_numpy(M.view(np.float64).copy()).cuda()
    pt = torch.empty_like(mt)
    ctx.xy_idft(mt, pt, 512)
    encV, encVT, encVi, encViT = (np.zeros(n2 * 2) for _ in range(4))
    orc.L.orc_encoder_matrices(n, P(encV), P(encVT), P(encVi), P(encViT))
    T = np.zeros(n2 * 2)
    R = np.zeros(n2 * 2)
    for ell in (0, 511):
        mm = np.ascontiguousarray(M[ell * n2:(ell + 1) * n2].view(np.float64))
        orc.L.orc_cmatmul(P(encVi), P(mm), P(T), n)
        orc.L.orc_cmatmul(P(T), P(encViT), P(R), n)
        g = pt.cpu().numpy()[ell * n2 * 2:(ell + 1) * n2 * 2]
        assert np.max(np.abs(g - R)) < 1e-12 * max(1.0, np.max(np.abs(R)))
    mt2 = torch.empty_like(mt)
    ctx.xy_dft(pt, mt2, 512)
    torch.cuda.synchronize()
    assert np.max(np.abs(mt2.cpu().numpy().view(np.complex128) - M)) < 1e-10


def test_wdft_pair_entry_points(mfhe, orc, small):
    """wdft_forward_centered_pair / wdft_inverse_pair (HE.cu:472-502, 1116-1145, 1174-1202): planar re/im."""
    import torch
    n, ctx, h = small
    n2 = n * n
    rng = np.random.default_rng(5)
    re = rng.integers(-2 ** 40, 2 ** 40, 512 * n2, dtype=np.int64)
    im = rng.integers(-2 ** 40, 2 ** 40, 512 * n2, dtype=np.int64)
    V = np.zeros(512 * 512 * 2)
    Vi = np.zeros(512 * 512 * 2)
    assert orc.L.orc_wdft_tables(P(V), P(Vi)) == 0
    z = (re.astype(np.float64) + 1j * im.astype(np.float64)).astype(np.complex128)
    ref = np.zeros(512 * n2 * 2)
    orc.L.orc_wdft_forward(P(np.ascontiguousarray(z.view(np.float64))), P(ref), P(V), n2, 512)
    ref = ref.view(np.complex128)
    ore = torch.empty(512 * n2, dtype=torch.float64, device="cuda")
    oim = torch.empty_like(ore)
    ctx.wdft_fwd_pair_i64(torch.from_numpy(re).cuda(), torch.from_numpy(im).cuda(), ore, oim)
    torch.cuda.synchronize()
    scale = np.max(np.abs(ref))
    assert np.max(np.abs(ore.cpu().numpy() - ref.real)) <= FP_TOL * scale
    assert np.max(np.abs(oim.cpu().numpy() - ref.imag)) <= FP_TOL * scale
    bre = torch.empty_like(ore)
    bim = torch.empty_like(ore)
    ctx.wdft_inv_pair(ore, oim, bre, bim)
    torch.cuda.synchronize()
    assert np.max(np.abs(bre.cpu().numpy() - re)) < 1e-9 * 2 ** 40
    assert np.max(np.abs(bim.cpu().numpy() - im)) < 1e-9 * 2 ** 40


def test_ct_add_and_mul_tensor_bit_exact(mfhe, small):
    """add_ciphertexts / multiply_ciphertexts_raw (HE.cu:631-669, 1710-1740) on matrix-major [b | a]."""
    import torch
    n, ctx, h = small
    rng = np.random.default_rng(6)
    c1 = np.concatenate([_rand_mat(rng, n), _rand_mat(rng, n)])
    c2 = np.concatenate([_rand_mat(rng, n), _rand_mat(rng, n)])
    half = c1.size // 2
    q = np.broadcast_to(np.array(RNS, np.uint64)[None, :, None], (512, 11, n * n)).ravel()
    res = torch.empty(c1.size, dtype=torch.int64, device="cuda")
    ctx.ct_add(_dev(mfhe, c1), _dev(mfhe, c2), res)
    qq = np.concatenate([q, q])
    s = c1 + c2
    np.testing.assert_array_equal(mfhe.to_host_u64(res), np.where(s >= qq, s - qq, s))
    d = [torch.empty(half, dtype=torch.int64, device="cuda") for _ in range(3)]
    ctx.ct_mul_tensor(_dev(mfhe, c1), _dev(mfhe, c2), *d)
    torch.cuda.synchronize()
    O = lambda a: a.astype(object)
    b1, a1, b2, a2, qo = O(c1[:half]), O(c1[half:]), O(c2[:half]), O(c2[half:]), O(q)
    want = [(b1 * b2) % qo, (b1 * a2 + a1 * b2) % qo, (a1 * a2) % qo]
    for got, w in zip(d, want):
        np.testing.assert_array_equal(mfhe.to_host_u64(got), w.astype(np.uint64))


def test_keygen_bit_exact_reference_geometry(mfhe, orc):
    """generate_secret_key (HE.cu:1272-1307): ternary s -> W-CRT -> X-NTT; no floating point -> exact."""
    import torch
    ctx = mfhe.Context(RNS, 6, CONV)
    sk = torch.empty(512 * 11 * 64, dtype=torch.int64, device="cuda")
    ctx.keygen(sk)
    h = orc.HE(64, RNS, 2.0 ** 35)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mfhe.to_host_u64(sk), h.keygen())


def test_encrypt_decrypt_vs_oracle(mfhe, orc, small):
    n, ctx, h = small
    _encrypt_decrypt_vs_oracle(mfhe, orc, n, ctx, h, RNS)


def test_encrypt_decrypt_vs_oracle_c4_moduli(mfhe, orc):
    """The same bit-exact check with BASELINE C4's parameter set (test_encode_encrypt_decrypt_decode_wcrt.cu:29-110):
    L = 16 primes of 35 bits, q = 1 mod 2^8 * 771, at small n."""
    from bench import gen_moduli
    moduli = gen_moduli(35, 197376, 16)
    n = 8
    ctx = mfhe.Context(moduli, 3, CONV)
    h = orc.HE(n, moduli, 2.0 ** 35)
    _encrypt_decrypt_vs_oracle(mfhe, orc, n, ctx, h, moduli)
    ctx.close()


def _encrypt_decrypt_vs_oracle(mfhe, orc, n, ctx, h, moduli):
    import torch
    Lq = len(moduli)
    words = 512 * Lq * n * n
    rng = np.random.default_rng(3)
    qm = np.array(moduli, np.uint64)[None, :, None]
    m_re, m_im = ((rng.integers(0, 2 ** 63, (512, Lq, n * n), dtype=np.uint64) % qm).ravel() for _ in range(2))
    sk_ref = h.keygen()
    sk = torch.empty(512 * Lq * n, dtype=torch.int64, device="cuda")
    ctx.keygen(sk)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mfhe.to_host_u64(sk), sk_ref)
    cre = torch.empty(2 * words, dtype=torch.int64, device="cuda")
    cim = torch.empty_like(cre)
    ctx.encrypt_pair(_dev(mfhe, m_re), _dev(mfhe, m_im), sk, cre, cim)
    ore, oim = h.encrypt_pair(m_re, m_im, sk_ref)
    torch.cuda.synchronize()
    gre, gim = mfhe.to_host_u64(cre), mfhe.to_host_u64(cim)
    np.testing.assert_array_equal(gre[words:], ore[words:])           # a: uniform sampler + W-CRT, exact
    np.testing.assert_array_equal(gim[words:], oim[words:])
    # b contains the Box-Muller Gaussian (device libm vs glibc may differ in the last ulp of log/cos,
    # which can move llround at a .5 boundary): require >= 99.999 % exact agreement
    assert np.mean(gre[:words] != ore[:words]) < 1e-5
    assert np.mean(gim[:words] != oim[:words]) < 1e-5
    # ... and exactly: b differs from the oracle's only by the W-CRT image of a noise difference (b is linear in
    # e), so the oracle's inverse W-CRT of (b_dev - b_orc) must be a noise difference in {-1, 0, +1}, the same
    # integer in every limb, nonzero only where the unrounded Box-Muller sample sits on a .5 rounding boundary
    # (HE.cu:605-627: the only step where device libm and glibc may differ)
    n2 = n * n
    q_el = np.array(moduli, dtype=object)[(np.arange(words) // n2) % Lq]
    q3 = np.array(moduli, np.uint64)[None, :, None]
    noise = []
    for got, want in ((gre, ore), (gim, oim)):
        d = ((got[:words].astype(object) - want[:words].astype(object)) % q_el).astype(np.uint64)
        poly, de = np.zeros_like(d), np.zeros_like(d)
        orc.L.orc_matrix_to_poly(P(d), P(poly), n, Lq, 512)
        orc.L.orc_wntt_inverse_matrix(P(poly), P(de), n, Lq, 512, P(U64(moduli)), orc.L.orc_he_VinvT(h.h))
        de = de.reshape(512, Lq, n2)
        sgn = np.where(de == 0, 0, np.where(de == 1, 1, np.where(de == q3 - 1, -1, 99)))
        assert (sgn != 99).all(), "ciphertexts differ by more than a +-1 noise step"
        assert (sgn == sgn[:, :1, :]).all(), "noise difference not the same integer in every limb"
        noise.append(sgn[:, 0, :])
    np.testing.assert_array_equal(noise[0], noise[1])   # re and im share e (HE.cu:605-608)
    for w, pos in zip(*np.nonzero(noise[0])):
        r1 = orc.L.orc_splitmix64(0xD6E8FEB86659FD93 ^ int(w * n2 + pos))
        r2 = orc.L.orc_splitmix64(r1)
        u1 = ((r1 >> 11) + 1.0) / 9007199254740992.0
        u2 = ((r2 >> 11) + 1.0) / 9007199254740992.0
        z = 3.2 * np.sqrt(-2.0 * np.log(u1)) * np.cos(6.283185307179586 * u2)
        assert abs(abs(z) % 1.0 - 0.5) < 1e-9, (w, pos, z)
    # decrypt on identical inputs is exact
    ev = torch.empty(words, dtype=torch.int64, device="cuda")
    ctx.decrypt_to_eval(cre, sk, ev)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mfhe.to_host_u64(ev), h.decrypt_to_eval(gre, sk_ref))


@pytest.mark.parametrize("n,L", [(8, 11), (16, 3), (64, 11), (64, 1), (8, 16), (64, 16)])
def test_encrypt_noise_small_operand_gemm_matches_factored(mfhe, n, L):
    """MFHE_OPT_ENC_E_SMALL (r06): the encrypt's Gaussian noise enters its W-CRT forward as the dense product with its
    one signed digit (|e| <= 27 from the Box-Muller bound) and is never written as residues.  1 (default): gemm.hip
    mod_gemm_mfma_smallb_kernel, 64 x 128 tiles where n^2 % 128 == 0, else 64 x 64; 0: the factored forward of its
    residues.  The ciphertexts are identical, for limbs of 5 and 6 digits (the reference moduli: limb 0 has 44
    bits), one limb, and BASELINE C4's 16 x 35-bit primes; with a through both ciphertexts (ENC_A_DIRECT 1) or through
    the poly-major buffer (0); for encrypt_pair and encrypt; and identical to the pair launch (HE_STREAMS 2), which
    keeps the factored form."""
    import torch
    from bench import gen_moduli
    moduli = RNS[:L] if L <= 11 else gen_moduli(35, 197376, L)
    ctx = mfhe.Context(moduli, n.bit_length() - 1, CONV)
    assert ctx.get_option(mfhe.OPT_ENC_E_SMALL) == 1
    words = 512 * L * n * n
    rng = np.random.default_rng(n * 7 + L)
    qm = np.array(moduli, np.uint64)[None, :, None]
    m_re, m_im = (_dev(mfhe, (rng.integers(0, 2 ** 63, (512, L, n * n), dtype=np.uint64) % qm).ravel())
                  for _ in range(2))
    sk = torch.empty(512 * L * n, dtype=torch.int64, device="cuda")
    ctx.keygen(sk)
    out, single = {}, {}
    for small, streams, adirect in ((1, 3, 1), (0, 3, 1), (1, 3, 0), (1, 2, 1), (1, 0, 1)):
        ctx.set_option(mfhe.OPT_ENC_E_SMALL, small)
        ctx.set_option(mfhe.OPT_HE_STREAMS, streams)
        ctx.set_option(mfhe.OPT_ENC_A_DIRECT, adirect)
        cre = torch.full((2 * words,), -1, dtype=torch.int64, device="cuda")
        cim = torch.full_like(cre, -1)
        ctx.encrypt_pair(m_re, m_im, sk, cre, cim)
        torch.cuda.synchronize()
        out[(small, streams, adirect)] = (mfhe.to_host_u64(cre), mfhe.to_host_u64(cim))
        if streams == 3 and adirect == 1:
            ct = torch.full((2 * words,), -1, dtype=torch.int64, device="cuda")
            ctx.encrypt(m_re, sk, ct)
            torch.cuda.synchronize()
            single[small] = mfhe.to_host_u64(ct)
    ref = out[(0, 3, 1)]
    for key, (a, b) in out.items():
        np.testing.assert_array_equal(a, ref[0], err_msg=str(key))
        np.testing.assert_array_equal(b, ref[1], err_msg=str(key))
    for small, ct in single.items():
        np.testing.assert_array_equal(ct, single[0], err_msg=f"encrypt, option {small}")
    with pytest.raises(mfhe.MfheError):
        ctx.set_option(mfhe.OPT_ENC_E_SMALL, 2)
    ctx.close()


@pytest.mark.parametrize("n,L", [(4, 2), (8, 11), (16, 3), (64, 11)])
def test_fused_ring_matches_unfused(mfhe, n, L):
    """encrypt_pair / decrypt_to_eval with the fused X-NTT * s * X-INTT row kernels (he.hip enc_ring_kernel,
    dec_ring_kernel; MFHE_OPT_HE_FUSED = 1, default) == the separate NTT / pointwise / combine kernels, bit-exact.
    decrypt_and_decode too: at n = 64 the fused path decrypts inside the inverse W-CRT's digitize (gemm.hip
    mfma_digitize_ifold_dec_kernel), the unfused one through decrypt_to_eval and the plain digitize.  r05: the fused
    encrypt with the shared a written into both ciphertexts by the W-CRT GEMM (MFHE_OPT_ENC_A_DIRECT 1, default) and
    decode's re / im chains on two streams (MFHE_OPT_HE_STREAMS 1, default) against both off."""
    import torch
    ctx = mfhe.Context(RNS[:L], n.bit_length() - 1, CONV)
    assert ctx.get_option(mfhe.OPT_HE_FUSED) == 1
    assert ctx.get_option(mfhe.OPT_ENC_A_DIRECT) == 1 and ctx.get_option(mfhe.OPT_HE_STREAMS) == 3
    words = 512 * L * n * n
    rng = np.random.default_rng(n + L)
    m_re, m_im = _rand_mat(rng, n, L), _rand_mat(rng, n, L)
    sk = torch.empty(512 * L * n, dtype=torch.int64, device="cuda")
    ctx.keygen(sk)
    res = {}
    for mode, direct, streams in ((1, 1, 1), (1, 0, 0), (0, 1, 1), (1, 1, 2)):
        ctx.set_option(mfhe.OPT_HE_FUSED, mode)
        ctx.set_option(mfhe.OPT_ENC_A_DIRECT, direct)
        ctx.set_option(mfhe.OPT_HE_STREAMS, streams)
        mode = (mode, direct) if streams != 2 else (mode, direct, 2)
        cre = torch.empty(2 * words, dtype=torch.int64, device="cuda")
        cim = torch.empty_like(cre)
        ctx.encrypt_pair(_dev(mfhe, m_re), _dev(mfhe, m_im), sk, cre, cim)
        ev = torch.empty(words, dtype=torch.int64, device="cuda")
        ctx.decrypt_to_eval(cre, sk, ev)
        msg = torch.empty(2 * 512 * n * n, dtype=torch.float64, device="cuda")
        ctx.decrypt_and_decode(cre, cim, sk, msg)
        torch.cuda.synchronize()
        res[mode] = [mfhe.to_host_u64(t) for t in (cre, cim, ev)] + [msg.cpu().numpy()]
    for other in ((1, 0), (0, 1), (1, 1, 2)):
        for a, b in zip(res[(1, 1)], res[other]):
            np.testing.assert_array_equal(a, b)
    # decrypt(encrypt(m)) = m + e: small noise around the message in the coefficient domain is checked by
    # the KAT pipelines; here the eval-domain result must differ from m_re (the encryption is not trivial)
    assert np.mean(res[(1, 1)][2] != m_re) > 0.5


def test_encode_stages_and_decode_vs_oracle(mfhe, orc, small):
    """encode_to_wntt_eval stage by stage: FP64 XY-IDFT and W-IDFT within tolerance of the oracle; the
    integer stage (quantize + RNS split + W-CRT, batched_encoder.cu:125-152 + HE.cu:716-747) bit-exact
    from identical doubles.  (End to end, one FP64 rounding difference before llround changes one
    coefficient, which the W-CRT spreads over a whole column -- tolerance parity only, SURVEY.md §8c.
    The default f64 MFMA GEMM sums in its own order, so its encode is checked bit-exact against the
    integer stage on its own doubles; the oracle-order VALU GEMM is checked against the oracle.)"""
    import torch
    n, ctx, h = small
    n2 = n * n
    ell, i = np.meshgrid(np.arange(512), np.arange(n2), indexing="ij")
    val = (ell * 10000 + i).astype(np.float64).ravel()
    msg = (val - 1j * val).astype(np.complex128)
    mt = torch.from_numpy(msg.view(np.float64).copy()).cuda()
    # oracle stages
    encV, encVT, encVi, encViT = (np.zeros(n2 * 2) for _ in range(4))
    orc.L.orc_encoder_matrices(n, P(encV), P(encVT), P(encVi), P(encViT))
    V = np.zeros(512 * 512 * 2)
    Vi = np.zeros(512 * 512 * 2)
    assert orc.L.orc_wdft_tables(P(V), P(Vi)) == 0
    xy = np.zeros(512 * n2 * 2)
    T = np.zeros(n2 * 2)
    m64 = np.ascontiguousarray(msg.view(np.float64))
    for l_ in range(512):
        orc.L.orc_cmatmul(P(encVi), P(m64[l_ * n2 * 2:]), P(T), n)
        R = np.zeros(n2 * 2)
        orc.L.orc_cmatmul(P(T), P(encViT), P(R), n)
        xy[l_ * n2 * 2:(l_ + 1) * n2 * 2] = R
    wc = np.zeros_like(xy)
    orc.L.orc_w_idft(P(xy), P(wc), P(Vi), n2, 512)
    # device stages
    gxy = torch.empty_like(mt)
    ctx.xy_idft(mt, gxy, 512)
    gwc = torch.empty_like(mt)
    ctx.wdft_inv(gxy, gwc)
    torch.cuda.synchronize()
    assert np.max(np.abs(gxy.cpu().numpy() - xy)) <= 1e-12 * np.max(np.abs(xy))
    assert np.max(np.abs(gwc.cpu().numpy() - wc)) <= FP_TOL * np.max(np.abs(wc))
    # integer stage from the oracle's doubles: bit-exact with the oracle's encoder output
    ore, oim = h.encode(msg)
    wct = torch.from_numpy(wc).cuda()
    words = 512 * 11 * n2
    cre = torch.empty(words, dtype=torch.int64, device="cuda")
    ev = torch.empty_like(cre)
    out = torch.empty_like(cre)
    for part, ref in ((0, ore), (1, oim)):
        ctx.rns_decompose(wct[part:], cre, 512, n2, in_stride=2)
        ctx.wcrt_fwd(cre, ev)
        ctx.poly_to_matrix(ev, out)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(mfhe.to_host_u64(out), ref)
    # full device encode == the integer stage run on the device's own W-IDFT doubles, bit-exact
    gre = torch.empty(words, dtype=torch.int64, device="cuda")
    gim = torch.empty_like(gre)
    ctx.encode(mt, gre, gim)
    for part, got in ((0, gre), (1, gim)):
        ctx.rns_decompose(gwc[part:], cre, 512, n2, in_stride=2)
        ctx.wcrt_fwd(cre, ev)
        ctx.poly_to_matrix(ev, out)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(mfhe.to_host_u64(out), mfhe.to_host_u64(got))
    # vs the oracle: with the VALU GEMM (the oracle's mul-then-add term order) the integer outputs are
    # equal except in at most 2 columns where llround saw a different double
    prev = ctx.get_option(mfhe.OPT_CGEMM_MFMA)
    ctx.set_option(mfhe.OPT_CGEMM_MFMA, 0)
    try:
        ctx.encode(mt, gre, gim)
        torch.cuda.synchronize()
    finally:
        ctx.set_option(mfhe.OPT_CGEMM_MFMA, prev)
    diff_cols = np.any((mfhe.to_host_u64(gre) != ore).reshape(512, 11, n2), axis=(0, 1))
    assert diff_cols.sum() <= 2
    # decode of the oracle's encoding vs the oracle's decode, and the reference 1e-3 bound
    pre = np.zeros_like(ore)
    pim = np.zeros_like(oim)
    orc.L.orc_matrix_to_poly(P(ore), P(pre), n, 11, 512)
    orc.L.orc_matrix_to_poly(P(oim), P(pim), n, 11, 512)
    dout = torch.empty_like(mt)
    ctx.decode(_dev(mfhe, pre), _dev(mfhe, pim), dout)
    ref = h.decode(pre, pim)
    torch.cuda.synchronize()
    got = dout.cpu().numpy().view(np.complex128)
    # FP64 stages: relative to the values (|msg| ~ 5e6 here).  The default W-DFT is factored (gemm.hip) with
    # tables from single cos / sin values, the oracle's is the reference's dense chain-of-products V
    # (HE.cu:282-290): they agree to a few 1e-13 relative, not to 1e-6 absolute on 5e6 (the dense MFMA: 2e-13)
    assert np.max(np.abs(got - ref)) < 1e-12 * np.max(np.abs(ref))
    assert np.max(np.abs(got - msg)) < 1e-3


def _ref_geometry_msg(pattern):
    n2 = 64 * 64
    ell, i = np.meshgrid(np.arange(512), np.arange(n2), indexing="ij")
    if pattern == "encode_decode":      # test_encode_decode_wcrt.cu:40-45
        v = (ell * 10000 + i).astype(np.float64)
        return (v - 1j * v).ravel()
    if pattern == "enc_dec":            # test_encode_encrypt_decrypt_decode_wcrt.cu:46-51
        v = ell + i * 0.001
        return (v - 1j * v).ravel()
    # main.cu:62-69
    return ((ell + i * 1e-5) + 1j * (ell - i * 1e-5)).ravel()


def test_he_streams_encode_decode_identical(mfhe):
    """MFHE_OPT_HE_STREAMS: encode's re / im W-CRT chains and decode's W-INTT + compose chains on two streams
    (1: side chain with its own digit planes and coefficient buffer) or as one launch per step with grids over both
    components (2: gemm.hip launch_mod_gemm_pair, the pair kernels) give the same words / doubles as one plain stream
    (0), at the reference geometry, called back to back."""
    import torch
    ctx = mfhe.Context(RNS, 6, CONV)
    ctx.reserve_workspace()
    msg = _ref_geometry_msg("encode_decode")
    mt = torch.from_numpy(msg.view(np.float64).copy()).cuda()
    words = 512 * 11 * 4096
    out = {}
    for streams in (1, 2, 3, 0):
        ctx.set_option(mfhe.OPT_HE_STREAMS, streams)
        re_ = torch.empty(words, dtype=torch.int64, device="cuda")
        im_ = torch.empty_like(re_)
        pre, pim = torch.empty_like(re_), torch.empty_like(re_)
        dec = torch.empty_like(mt)
        for _ in range(3):
            ctx.encode(mt, re_, im_)
            ctx.matrix_to_poly(re_, pre)
            ctx.matrix_to_poly(im_, pim)
            ctx.decode(pre, pim, dec)
        torch.cuda.synchronize()
        out[streams] = (mfhe.to_host_u64(re_), mfhe.to_host_u64(im_), dec.cpu().numpy())
    for other in (2, 3, 0):
        for a, b in zip(out[1], out[other]):
            np.testing.assert_array_equal(a, b)
    assert np.max(np.abs(out[1][2].view(np.complex128) - msg)) < 1e-3


@pytest.mark.parametrize("case", ["random", "extreme"])
def test_decrypt_and_decode_stream_modes_agree_on_any_words(mfhe, case):
    """decrypt_and_decode (the decrypt fused into the inverse W-CRT digitize) gives the same doubles with the decode's
    re / im on one stream (HE_STREAMS 0), as a pair launch (2) and on the side stream (3), at the reference geometry,
    for random residues in every ciphertext word and key word (not only keygen's keys) and for all-(q - 1) / zero
    words.  MFHE_OPT_DEC_MM (the ring product on the matrix cores, r05: 2.4x slower) was removed in r06: only 0 is
    accepted."""
    import torch
    ctx = mfhe.Context(RNS, 6, CONV)
    ctx.reserve_workspace()
    assert ctx.get_option(mfhe.OPT_DEC_MM) == 0
    ctx.set_option(mfhe.OPT_DEC_MM, 0)
    with pytest.raises(mfhe.MfheError):
        ctx.set_option(mfhe.OPT_DEC_MM, 1)
    rng = np.random.default_rng(11)
    q = np.array(RNS, np.uint64)[None, :, None]
    if case == "random":
        cre = _rand_mat(rng, 64)
        cre = np.concatenate([cre, _rand_mat(rng, 64)])
        cim = np.concatenate([_rand_mat(rng, 64), _rand_mat(rng, 64)])
        sk = (rng.integers(0, 2 ** 63, (512, 11, 64), dtype=np.uint64) % q).ravel()
    else:
        full = np.broadcast_to(q - 1, (512, 11, 4096)).ravel()
        cre = np.concatenate([full, full])
        cim = np.concatenate([np.zeros_like(full), full])
        sk = np.broadcast_to(q - 1, (512, 11, 64)).ravel().copy()
    dcre, dcim, dsk = (mfhe.to_device_u64(np.ascontiguousarray(x)) for x in (cre, cim, sk))
    out = {}
    for streams in (0, 2, 3):
        ctx.set_option(mfhe.OPT_HE_STREAMS, streams)
        res = torch.empty(512 * 4096 * 2, dtype=torch.float64, device="cuda")
        ctx.decrypt_and_decode(dcre, dcim, dsk, res)
        torch.cuda.synchronize()
        out[streams] = res.cpu().numpy()
    ref = out[0]
    assert np.all(np.isfinite(ref))
    for k, v in out.items():
        np.testing.assert_array_equal(v, ref, err_msg=str(k))


def test_pipeline_graph_capture_replays_identically(mfhe):
    """encode -> encrypt_pair -> decrypt_and_decode captured into one HIP graph (torch.cuda.CUDAGraph) after
    mfhe_ctx_reserve_workspace: the side stream of MFHE_OPT_HE_STREAMS joins the capture through its fork / join
    events and nothing allocates, so the replay writes the same words and doubles as the eager calls."""
    import torch
    ctx = mfhe.Context(RNS, 6, CONV)
    ctx.reserve_workspace()
    msg = _ref_geometry_msg("encode_decode")
    mt = torch.from_numpy(msg.view(np.float64).copy()).cuda()
    words = 512 * 11 * 4096
    sk = torch.empty(512 * 11 * 64, dtype=torch.int64, device="cuda")
    ctx.keygen(sk)
    bufs = [torch.empty(words, dtype=torch.int64, device="cuda") for _ in range(2)]
    cts = [torch.empty(2 * words, dtype=torch.int64, device="cuda") for _ in range(2)]
    out = torch.empty_like(mt)

    def run():
        ctx.encode(mt, bufs[0], bufs[1])
        ctx.encrypt_pair(bufs[0], bufs[1], sk, cts[0], cts[1])
        ctx.decrypt_and_decode(cts[0], cts[1], sk, out)

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        run()   # warm-up on the capture stream (lazy tables, launch attributes)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    eager = [mfhe.to_host_u64(t) for t in cts] + [out.cpu().numpy()]
    for t in cts:
        t.zero_()
    out.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        run()
    g.replay()
    torch.cuda.synchronize()
    got = [mfhe.to_host_u64(t) for t in cts] + [out.cpu().numpy()]
    for a, b in zip(eager, got):
        np.testing.assert_array_equal(a, b)
    assert np.max(np.abs(got[2].view(np.complex128) - msg)) < 1e-3


def test_kat6_encode_decode_reference_geometry(mfhe):
    """test_encode_decode_wcrt.cu at full reference geometry (n=64, phi=512, L=11): s = 0, a = 0."""
    import torch
    ctx = mfhe.Context(RNS, 6, CONV)
    ctx.reserve_workspace()
    msg = _ref_geometry_msg("encode_decode")
    mt = torch.from_numpy(msg.view(np.float64).copy()).cuda()
    words = 512 * 11 * 4096
    re_ = torch.empty(words, dtype=torch.int64, device="cuda")
    im_ = torch.empty_like(re_)
    ctx.encode(mt, re_, im_)
    # decrypt_and_decode with a = 0 and s = 0 reduces to decode(matrix_to_poly(b))
    pre, pim = torch.empty_like(re_), torch.empty_like(re_)
    ctx.matrix_to_poly(re_, pre)
    ctx.matrix_to_poly(im_, pim)
    out = torch.empty_like(mt)
    ctx.decode(pre, pim, out)
    torch.cuda.synchronize()
    err = np.max(np.abs(out.cpu().numpy().view(np.complex128) - msg))
    assert err < 1e-3, err
    # the full decrypt_and_decode path with a zero key gives the same answer
    ct_re = torch.cat([re_, torch.zeros_like(re_)])
    ct_im = torch.cat([im_, torch.zeros_like(im_)])
    sk0 = torch.zeros(512 * 11 * 64, dtype=torch.int64, device="cuda")
    out2 = torch.empty_like(mt)
    ctx.decrypt_and_decode(ct_re, ct_im, sk0, out2)
    torch.cuda.synchronize()
    assert torch.equal(out, out2)


@pytest.mark.parametrize("pattern,tol", [("enc_dec", 1e-3), ("main", 1e-4)])
def test_kat7_kat8_encrypt_decrypt_reference_geometry(mfhe, pattern, tol):
    """test_encode_encrypt_decrypt_decode_wcrt.cu (< 1e-3) and main.cu (< 1e-4) at n=64, L=11."""
    import torch
    ctx = mfhe.Context(RNS, 6, CONV)
    ctx.reserve_workspace()
    sk = torch.empty(512 * 11 * 64, dtype=torch.int64, device="cuda")
    ctx.keygen(sk)
    msg = _ref_geometry_msg(pattern)
    mt = torch.from_numpy(msg.view(np.float64).copy()).cuda()
    words = 512 * 11 * 4096
    re_ = torch.empty(words, dtype=torch.int64, device="cuda")
    im_ = torch.empty_like(re_)
    ctx.encode(mt, re_, im_)
    cre = torch.empty(2 * words, dtype=torch.int64, device="cuda")
    cim = torch.empty_like(cre)
    ctx.encrypt_pair(re_, im_, sk, cre, cim)
    out = torch.empty_like(mt)
    ctx.decrypt_and_decode(cre, cim, sk, out)
    torch.cuda.synchronize()
    err = np.max(np.abs(out.cpu().numpy().view(np.complex128) - msg))
    assert err < tol, err


@pytest.mark.parametrize("n,L", [(8, 11), (64, 11), (4, 2), (16, 1)])
def test_wcrt_mfma_matches_valu_and_oracle(mfhe, orc, n, L):
    """W-CRT GEMM on i8 MFMA (digit-split exact product, gemm.hip) == the u128 VALU kernel == oracle,
    all three layouts (matrix->poly, poly->matrix, vector), bit-exact.  Modes: 1 = LDS-staged with the
    forward factored through 771 = 3 x 257 (default), 3 = LDS-staged dense, 2 = global fragments, 0 = VALU; the
    LDS-staged modes under each K pipeline (MFHE_OPT_WCRT_PIPE 0: auto, 1: two 64-k stages, 2: 4-slot 32-k ring,
    3: ring with one-ahead A-fragment reads)."""
    import torch
    log_n = n.bit_length() - 1
    ctx = mfhe.Context(RNS[:L], log_n, CONV)
    assert ctx.get_option(mfhe.OPT_WCRT_MFMA) == 1
    rng = np.random.default_rng(n * 100 + L)
    x = _rand_mat(rng, n, L)
    outs = {}
    modes = [(1, 0), (1, 1), (1, 2), (1, 3), (3, 0), (3, 1), (3, 2), (3, 3), (2, 0), (0, 0)]
    for mf, pipe in modes:
        ctx.set_option(mfhe.OPT_WCRT_MFMA, mf)
        ctx.set_option(mfhe.OPT_WCRT_PIPE, pipe)
        d = _dev(mfhe, x)
        f = torch.empty_like(d)
        ctx.wcrt_fwd(d, f)
        b = torch.empty_like(d)
        ctx.wcrt_inv(f, b)
        v = (rng.integers(0, 2 ** 63, (512, L, n), dtype=np.uint64) % np.array(RNS[:L], np.uint64)[None, :, None]).ravel()
        vo = torch.empty(v.size, dtype=torch.int64, device="cuda")
        ctx.wcrt_fwd_vector(_dev(mfhe, v), vo)
        torch.cuda.synchronize()
        outs[mf, pipe] = (mfhe.to_host_u64(f), mfhe.to_host_u64(b), mfhe.to_host_u64(vo))
        np.testing.assert_array_equal(outs[mf, pipe][1], x)
        rng = np.random.default_rng(n * 100 + L)   # same vector input for both runs
        _rand_mat(rng, n, L)
    for key in modes[:-1]:
        for a, b in zip(outs[key], outs[0, 0]):
            np.testing.assert_array_equal(a, b)
    if n <= 8:
        h = orc.HE(n, RNS[:L], 2.0 ** 35)
        ref = np.zeros_like(x)
        orc.L.orc_wntt_forward_matrix(P(x), P(ref), n, L, 512, P(U64(RNS[:L])), orc.L.orc_he_V(h.h))
        np.testing.assert_array_equal(outs[1, 0][0], ref)


@pytest.mark.parametrize("kind", ["constant", "random"])
def test_encode_quantize_near_int64_limit(mfhe, small, kind):
    """The encode's quantization (llround(v * delta), batched_encoder.cu:125-152) runs fused into the W-CRT digitize
    (MFHE_OPT_WCRT_MFMA 1, default: an exact FP64 centred reduction of round(v * delta)) or as rns_decompose's
    int64 llround + the dense GEMM (mode 3).  Both are exact on the reference's llround range |v * delta| < 2^63
    (mfhe.h mfhe_encode); here with values up to 2^62.9 / delta (a constant message lands as one coefficient of
    that size per lane) they agree bit for bit."""
    import torch
    n, ctx, h = small
    n2 = n * n
    rng = np.random.default_rng(11)
    big = 2.0 ** 62.9 / 2.0 ** 35
    if kind == "constant":
        msg = np.full(512 * n2, big * (1 - 1j), np.complex128)
    else:
        msg = (rng.uniform(-big, big, 512 * n2) + 1j * rng.uniform(-big, big, 512 * n2)) / 4
    mt = torch.from_numpy(msg.view(np.float64).copy()).cuda()
    words = 512 * 11 * n2
    outs = {}
    prev = ctx.get_option(mfhe.OPT_WCRT_MFMA)
    try:
        for mf in (1, 3, 0):
            ctx.set_option(mfhe.OPT_WCRT_MFMA, mf)
            re_ = torch.empty(words, dtype=torch.int64, device="cuda")
            im_ = torch.empty_like(re_)
            ctx.encode(mt, re_, im_)
            torch.cuda.synchronize()
            outs[mf] = (mfhe.to_host_u64(re_), mfhe.to_host_u64(im_))
    finally:
        ctx.set_option(mfhe.OPT_WCRT_MFMA, prev)
    for mf in (3, 0):
        np.testing.assert_array_equal(outs[1][0], outs[mf][0])
        np.testing.assert_array_equal(outs[1][1], outs[mf][1])


@pytest.mark.parametrize("n,log_n,L", [(8, 3, 11), (64, 6, 11), (16, 4, 3)])
def test_layout_transforms_vs_oracle(mfhe, orc, n, log_n, L):
    """matrix_to_poly_kernel / poly_to_matrix_kernel (HE.cu:1330-1368): matrix-major [phi][L][n*n] <->
    poly-major [phi*n][L][n], standalone, bit-exact against the oracle in both directions, and a round trip."""
    import torch
    ctx = mfhe.Context(RNS[:L], log_n, CONV)
    x = _rand_mat(np.random.default_rng(n + L), n, L)
    ref = np.empty_like(x)
    orc.L.orc_matrix_to_poly(P(x), P(ref), n, L, 512)
    got = torch.empty(x.size, dtype=torch.int64, device="cuda")
    ctx.matrix_to_poly(_dev(mfhe, x), got)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mfhe.to_host_u64(got), ref)
    back_ref = np.empty_like(x)
    orc.L.orc_poly_to_matrix(P(ref), P(back_ref), n, L, 512)
    np.testing.assert_array_equal(back_ref, x)
    back = torch.empty_like(got)
    ctx.poly_to_matrix(got, back)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mfhe.to_host_u64(back), x)


def test_he_wrappers_reject_undersized_buffers(mfhe, small):
    """The Python layer checks every fixed-geometry buffer (phi = 512 lanes) before a raw pointer crosses the
    C ABI: an undersized tensor is a ValueError on the host, never an out-of-bounds device access."""
    import torch
    n, ctx, _ = small
    W = 512 * 11 * n * n
    big = torch.zeros(2 * W, dtype=torch.int64, device="cuda")
    short = torch.zeros(W - 1, dtype=torch.int64, device="cuda")
    msg = torch.zeros(2 * 512 * n * n, dtype=torch.float64, device="cuda")
    sk = torch.zeros(512 * 11 * n, dtype=torch.int64, device="cuda")
    with pytest.raises(ValueError):
        ctx.matrix_to_poly(short, big)
    with pytest.raises(ValueError):
        ctx.wcrt_fwd(big, short)
    with pytest.raises(ValueError):
        ctx.encode(msg[:-1], big, big)
    with pytest.raises(ValueError):
        ctx.keygen(sk[:-1])
    with pytest.raises(ValueError):
        ctx.encrypt_pair(big, big, sk, big, short)
    with pytest.raises(ValueError):
        ctx.decrypt_and_decode(big, big[:W], sk, msg)
    with pytest.raises(ValueError):
        ctx.ct_add(big, big, short)
    # the exact sizes pass
    ctx.matrix_to_poly(big[:W], big[W:])
    torch.cuda.synchronize()
