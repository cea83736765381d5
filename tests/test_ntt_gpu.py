"""GPU parity: batched NTT kernels (through include/mfhe.h) vs the CPU oracle, bit-exact.

Reference behaviour being matched: xy_ntt_forward/backward_phantom -> phantom fnwt_1d/inwt_1d
(ntt_core.cu:443-460), xy_ntt_forward/backward_gl and custom_ntt_forward/backward
(ntt_core.cu:394-431, 462-481), apply_gl_perm (ntt_core.cu:433-441).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RNS = [17592186435073, 17182765057, 17184541441, 17186120449, 17186515201, 17186909953,
       17188883713, 17190462721, 17190857473, 17191844353, 17192831233]


def rand_residues(rng, batch, moduli, N):
    q = np.array(moduli, dtype=np.uint64)[None, :, None]
    return (rng.integers(0, 2 ** 63, (batch, len(moduli), N), dtype=np.uint64) % q).ravel()


def _roundtrip(mfhe, orc, ctx, data, nl_moduli, log_n, arith):
    import torch
    ctx.set_arith(arith)
    L_ = len(nl_moduli)
    d = mfhe.to_device_u64(data)
    ctx.ntt_fwd(d)
    torch.cuda.synchronize()
    got = mfhe.to_host_u64(d)
    ref = orc.phantom_fwd(data, L_, log_n, nl_moduli)
    np.testing.assert_array_equal(got, ref)
    ctx.ntt_inv(d)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mfhe.to_host_u64(d), data)


@pytest.mark.parametrize("log_n", list(range(1, 18)))
@pytest.mark.parametrize("arith", [1, 2])
def test_phantom_ntt_matches_oracle(mfhe, orc, log_n, arith):
    N = 1 << log_n
    moduli = orc.gen_primes(50 if arith == 1 else 61, 4 * N, 3)
    if arith == 1:
        moduli = orc.gen_primes(50, 4 * N, 3)
    batch = max(1, min(5, (1 << 18) // (N * 3)))
    ctx = mfhe.Context(moduli, log_n, mfhe.CONV_PHANTOM)
    if arith == 2 and moduli[0] >= 2 ** 50:
        assert ctx.info().arith == mfhe.ARITH_U64
    rng = np.random.default_rng(log_n)
    data = rand_residues(rng, batch, moduli, N)
    _roundtrip(mfhe, orc, ctx, data, moduli, log_n, arith)


@pytest.mark.parametrize("arith", [1, 2])
def test_phantom_inverse_of_random_matches_oracle(mfhe, orc, arith):
    import torch
    log_n = 16
    moduli = orc.gen_primes(49, 1 << 18, 2)
    ctx = mfhe.Context(moduli, log_n)
    ctx.set_arith(arith)
    data = rand_residues(np.random.default_rng(1), 2, moduli, 1 << log_n)
    d = mfhe.to_device_u64(data)
    ctx.ntt_inv(d)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mfhe.to_host_u64(d), orc.phantom_inv(data, 2, log_n, moduli))


@pytest.mark.parametrize("arith", [1, 2])
def test_kat1_reference_geometry_roundtrip(mfhe, orc, arith):
    """test_custom_ntt_roundtrip.cu:63-112 at reference geometry: n = 64, L = 11, batch 1 and 32768,
    input (b+l+x+1) mod q; forward must also equal the oracle (phantom) bit-exactly."""
    ctx = mfhe.Context(RNS, 6)
    for batch in (1, 512 * 64):
        b = np.arange(batch, dtype=np.uint64)[:, None, None]
        l = np.arange(11, dtype=np.uint64)[None, :, None]
        x = np.arange(64, dtype=np.uint64)[None, None, :]
        data = ((b + l + x + 1) % np.array(RNS, np.uint64)[None, :, None]).ravel()
        _roundtrip(mfhe, orc, ctx, data, RNS, 6, arith)


def test_extreme_moduli_and_values(mfhe, orc):
    """F64 path edge: the largest primes below 2^50 with all-(q-1) and all-zero inputs."""
    import torch
    for log_n in (6, 12, 16, 17):
        N = 1 << log_n
        moduli = orc.gen_primes(50, 2 * N, 2)
        assert all(q < 2 ** 50 for q in moduli)
        ctx = mfhe.Context(moduli, log_n)
        assert ctx.info().arith == mfhe.ARITH_F64
        for fill in ("max", "zero", "alt"):
            q = np.array(moduli, np.uint64)[None, :, None]
            if fill == "max":
                data = np.broadcast_to(q - 1, (2, 2, N)).copy().ravel()
            elif fill == "zero":
                data = np.zeros(2 * 2 * N, np.uint64)
            else:
                data = np.where(np.arange(N)[None, None, :] % 2 == 0, q - 1, 0).astype(np.uint64)
                data = np.broadcast_to(data, (2, 2, N)).copy().ravel()
            d = mfhe.to_device_u64(data)
            ctx.ntt_fwd(d)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(mfhe.to_host_u64(d), orc.phantom_fwd(data, 2, log_n, moduli))
            ctx.ntt_inv(d)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(mfhe.to_host_u64(d), data)


def test_extreme_moduli_and_values_u64(mfhe, orc):
    """U64 path edge: the largest primes below 2^62 (the Harvey 4q < 2^64 limit) with all-(q-1), all-zero
    and alternating inputs, single-pass and two-pass sizes."""
    import torch
    for log_n in (6, 14, 16, 17):
        N = 1 << log_n
        moduli = orc.gen_primes(62, 2 * N, 2)
        assert all(2 ** 61 < q < 2 ** 62 for q in moduli)
        ctx = mfhe.Context(moduli, log_n)
        assert ctx.info().arith == mfhe.ARITH_U64
        q = np.array(moduli, np.uint64)[None, :, None]
        for fill in ("max", "zero", "alt"):
            if fill == "max":
                data = np.broadcast_to(q - 1, (2, 2, N)).copy().ravel()
            elif fill == "zero":
                data = np.zeros(2 * 2 * N, np.uint64)
            else:
                data = np.where(np.arange(N)[None, None, :] % 2 == 0, q - 1, 0).astype(np.uint64)
                data = np.broadcast_to(data, (2, 2, N)).copy().ravel()
            d = mfhe.to_device_u64(data)
            ctx.ntt_fwd(d)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(mfhe.to_host_u64(d), orc.phantom_fwd(data, 2, log_n, moduli))
            ctx.ntt_inv(d)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(mfhe.to_host_u64(d), data)


@pytest.mark.parametrize("log_n", list(range(1, 18)))
def test_u60_forward_matches_oracle_and_harvey(mfhe, orc, log_n):
    """The lazy U60 forward schedule (ntt_arith.hpp ArithU60: u inputs reduced once per round, unreduced
    intermediate, FP32-quotient canonicalisation) on the largest primes below 2^60, where its 16q < 2^64 bound is
    tightest: random, all-(q-1), all-zero and alternating inputs, bit-exact against the oracle and against the
    Harvey schedule (MFHE_OPT_NTT_U60 0) on every plan shape log n 1..17."""
    import torch
    N = 1 << log_n
    moduli = orc.gen_primes(60, 2 * N, 3)
    assert all(2 ** 59 < q < 2 ** 60 for q in moduli)
    ctx = mfhe.Context(moduli, log_n)
    assert ctx.info().arith == mfhe.ARITH_U64 and ctx.get_option(mfhe.OPT_NTT_U60) == 1
    q = np.array(moduli, np.uint64)[None, :, None]
    rng = np.random.default_rng(60 + log_n)
    fills = {"rand": rand_residues(rng, 2, moduli, N),
             "max": np.broadcast_to(q - 1, (2, 3, N)).copy().ravel(),
             "zero": np.zeros(2 * 3 * N, np.uint64),
             "alt": np.broadcast_to(np.where(np.arange(N)[None, None, :] % 2 == 0, q - 1, 0).astype(np.uint64),
                                    (2, 3, N)).copy().ravel()}
    for name, data in fills.items():
        ref = orc.phantom_fwd(data, 3, log_n, moduli)
        outs = []
        for u60 in (1, 0):
            ctx.set_option(mfhe.OPT_NTT_U60, u60)
            d = mfhe.to_device_u64(data)
            ctx.ntt_fwd(d)
            torch.cuda.synchronize()
            outs.append(mfhe.to_host_u64(d))
            np.testing.assert_array_equal(outs[-1], ref, err_msg=f"{name} u60={u60}")
        ctx.set_option(mfhe.OPT_NTT_U60, 1)
        d = mfhe.to_device_u64(ref)
        ctx.ntt_inv(d)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(mfhe.to_host_u64(d), data, err_msg=name)


def test_u60_option_is_effective_only_below_2_60(mfhe, orc):
    ctx = mfhe.Context(orc.gen_primes(61, 1 << 12, 2), 10)
    assert ctx.get_option(mfhe.OPT_NTT_U60) == 0          # a modulus >= 2^60: Harvey schedule
    ctx.set_option(mfhe.OPT_NTT_U60, 1)
    assert ctx.get_option(mfhe.OPT_NTT_U60) == 0
    ctx2 = mfhe.Context(orc.gen_primes(55, 1 << 12, 2), 10)
    assert ctx2.get_option(mfhe.OPT_NTT_U60) == 1
    ctx2.set_option(mfhe.OPT_NTT_U60, 0)
    assert ctx2.get_option(mfhe.OPT_NTT_U60) == 0
    with pytest.raises(mfhe.MfheError):
        ctx2.set_option(mfhe.OPT_NTT_U60, 2)


def test_empty_batch_is_a_no_op(mfhe, orc):
    """batch 0 (an empty ragged tail) launches nothing and touches nothing, on every plan."""
    import torch
    for log_n in (6, 14, 16):
        moduli = orc.gen_primes(50, 4 << log_n, 2)
        ctx = mfhe.Context(moduli, log_n)
        sentinel = torch.full((16,), 7, dtype=torch.int64, device="cuda")
        ctx.ntt_fwd(sentinel, batch=0)
        ctx.ntt_inv(sentinel, batch=0)
        torch.cuda.synchronize()
        assert bool((sentinel == 7).all())


def test_limb_subrange(mfhe, orc):
    """start_limb / nlimbs select moduli start..start+nl-1 (the fnwt_1d start_modulus_idx)."""
    import torch
    log_n = 12
    moduli = orc.gen_primes(50, 1 << 14, 5)
    ctx = mfhe.Context(moduli, log_n)
    sub = moduli[2:4]
    data = rand_residues(np.random.default_rng(2), 3, sub, 1 << log_n)
    d = mfhe.to_device_u64(data)
    ctx.ntt_fwd(d, batch=3, start_limb=2, nlimbs=2)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mfhe.to_host_u64(d), orc.phantom_fwd(data, 2, log_n, sub))


@pytest.mark.parametrize("log_n", [2, 6, 9, 12, 14])
@pytest.mark.parametrize("arith", [1, 2])
def test_gl_and_cyclic_match_oracle(mfhe, orc, log_n, arith):
    import torch
    N = 1 << log_n
    moduli = RNS if log_n <= 6 else orc.gen_primes(48, 4 * N, 3)
    ctx = mfhe.Context(moduli, log_n, mfhe.CONV_PHANTOM | mfhe.CONV_GL)
    ctx.set_arith(arith)
    data = rand_residues(np.random.default_rng(log_n), 3, moduli, N)
    for fwd, inv, ofwd, oinv in ((ctx.gl_ntt_fwd, ctx.gl_ntt_inv, orc.gl_fwd, orc.gl_bwd),
                                 (ctx.cyclic_ntt_fwd, ctx.cyclic_ntt_inv, orc.custom_fwd, orc.custom_bwd)):
        d = mfhe.to_device_u64(data)
        fwd(d)
        torch.cuda.synchronize()
        ref = ofwd(data, len(moduli), N, moduli)
        np.testing.assert_array_equal(mfhe.to_host_u64(d), ref)
        d2 = mfhe.to_device_u64(ref)
        inv(d2)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(mfhe.to_host_u64(d2), oinv(ref, len(moduli), N, moduli))
        np.testing.assert_array_equal(mfhe.to_host_u64(d2), data)


def test_kat4_gl_product_on_gpu(mfhe, orc):
    """test_custom_ntt_roundtrip.cu:256-319 on the device: product mod X^n - i."""
    import torch
    q = RNS[0]
    n = 64
    ctx = mfhe.Context([q], 6, mfhe.CONV_GL)
    psi4n = orc.L.orc_get_psi4n(q, n)
    iroot = pow(psi4n, n, q)
    a = np.array([(j + 1) % q for j in range(n)], np.uint64)
    b = np.array([(j + 3) % q for j in range(n)], np.uint64)
    da, db = mfhe.to_device_u64(a), mfhe.to_device_u64(b)
    ctx.gl_ntt_fwd(da)
    ctx.gl_ntt_fwd(db)
    torch.cuda.synchronize()
    fa, fb = mfhe.to_host_u64(da), mfhe.to_host_u64(db)
    prod = np.array([int(x) * int(y) % q for x, y in zip(fa, fb)], np.uint64)
    dp = mfhe.to_device_u64(prod)
    ctx.gl_ntt_inv(dp)
    torch.cuda.synchronize()
    ref = [0] * n
    for j in range(n):
        for k in range(n):
            p = int(a[j]) * int(b[k]) % q
            if j + k < n:
                ref[j + k] = (ref[j + k] + p) % q
            else:
                ref[j + k - n] = (ref[j + k - n] + p * iroot) % q
    assert [int(v) for v in mfhe.to_host_u64(dp)] == ref


def test_gl_perm_matches_oracle(mfhe, orc):
    import torch
    ctx = mfhe.Context(RNS, 6, mfhe.CONV_GL)
    data = rand_residues(np.random.default_rng(9), 7, RNS, 64)
    d = mfhe.to_device_u64(data)
    for inverse in (False, True):
        out = torch.empty_like(d)
        ctx.gl_perm(d, out, 7, inverse=inverse)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(mfhe.to_host_u64(out), orc.gl_perm(data, 11, 64, inverse))


def test_raw_phantom_surface(mfhe, orc):
    """fnwt_1d / inwt_1d over the context's phantom-format tables (DNTTTable surface)."""
    import torch
    ctx = mfhe.Context(RNS, 6)
    tw, tws, itw, itws, ninv, ninvs, dmod = ctx.ntt_tables()
    data = rand_residues(np.random.default_rng(4), 1, RNS, 64)
    d = mfhe.to_device_u64(data)
    mfhe.fnwt_1d(d, tw, tws, dmod, 64, 11, 0)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mfhe.to_host_u64(d), orc.phantom_fwd(data, 11, 6, RNS))
    mfhe.inwt_1d(d, itw, itws, dmod, ninv, ninvs, 64, 11, 0)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mfhe.to_host_u64(d), data)
    # tables equal the oracle's phantom host tables
    t = np.zeros(11 * 64, np.uint64)
    import ctypes
    import hip_util
    hip_util.d2h(t, tw)
    for l in (0, 10):
        otw = orc.phantom_tables(6, RNS[l])[0]
        np.testing.assert_array_equal(t[l * 64:(l + 1) * 64], otw)


def test_invalid_arguments(mfhe):
    ctx = mfhe.Context(RNS, 6)
    import torch
    d = torch.zeros(64 * 11, dtype=torch.int64, device="cuda")
    with pytest.raises(mfhe.MfheError) as e:
        ctx.ntt_fwd(d, batch=1, start_limb=5, nlimbs=7)
    assert e.value.code == mfhe.EINVAL
    with pytest.raises(mfhe.MfheError) as e:
        ctx.gl_ntt_fwd(d)
    assert e.value.code == mfhe.ENOTREADY
    with pytest.raises(mfhe.MfheError) as e:
        mfhe.Context([97], 6)   # 2N = 128 does not divide 96
    assert e.value.code == mfhe.EUNSUPPORTED


@pytest.mark.parametrize("log_n", [12, 13, 14, 15, 16, 17])
def test_two_pass_plans_and_chunking(mfhe, orc, log_n):
    """MFHE_OPT_NTT_PLAN = 2 (two passes from log_n 12) and batch chunking (uneven tail chunk)."""
    import torch
    N = 1 << log_n
    moduli = orc.gen_primes(50, 4 * N, 3)
    ctx = mfhe.Context(moduli, log_n)
    ctx.set_option(mfhe.OPT_NTT_PLAN, 2)
    batch = 5
    ctx.set_option(mfhe.OPT_NTT_CHUNK_BYTES, 2 * 3 * N * 8)   # chunks of 2 polys -> 2, 2, 1
    data = rand_residues(np.random.default_rng(100 + log_n), batch, moduli, N)
    for arith in (1, 2):
        ctx.set_arith(arith)
        d = mfhe.to_device_u64(data)
        ctx.ntt_fwd(d)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(mfhe.to_host_u64(d), orc.phantom_fwd(data, 3, log_n, moduli))
        ctx.ntt_inv(d)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(mfhe.to_host_u64(d), data)


@pytest.mark.parametrize("batch,nl,start", [(1, 1, 0), (5, 3, 1), (300, 2, 2), (1023, 1, 3), (64, 4, 0)])
def test_single_pass_14_matches_oracle_and_other_plans(mfhe, orc, batch, nl, start):
    """N = 2^14 pipelined single pass (ntt_single14.hpp, plan 0 = auto / 3; FP64): bit-exact against the oracle
    (forward and the inverse of random data), exact round trip, and equal to the two-pass (2) and the plain single
    pass (1).  Batches that leave some workgroups with one polynomial, several, or a limb change inside their
    polynomial walk (the LDS twiddle table is reloaded), a limb sub-range, and the largest primes < 2^50 with the
    all-(q - 1) input as the first polynomial."""
    import torch
    log_n, N = 14, 1 << 14
    moduli = orc.gen_primes(50, 4 * N, start + nl)
    ctx = mfhe.Context(moduli, log_n)
    assert ctx.info().arith == mfhe.ARITH_F64
    sub = moduli[start:start + nl]
    rng = np.random.default_rng(batch * 7 + nl)
    data = rand_residues(rng, batch, sub, N)
    data[:nl * N] = (np.array(sub, np.uint64)[:, None] - np.uint64(1)).repeat(N, axis=1).ravel()
    want_f = orc.phantom_fwd(data, nl, log_n, sub) if batch <= 300 else None
    got = {}
    for plan in (0, 3, 2, 1):
        ctx.set_option(mfhe.OPT_NTT_PLAN, plan)
        d = mfhe.to_device_u64(data)
        ctx.ntt_fwd(d, batch=batch, start_limb=start, nlimbs=nl)
        torch.cuda.synchronize()
        got[plan] = mfhe.to_host_u64(d)
        ctx.ntt_inv(d, batch=batch, start_limb=start, nlimbs=nl)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(mfhe.to_host_u64(d), data)
    if want_f is not None:
        np.testing.assert_array_equal(got[0], want_f)
    for plan in (3, 2, 1):
        np.testing.assert_array_equal(got[plan], got[0])
    # the inverse of arbitrary residues (not the forward's output) against the oracle
    if batch <= 64:
        ctx.set_option(mfhe.OPT_NTT_PLAN, 0)
        d = mfhe.to_device_u64(data)
        ctx.ntt_inv(d, batch=batch, start_limb=start, nlimbs=nl)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(mfhe.to_host_u64(d), orc.phantom_inv(data, nl, log_n, sub))


def test_plan_3_is_auto_for_u64_at_14(mfhe, orc):
    """MFHE_OPT_NTT_PLAN 3 is documented as auto (include/mfhe.h): on the U64 path at log_n 14 it must run auto's two
    passes, not fall through to the plain single pass.  Checked by output (oracle) under plans 0 and 3
    and by the plan the context reports (OPT_NTT_PLAN_EFFECTIVE, the function the planner itself uses)."""
    import torch
    log_n, N = 14, 1 << 14
    moduli = orc.gen_primes(60, 4 * N, 2)
    ctx = mfhe.Context(moduli, log_n)
    assert ctx.info().arith == mfhe.ARITH_U64   # 60-bit primes: the FP64 path cannot take them
    data = rand_residues(np.random.default_rng(14), 3, moduli, N)
    want = orc.phantom_fwd(data, 2, log_n, moduli)
    for plan in (0, 3):
        ctx.set_option(mfhe.OPT_NTT_PLAN, plan)
        d = mfhe.to_device_u64(data)
        ctx.ntt_fwd(d, batch=3)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(mfhe.to_host_u64(d), want)
        assert ctx.get_option(mfhe.OPT_NTT_PLAN_EFFECTIVE) == 2   # two passes
    ctx.close()


def test_fused_option_removed(mfhe, orc):
    """MFHE_OPT_NTT_FUSED (the one-launch XCD-L2 hand-off, r02-r03) was removed in r04: its hand-off was never
    proven and it was slower.  0 is still accepted; anything else fails loudly."""
    ctx = mfhe.Context(orc.gen_primes(50, 1 << 18, 1), 16)
    ctx.set_option(mfhe.OPT_NTT_FUSED, 0)
    assert ctx.get_option(mfhe.OPT_NTT_FUSED) == 0
    with pytest.raises(mfhe.MfheError):
        ctx.set_option(mfhe.OPT_NTT_FUSED, 1)
    for gone in (7, 8):   # the lag / error-word options went with it
        with pytest.raises(mfhe.MfheError):
            ctx.get_option(gone)
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("batch,nl", [(3, 2), (17, 1)])
def test_packed_intermediate_matches_oracle(mfhe, orc, batch, nl):
    """MFHE_OPT_NTT_PACK (N = 2^16 forward two-pass, 50-bit packed intermediate units written over the column
    tile's own lines): bit-exact vs the oracle and vs the unpacked plan, with chunking that splits the batch."""
    import torch
    N = 1 << 16
    moduli = orc.gen_primes(50, 4 * N, nl)
    ctx = mfhe.Context(moduli, 16)
    data = rand_residues(np.random.default_rng(batch), batch, moduli, N)
    want = orc.phantom_fwd(data, nl, 16, moduli)
    for chunk in (0, 2 * nl * N * 8):
        ctx.set_option(mfhe.OPT_NTT_CHUNK_BYTES, chunk)
        ctx.set_option(mfhe.OPT_NTT_PACK, 1)
        d = mfhe.to_device_u64(data)
        ctx.ntt_fwd(d, batch=batch)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(mfhe.to_host_u64(d), want)
    ctx.set_option(mfhe.OPT_NTT_PACK, 0)
    assert ctx.get_option(mfhe.OPT_NTT_PACK) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("log_n", [15, 16, 17])
@pytest.mark.parametrize("batch,nl", [(1, 1), (7, 3), (33, 2)])
def test_column_pass_dma_prefetch_matches_oracle(mfhe, orc, log_n, batch, nl):
    """MFHE_OPT_NTT_PREFETCH = 2 (ntt_coldb.hpp: forward column pass with the next tile's LDS-DMA in flight, counted
    vmcnt waits, twiddles reloaded per limb): bit-exact vs the oracle on a limb sub-range, with and without
    chunking (chunks of 2 polynomials: tiles of several limbs per workgroup, a last chunk of one), and exact
    roundtrip through the unchanged inverse."""
    import torch
    N = 1 << log_n
    moduli = orc.gen_primes(50, 4 * N, nl + 1)
    ctx = mfhe.Context(moduli, log_n)
    assert ctx.get_option(mfhe.OPT_NTT_PREFETCH) == 2   # the default
    data = rand_residues(np.random.default_rng(11 * log_n + batch), batch, moduli[1:], N)
    want = orc.phantom_fwd(data, nl, log_n, moduli[1:])
    for chunk in (0, 2 * nl * N * 8):
        ctx.set_option(mfhe.OPT_NTT_CHUNK_BYTES, chunk)
        d = mfhe.to_device_u64(data)
        ctx.ntt_fwd(d, batch=batch, start_limb=1, nlimbs=nl)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(mfhe.to_host_u64(d), want)
        ctx.ntt_inv(d, batch=batch, start_limb=1, nlimbs=nl)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(mfhe.to_host_u64(d), data)


def test_plan5_removed(mfhe, orc):
    """MFHE_OPT_NTT_PLAN 5 (the one-launch N = 2^16 forward with the column -> block hand-off in each XCD's L2, r05) and
    its timeout word MFHE_OPT_NTT_XL2_TIMEOUT (16) were removed in r06. Its SQ counters showed it latency-bound at the
    one wave per SIMD its 132 KiB of LDS allows (profiles/r06_xl2_sq_pmc.txt), and it ran slower than the two passes.
    Both options now fail loudly. The plans that remain are still accepted."""
    ctx = mfhe.Context(orc.gen_primes(50, 1 << 18, 1), 16)
    for plan in (0, 1, 2, 3):
        ctx.set_option(mfhe.OPT_NTT_PLAN, plan)
    for bad in (4, 5):
        with pytest.raises(mfhe.MfheError) as e:
            ctx.set_option(mfhe.OPT_NTT_PLAN, bad)
        assert e.value.code == mfhe.EINVAL
    with pytest.raises(mfhe.MfheError):
        ctx.get_option(16)
    ctx.close()
