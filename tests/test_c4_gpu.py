"""BASELINE C4 (encode + encrypt + decrypt + decode with CRT, residues sharded across GPUs) on one GPU.

Reference flow: test/test_encode_encrypt_decrypt_decode_wcrt.cu:29-110 (input v = l + 0.001 i as the pair
(v, -v), check max |err| < 1e-3) through encode_to_wntt_eval (batched_encoder.cu:161-228), encrypt_pair
(HE.cu:1455-1552) and decrypt_and_decode (HE.cu:1691-1708), here at L = 16 moduli q = 1 mod 2^8 * 771.

* Every integer stage of a residue shard (limbs [g*L/G, (g+1)*L/G), mfhe_ctx_set_limb_shard) must be exactly
  those limbs of the unsharded stage: encode, keygen, encrypt_pair, decrypt_to_eval, for G = 2 and 4.
* The sharded decode through a 1-rank RCCL communicator (the native exchange path) must equal the
  unsharded decrypt_and_decode bit for bit.  The G > 1 receive layout is pinned by test_dist_gpu.py and the
  gloo tests.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

L, N_LOG, PHI = 16, 6, 512


def _moduli(orc):
    # the 16 largest primes < 2^35 with q = 1 mod 197376 (= 2^8 * 771): reference-sized limbs (config.h:32-44)
    return orc.gen_primes(35, 197376, L)


def _message():
    n2 = 1 << (2 * N_LOG)
    ell = np.arange(PHI)[:, None] * np.ones((1, n2))
    v = ell + 0.001j                           # test_encode_encrypt_decrypt_decode_wcrt.cu:44-52
    return v.ravel()


@pytest.fixture(scope="module")
def full(mfhe, orc):
    import torch
    moduli = _moduli(orc)
    ctx = mfhe.Context(moduli, N_LOG, mfhe.CONV_PHANTOM | mfhe.CONV_WCRT)
    ctx.reserve_workspace()
    n2, words = 1 << (2 * N_LOG), PHI * L * (1 << (2 * N_LOG))
    msg = _message()
    mt = torch.from_numpy(msg.view(np.float64).copy()).cuda()
    out = {k: torch.empty(words, dtype=torch.int64, device="cuda") for k in ("re", "im")}
    ctx.encode(mt, out["re"], out["im"])
    sk = torch.empty(PHI * L * (1 << N_LOG), dtype=torch.int64, device="cuda")
    ctx.keygen(sk)
    cre, cim = (torch.empty(2 * words, dtype=torch.int64, device="cuda") for _ in range(2))
    ctx.encrypt_pair(out["re"], out["im"], sk, cre, cim)
    ev = torch.empty(words, dtype=torch.int64, device="cuda")
    ctx.decrypt_to_eval(cre, sk, ev)
    res = torch.empty_like(mt)
    ctx.decrypt_and_decode(cre, cim, sk, res)
    torch.cuda.synchronize()
    yield dict(ctx=ctx, moduli=moduli, msg=msg, mt=mt, enc=out, sk=sk, cre=cre, cim=cim, ev=ev, res=res)
    ctx.close()


def _limbs(t, lo, hi, inner):
    """Limbs [lo, hi) of a [..][L][inner] u64 tensor, flattened."""
    return t.view(-1, L, inner)[:, lo:hi, :].reshape(-1)


def test_c4_unsharded_roundtrip(full):
    err = np.max(np.abs(full["res"].cpu().numpy().view(np.complex128) - full["msg"]))
    assert err < 1e-3, err       # the reference's pass criterion (test_...decode_wcrt.cu:109)


@pytest.mark.parametrize("G", [2, 4])
def test_c4_shard_integer_stages_are_slices(mfhe, full, G):
    import torch
    n, n2, lg = 1 << N_LOG, 1 << (2 * N_LOG), L // G
    words = PHI * lg * n2
    for g in range(G):
        lo, hi = g * lg, (g + 1) * lg
        c = mfhe.Context(full["moduli"][lo:hi], N_LOG, mfhe.CONV_PHANTOM | mfhe.CONV_WCRT)
        c.set_limb_shard(lo, L)
        re, im = (torch.empty(words, dtype=torch.int64, device="cuda") for _ in range(2))
        c.encode(full["mt"], re, im)
        sk = torch.empty(PHI * lg * n, dtype=torch.int64, device="cuda")
        c.keygen(sk)
        cre, cim = (torch.empty(2 * words, dtype=torch.int64, device="cuda") for _ in range(2))
        c.encrypt_pair(re, im, sk, cre, cim)
        ev = torch.empty(words, dtype=torch.int64, device="cuda")
        c.decrypt_to_eval(cre, sk, ev)
        torch.cuda.synchronize()
        assert torch.equal(re, _limbs(full["enc"]["re"], lo, hi, n2))
        assert torch.equal(im, _limbs(full["enc"]["im"], lo, hi, n2))
        assert torch.equal(sk, _limbs(full["sk"], lo, hi, n))
        for mine, whole in ((cre, full["cre"]), (cim, full["cim"])):   # [b | a], each [512][L][n2]
            w_all = PHI * L * n2
            assert torch.equal(mine[:words], _limbs(whole[:w_all], lo, hi, n2))
            assert torch.equal(mine[words:], _limbs(whole[w_all:], lo, hi, n2))
        assert torch.equal(ev, _limbs(full["ev"], lo, hi, n))          # poly-major [512 n][L][n]
        c.close()


@pytest.mark.parametrize("mode", ["allgather", "alltoall"])
def test_c4_sharded_decode_one_rank_equals_unsharded(mfhe, full, mode):
    import torch
    c_all = mfhe.Context(full["moduli"], N_LOG, mfhe.CONV_PHANTOM)
    comm = mfhe.Comm.from_id(mfhe.Comm.unique_id(), 1, 0)
    try:
        out = torch.empty_like(full["mt"])
        full["ctx"].decrypt_and_decode_sharded(c_all, comm, mode, full["cre"], full["cim"], full["sk"], out)
        torch.cuda.synchronize()
        assert torch.equal(out, full["res"])
    finally:
        comm.close()
        c_all.close()


def test_limb_shard_rejects_bad_ranges(mfhe, full):
    c = mfhe.Context(full["moduli"][:4], N_LOG, mfhe.CONV_PHANTOM)
    with pytest.raises(mfhe.MfheError):
        c.set_limb_shard(14, 16)
    with pytest.raises(mfhe.MfheError):
        c.set_limb_shard(0, 3)
    c.set_limb_shard(12, 16)
    c.close()


def test_sharded_decode_rejects_mismatched_parameter_sets(mfhe, orc, full):
    """ctx_all must hold this rank's moduli at limbs rank * L_shard..: a different prime set of the same size
    is an error (not silently wrong messages)."""
    import torch
    other = orc.gen_primes(34, 197376, L)                 # 16 different primes
    assert set(other).isdisjoint(full["moduli"])
    c_bad = mfhe.Context(other, N_LOG, mfhe.CONV_PHANTOM)
    # the right primes at another scale: the compose would divide by the wrong delta
    c_delta = mfhe.Context(full["moduli"], N_LOG, mfhe.CONV_PHANTOM, delta=2.0 ** 30)
    comm = mfhe.Comm.from_id(mfhe.Comm.unique_id(), 1, 0)
    try:
        out = torch.empty_like(full["mt"])
        for bad in (c_bad, c_delta):
            with pytest.raises(mfhe.MfheError):
                full["ctx"].decrypt_and_decode_sharded(bad, comm, "allgather", full["cre"], full["cim"], full["sk"],
                                                       out)
    finally:
        comm.close()
        c_bad.close()
        c_delta.close()
