"""GPU parity at the full BASELINE shapes, through the C ABI, against the oracle's committed digests.

BASELINE.json configs exercised at exactly the shape they name (tests/golden/fullshape.py):
  C2        N = 2^14, L = 4, batch 256: forward + inverse NTT
  C3        N = 2^16, L = 8, batch 1024: forward + inverse NTT (F64 and U64 arithmetic, DMA and plain
            column passes), 60-bit primes (U64), and the encode -> NTT -> INTT -> decode-with-CRT chain
            (RNS decompose, forward NTT, inverse NTT, wide CRT compose -> f64) plus the full-path
            integer CRT compose of uniform residues
  C5 shard  N = 2^17, 32 moduli, batch 4096, limbs 4..7 (one GPU's residue shard of 8)
Reference behaviour matched: phantom fnwt_1d / inwt_1d via xy_ntt_forward/backward_phantom
(ntt_core.cu:443-460), quantize_coeff_to_rns_kernel (batched_encoder.cu:125-152),
crt_compose_centerlift_big (encoder.cu:191-245) and he_big_to_f64 (HE.cu:917-924); the reference's
own full-batch round trip is test_custom_ntt_roundtrip.cu:63-112, its encode/decode chain
test_encode_decode_wcrt.cu:29-116.  Expected digests: tests/golden/make_digests.py (CPU oracle).
"""
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
import fullshape as F  # noqa: E402

pytestmark = pytest.mark.gpu

@pytest.fixture(scope="module")
def dig():
    with np.load(Path(__file__).resolve().parent / "golden" / "digests.npz") as z:
        return {k: z[k] for k in z.files}


def _upload_residues(orc, d, cfg, moduli):
    import torch
    N = 1 << cfg["log_n"]
    nl, B = cfg["nl"], cfg["batch"]
    step = F.CHUNK_POLYS[cfg["log_n"]]
    per = nl * N
    for p0 in range(0, B, step):
        nb = min(step, B - p0)
        x = orc.fill_residues(nb, nl, N, moduli, cfg["seed"], p0)
        d[p0 * per:(p0 + nb) * per].copy_(torch.from_numpy(x.view(np.int64)))


def _digest_device(d, npoly, words_per_poly, chunk_polys, extra=None, extra_per_poly=0):
    """Per-poly digests of a device buffer, downloaded in chunks."""
    import torch
    torch.cuda.synchronize()
    out = []
    for p0 in range(0, npoly, chunk_polys):
        nb = min(chunk_polys, npoly - p0)
        h = d[p0 * words_per_poly:(p0 + nb) * words_per_poly].cpu().numpy()
        e = None if extra is None else extra[p0 * extra_per_poly:(p0 + nb) * extra_per_poly].cpu().numpy()
        out.append(F.poly_digests(h, nb, extra=e))
    return np.concatenate(out)


def _check(got, want, what):
    bad = F.first_mismatch(got, want)
    assert bad is None, f"{what}: polynomial {bad} differs from the oracle (top digest {F.top_digest(got)} " \
                        f"vs {F.top_digest(want)})"


def _run_ntt_config(mfhe, orc, dig, name, arith=0, prefetch=None):
    import torch
    cfg = F.NTT_CONFIGS[name]
    N = 1 << cfg["log_n"]
    allm = F.moduli_for(cfg)
    ms = F.shard_moduli(cfg)
    ctx = mfhe.Context(allm, cfg["log_n"])
    if arith:
        ctx.set_arith(arith)
    if prefetch is not None:   # default 2: the DMA column pass; 0: the plain column pass
        ctx.set_option(mfhe.OPT_NTT_PREFETCH, prefetch)
    B, nl, st = cfg["batch"], cfg["nl"], cfg["start"]
    per = nl * N
    step = F.CHUNK_POLYS[cfg["log_n"]]
    d = torch.empty(B * per, dtype=torch.int64, device="cuda")
    _upload_residues(orc, d, cfg, ms)
    ctx.ntt_fwd(d, batch=B, start_limb=st, nlimbs=nl)
    if "fwd" in cfg["kinds"]:
        _check(_digest_device(d, B, per, step), dig[f"{name}_fwd"], f"{name} forward NTT")
    ctx.ntt_inv(d, batch=B, start_limb=st, nlimbs=nl)
    _check(_digest_device(d, B, per, step), dig[f"{name}_in"], f"{name} inverse(forward(x)) == x")
    if "inv" in cfg["kinds"]:
        ctx.ntt_inv(d, batch=B, start_limb=st, nlimbs=nl)
        _check(_digest_device(d, B, per, step), dig[f"{name}_inv"], f"{name} inverse NTT")
    del d
    torch.cuda.empty_cache()


def test_c2_full_shape(mfhe, orc, dig):
    _run_ntt_config(mfhe, orc, dig, "c2")


@pytest.mark.parametrize("arith,prefetch", [(0, None), (2, None), (0, 0), (2, 0)],
                         ids=["f64", "u64", "f64-plain-colpass", "u64-plain-colpass"])
def test_c3_full_shape(mfhe, orc, dig, arith, prefetch):
    _run_ntt_config(mfhe, orc, dig, "c3", arith, prefetch)


def test_c3_60bit_primes_full_shape(mfhe, orc, dig):
    _run_ntt_config(mfhe, orc, dig, "c3u60")


@pytest.mark.parametrize("prefetch", [None, 0], ids=["default", "plain-colpass"])
def test_c5_shard_full_shape(mfhe, orc, dig, prefetch):
    _run_ntt_config(mfhe, orc, dig, "c5shard", prefetch=prefetch)


def test_c3_encode_ntt_intt_decode_full_shape(mfhe, orc, dig):
    """C3: messages -> RNS decompose -> forward NTT -> inverse NTT -> wide CRT compose -> f64, batch 1024,
    every stage's full output checked against the oracle's digest; then the integer (bigint) compose of
    uniform residues, which takes the full path rather than the small-value fast path."""
    import torch
    cfg = F.NTT_CONFIGS[F.C3_PIPE["cfg"]]
    N, B, L = 1 << cfg["log_n"], cfg["batch"], cfg["L"]
    ms = F.moduli_for(cfg)
    ctx = mfhe.Context(ms, cfg["log_n"], delta=F.C3_PIPE["delta"])
    W = ctx.crt_words
    assert W == int(dig["c3pipe_W"][0])
    step = F.CHUNK_POLYS[cfg["log_n"]]
    msg = torch.empty(B * N, dtype=torch.float64, device="cuda")
    for p0 in range(0, B, step):
        nb = min(step, B - p0)
        msg[p0 * N:(p0 + nb) * N].copy_(torch.from_numpy(orc.fill_messages(nb * N, F.C3_PIPE["msg_seed"], p0 * N)))
    res = torch.empty(B * L * N, dtype=torch.int64, device="cuda")
    ctx.rns_decompose(msg, res, B, N)
    _check(_digest_device(res, B, L * N, step), dig["c3pipe_decomp"], "C3 RNS decompose")
    ctx.ntt_fwd(res, batch=B)
    _check(_digest_device(res, B, L * N, step), dig["c3pipe_decomp_fwd"], "C3 forward NTT of the residues")
    ctx.ntt_inv(res, batch=B)
    out = torch.empty(B * N, dtype=torch.float64, device="cuda")
    ctx.crt_compose_f64(res, out, B, N)
    _check(_digest_device(out, B, N, step), dig["c3pipe_compose_f64"], "C3 decode (compose -> f64)")
    err = (out - msg).abs().max().item()
    assert err < 1e-9, f"round trip error {err}"
    del msg, out
    _upload_residues(orc, res, cfg, ms)
    mag = torch.empty(B * N * W, dtype=torch.int64, device="cuda")
    neg = torch.empty(B * N, dtype=torch.uint8, device="cuda")
    ctx.crt_compose(res, mag, neg, B, N)
    _check(_digest_device(mag, B, N * W, step, extra=neg, extra_per_poly=N), dig["c3pipe_compose_int"],
           "C3 wide CRT compose (uniform residues, full path)")
    del res, mag, neg
    torch.cuda.empty_cache()


@pytest.mark.parametrize("prefetch", [None, 0], ids=["default", "plain-colpass"])
def test_c4_shard_full_shape(mfhe, orc, dig, prefetch):
    """BASELINE C4's per-GPU NTT shape (N = 2^16, 16 moduli, batch 1024, limbs 4..7 of GPU 1 of 4), forward and
    inverse against the oracle's digests."""
    _run_ntt_config(mfhe, orc, dig, "c4shard", prefetch=prefetch)
