"""Golden vectors (tests/golden/golden.npz, made by tests/golden/make_golden.py).

CPU: the oracle must still reproduce every frozen output (pins the oracle against drift).
GPU: the HIP path must reproduce them bit-exactly (integer) / exactly-rounded (f64 dequantize).
"""
from pathlib import Path

import numpy as np
import pytest

import oracle as O

G = np.load(Path(__file__).resolve().parent / "golden" / "golden.npz")
RNS = [17592186435073, 17182765057, 17184541441, 17186120449, 17186515201, 17186909953,
       17188883713, 17190462721, 17190857473, 17191844353, 17192831233]
DELTA = 2.0 ** 35


def test_oracle_reproduces_golden():
    x = G["ref64_in"]
    np.testing.assert_array_equal(O.phantom_fwd(x, 11, 6, RNS), G["ref64_phantom_fwd"])
    np.testing.assert_array_equal(O.gl_fwd(x, 11, 64, RNS), G["ref64_gl_fwd"])
    np.testing.assert_array_equal(O.custom_fwd(x, 11, 64, RNS), G["ref64_cyclic_fwd"])
    np.testing.assert_array_equal(O.gl_perm(x, 11, 64), G["ref64_gl_perm"])
    np.testing.assert_array_equal(O.phantom_fwd(G["ref64_pattern1_in"], 11, 6, RNS), G["ref64_pattern1_phantom_fwd"])
    np.testing.assert_array_equal(O.gl_fwd(G["ref64_pattern7_in"], 11, 64, RNS), G["ref64_pattern7_gl_fwd"])
    np.testing.assert_array_equal(O.phantom_fwd(G["c1_in"], 1, 12, G["c1_moduli"]), G["c1_phantom_fwd"])
    np.testing.assert_array_equal(O.phantom_fwd(G["c2_in"], 2, 14, G["c2_moduli"]), G["c2_phantom_fwd"])
    mag, neg = O.crt_compose(G["crt_in"], 2, 11, 128, RNS, W=7)
    np.testing.assert_array_equal(mag.ravel(), G["crt_mag"])
    np.testing.assert_array_equal(neg, G["crt_neg"])
    np.testing.assert_array_equal(O.big_to_f64(mag, neg, 7, DELTA), G["crt_f64"])
    np.testing.assert_array_equal(O.rns_decompose(G["rns_in"], 1, 256, RNS, DELTA), G["rns_out"])
    np.testing.assert_array_equal(O.HE(4, RNS, DELTA).keygen(), G["keygen_n4_sk"])
    # inverses recover the inputs
    np.testing.assert_array_equal(O.phantom_inv(G["c2_phantom_fwd"], 2, 14, G["c2_moduli"]), G["c2_in"])


@pytest.mark.gpu
def test_device_reproduces_golden(mfhe):
    import torch

    def run(ctx, fn, data, *a):
        d = mfhe.to_device_u64(data)
        getattr(ctx, fn)(d, *a)
        torch.cuda.synchronize()
        return mfhe.to_host_u64(d)

    c64 = mfhe.Context(RNS, 6, mfhe.CONV_PHANTOM | mfhe.CONV_GL)
    x = G["ref64_in"]
    np.testing.assert_array_equal(run(c64, "ntt_fwd", x), G["ref64_phantom_fwd"])
    np.testing.assert_array_equal(run(c64, "gl_ntt_fwd", x), G["ref64_gl_fwd"])
    np.testing.assert_array_equal(run(c64, "cyclic_ntt_fwd", x), G["ref64_cyclic_fwd"])
    np.testing.assert_array_equal(run(c64, "ntt_fwd", G["ref64_pattern1_in"]), G["ref64_pattern1_phantom_fwd"])
    np.testing.assert_array_equal(run(c64, "gl_ntt_fwd", G["ref64_pattern7_in"]), G["ref64_pattern7_gl_fwd"])
    src = mfhe.to_device_u64(x)
    dst = torch.empty_like(src)
    c64.gl_perm(src, dst, 4)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mfhe.to_host_u64(dst), G["ref64_gl_perm"])
    for tag, logn, L in (("c1", 12, 1), ("c2", 14, 2)):
        c = mfhe.Context([int(q) for q in G[f"{tag}_moduli"]], logn, mfhe.CONV_PHANTOM)
        np.testing.assert_array_equal(run(c, "ntt_fwd", G[f"{tag}_in"]), G[f"{tag}_phantom_fwd"])
    # CRT compose at the reference's 7-word stride, dequantize, decompose
    c11 = mfhe.Context(RNS, 6, mfhe.CONV_PHANTOM)
    c11.set_option(mfhe.OPT_CRT_WORDS, 7)
    src = mfhe.to_device_u64(G["crt_in"])
    mag = torch.empty(256 * 7, dtype=torch.int64, device="cuda")
    neg = torch.empty(256, dtype=torch.uint8, device="cuda")
    c11.crt_compose(src, mag, neg, 2, 128)
    f = torch.empty(256, dtype=torch.float64, device="cuda")
    c11.crt_compose_f64(src, f, 2, 128)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mfhe.to_host_u64(mag), G["crt_mag"])
    np.testing.assert_array_equal(neg.cpu().numpy(), G["crt_neg"])
    np.testing.assert_array_equal(f.cpu().numpy(), G["crt_f64"])
    v = torch.from_numpy(G["rns_in"].copy()).cuda()
    r = torch.empty(256 * 11, dtype=torch.int64, device="cuda")
    c11.rns_decompose(v, r, 1, 256)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mfhe.to_host_u64(r), G["rns_out"])
    # W-CRT forward (n = 2, L = 2) and keygen (n = 4, L = 11)
    cw = mfhe.Context(RNS[:2], 1, mfhe.CONV_PHANTOM | mfhe.CONV_WCRT)
    w = mfhe.to_device_u64(G["wcrt_in"])
    wo = torch.empty_like(w)
    cw.wcrt_fwd(w, wo)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mfhe.to_host_u64(wo), G["wcrt_fwd"])
    ck = mfhe.Context(RNS, 2, mfhe.CONV_PHANTOM | mfhe.CONV_WCRT)
    sk = torch.empty(512 * 11 * 4, dtype=torch.int64, device="cuda")
    ck.keygen(sk)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mfhe.to_host_u64(sk), G["keygen_n4_sk"])
