#!/usr/bin/env python3
"""Generate tests/golden/golden.npz: small input/output vectors for the hot path.

The reference cannot be built or run in this container (no nvcc, empty phantom-fhe
submodule, NVIDIA-only PTX), so the vectors are produced by the CPU oracle (oracle/mfhe_oracle.c),
which is itself pinned to the reference's known-answer tests (tests/test_oracle_kat.py).  Freezing
them here makes the GPU parity tests independent of the oracle build, and makes any oracle drift
visible (tests/test_golden.py re-derives every output on the CPU).

Inputs are deterministic (numpy default_rng with fixed seeds, or the reference's own input
patterns where named).  Run: python tests/golden/make_golden.py
"""
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
import oracle as O  # noqa: E402

RNS = [17592186435073, 17182765057, 17184541441, 17186120449, 17186515201, 17186909953,
       17188883713, 17190462721, 17190857473, 17191844353, 17192831233]   # config.h:32-44
DELTA = 2.0 ** 35


def rand_res(rng, shape, moduli):
    q = np.array(moduli, np.uint64)[None, :, None]
    return (rng.integers(0, 2 ** 63, shape, dtype=np.uint64) % q).ravel()


def main():
    g = {}
    rng = np.random.default_rng(0x4D464845)
    # reference geometry n = 64, L = 11: phantom X-NTT, GL NTT, cyclic NTT, GL permutation
    x = rand_res(rng, (4, 11, 64), RNS)
    g["ref64_in"] = x
    g["ref64_phantom_fwd"] = O.phantom_fwd(x, 11, 6, RNS)
    g["ref64_gl_fwd"] = O.gl_fwd(x, 11, 64, RNS)
    g["ref64_cyclic_fwd"] = O.custom_fwd(x, 11, 64, RNS)
    g["ref64_gl_perm"] = O.gl_perm(x, 11, 64)
    # test_custom_ntt_roundtrip.cu:63-72 / :115-124 input patterns (b + l + x + 1 / + 7) mod q_l, 2 polys
    b, l, xx = np.meshgrid(np.arange(2, dtype=np.uint64), np.arange(11, dtype=np.uint64),
                           np.arange(64, dtype=np.uint64), indexing="ij")
    q = np.array(RNS, np.uint64)[None, :, None]
    pat1 = ((b + l + xx + np.uint64(1)) % q).ravel()
    pat7 = ((b + l + xx + np.uint64(7)) % q).ravel()
    g["ref64_pattern1_in"] = pat1
    g["ref64_pattern1_phantom_fwd"] = O.phantom_fwd(pat1, 11, 6, RNS)
    g["ref64_pattern7_in"] = pat7
    g["ref64_pattern7_gl_fwd"] = O.gl_fwd(pat7, 11, 64, RNS)
    # C1: N = 2^12, one 50-bit modulus (BASELINE configs[0]); C2 shape at N = 2^14, 2 limbs
    m12 = O.gen_primes(50, 1 << 14, 1)
    y = rand_res(rng, (1, 1, 4096), m12)
    g["c1_moduli"] = np.array(m12, np.uint64)
    g["c1_in"] = y
    g["c1_phantom_fwd"] = O.phantom_fwd(y, 1, 12, m12)
    m14 = O.gen_primes(50, 1 << 16, 2)
    z = rand_res(rng, (1, 2, 16384), m14)
    g["c2_moduli"] = np.array(m14, np.uint64)
    g["c2_in"] = z
    g["c2_phantom_fwd"] = O.phantom_fwd(z, 2, 14, m14)
    # wide CRT compose (W = 7, the reference stride) + f64/delta, RNS decompose
    c = rand_res(rng, (2, 11, 128), RNS)
    g["crt_in"] = c
    mag, neg = O.crt_compose(c, 2, 11, 128, RNS, W=7)
    g["crt_mag"], g["crt_neg"] = mag.ravel(), neg
    g["crt_f64"] = O.big_to_f64(mag, neg, 7, DELTA)
    v = rng.uniform(-1.0, 1.0, 256) * rng.choice([1.0, 1e3, 1e6], 256)
    g["rns_in"] = v
    g["rns_out"] = O.rns_decompose(v, 1, 256, RNS, DELTA)
    # W-CRT forward (matrix-major -> poly-major) at n = 2, L = 2 and keygen at n = 4, L = 11
    h2 = O.HE(2, RNS[:2], DELTA)
    w = rand_res(rng, (512, 2, 4), RNS[:2])
    out = np.zeros_like(w)
    O.L.orc_wntt_forward_matrix(O.P(w), O.P(out), 2, 2, 512, O.P(O.U64(RNS[:2])), O.L.orc_he_V(h2.h))
    g["wcrt_in"], g["wcrt_fwd"] = w, out
    h4 = O.HE(4, RNS, DELTA)
    g["keygen_n4_sk"] = h4.keygen()
    np.savez_compressed(HERE / "golden.npz", **g)
    total = sum(a.nbytes for a in g.values())
    print(f"wrote {len(g)} arrays, {total / 1024:.0f} KiB uncompressed")


if __name__ == "__main__":
    main()
