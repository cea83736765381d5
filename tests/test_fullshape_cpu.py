"""CPU side of the full-shape digests (tests/golden/fullshape.py): the committed per-polynomial
digests must be reproducible from the oracle.  Re-deriving every polynomial takes about a minute
(tests/golden/make_digests.py), so this re-derives the first and the last polynomial of each
configuration, which pins the input generator, the moduli and the digest scheme."""
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
import fullshape as F  # noqa: E402


@pytest.fixture(scope="module")
def dig():
    with np.load(Path(__file__).resolve().parent / "golden" / "digests.npz") as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("name", list(F.NTT_CONFIGS))
def test_ntt_digest_samples(orc, dig, name):
    cfg = F.NTT_CONFIGS[name]
    N = 1 << cfg["log_n"]
    ms = F.shard_moduli(cfg)
    nl = cfg["nl"]
    assert dig[f"{name}_in"].shape == (cfg["batch"], 32)
    for p in (0, cfg["batch"] - 1):
        x = orc.fill_residues(1, nl, N, ms, cfg["seed"], p)
        assert (F.poly_digests(x, 1)[0] == dig[f"{name}_in"][p]).all()
        if "fwd" in cfg["kinds"]:
            y = orc.phantom_fwd(x, nl, cfg["log_n"], ms)
            assert (F.poly_digests(y, 1)[0] == dig[f"{name}_fwd"][p]).all()
        if "inv" in cfg["kinds"]:
            y = orc.phantom_inv(x, nl, cfg["log_n"], ms)
            assert (F.poly_digests(y, 1)[0] == dig[f"{name}_inv"][p]).all()


def test_c3_pipeline_digest_samples(orc, dig):
    cfg = F.NTT_CONFIGS[F.C3_PIPE["cfg"]]
    N, L = 1 << cfg["log_n"], cfg["L"]
    ms = F.moduli_for(cfg)
    W = int(dig["c3pipe_W"][0])
    assert W == orc.crt_words(ms)
    for p in (0, cfg["batch"] - 1):
        msg = orc.fill_messages(N, F.C3_PIPE["msg_seed"], p * N)
        r = orc.rns_decompose(msg, 1, N, ms, F.C3_PIPE["delta"])
        assert (F.poly_digests(r, 1)[0] == dig["c3pipe_decomp"][p]).all()
        assert (F.poly_digests(orc.phantom_fwd(r, L, cfg["log_n"], ms), 1)[0] == dig["c3pipe_decomp_fwd"][p]).all()
        mag, neg = orc.crt_compose(r, 1, L, N, ms, W)
        f = orc.big_to_f64(mag, neg, W, F.C3_PIPE["delta"])
        assert np.abs(f - msg).max() < 1e-9
        assert (F.poly_digests(f, 1)[0] == dig["c3pipe_compose_f64"][p]).all()
        x = orc.fill_residues(1, L, N, ms, cfg["seed"], p)
        mag, neg = orc.crt_compose(x, 1, L, N, ms, W)
        assert (F.poly_digests(mag, 1, extra=neg)[0] == dig["c3pipe_compose_int"][p]).all()


def test_input_generator_is_splitmix64(orc):
    """orc_fill_residues element i = splitmix64(seed + i) mod q_l (pure-Python restatement)."""
    M = (1 << 64) - 1

    def sm(x):
        z = (x + 0x9E3779B97F4A7C15) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)

    ms = [97, 193, 257]
    x = orc.fill_residues(2, 3, 8, ms, 12345, 0).reshape(2, 3, 8)
    for p in range(2):
        for l in range(3):
            for c in range(8):
                assert int(x[p, l, c]) == sm(12345 + (p * 3 + l) * 8 + c) % ms[l]
    m = orc.fill_messages(4, 99, 10)
    for i in range(4):
        assert m[i] == (sm(99 + 10 + i) >> 11) * 2.0 ** -52 - 1.0
