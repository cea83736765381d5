#!/usr/bin/env python3
"""Generate tests/golden/digests.npz: per-polynomial SHA-256 digests of the CPU oracle's outputs at the
full BASELINE shapes (tests/golden/fullshape.py describes the configurations and the digest scheme).

The reference cannot be built or run in this container, so the expected outputs come
from the oracle (oracle/mfhe_oracle.c), which is pinned to the reference's known-answer tests
(tests/test_oracle_kat.py).  Streams each configuration in chunks of polynomials, so the 16 GiB C5
shard never has to be resident.  Run: python tests/golden/make_digests.py   (about a minute on 8 cores)
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(HERE))
import oracle as O  # noqa: E402
import fullshape as F  # noqa: E402


def ntt_digests(name: str, cfg: dict) -> dict:
    N = 1 << cfg["log_n"]
    ms = F.shard_moduli(cfg)
    nl, B = cfg["nl"], cfg["batch"]
    step = F.CHUNK_POLYS[cfg["log_n"]]
    out = {k: [] for k in cfg["kinds"]}
    out["in"] = []
    for p0 in range(0, B, step):
        nb = min(step, B - p0)
        x = O.fill_residues(nb, nl, N, ms, cfg["seed"], p0)
        out["in"].append(F.poly_digests(x, nb))
        if "fwd" in out:
            out["fwd"].append(F.poly_digests(O.phantom_fwd(x, nl, cfg["log_n"], ms), nb))
        if "inv" in out:
            out["inv"].append(F.poly_digests(O.phantom_inv(x, nl, cfg["log_n"], ms), nb))
    return {f"{name}_{k}": np.concatenate(v) for k, v in out.items()}


def c3_pipeline() -> dict:
    cfg = F.NTT_CONFIGS[F.C3_PIPE["cfg"]]
    N, B, L = 1 << cfg["log_n"], cfg["batch"], cfg["L"]
    ms = F.moduli_for(cfg)
    W = O.crt_words(ms)
    step = F.CHUNK_POLYS[cfg["log_n"]]
    out = {k: [] for k in ("decomp", "decomp_fwd", "compose_f64", "compose_int")}
    for p0 in range(0, B, step):
        nb = min(step, B - p0)
        msg = O.fill_messages(nb * N, F.C3_PIPE["msg_seed"], p0 * N)
        r = O.rns_decompose(msg, nb, N, ms, F.C3_PIPE["delta"])
        out["decomp"].append(F.poly_digests(r, nb))
        out["decomp_fwd"].append(F.poly_digests(O.phantom_fwd(r, L, cfg["log_n"], ms), nb))
        mag, neg = O.crt_compose(r, nb, L, N, ms, W)
        out["compose_f64"].append(F.poly_digests(O.big_to_f64(mag, neg, W, F.C3_PIPE["delta"]), nb))
        x = O.fill_residues(nb, L, N, ms, cfg["seed"], p0)
        mag, neg = O.crt_compose(x, nb, L, N, ms, W)
        out["compose_int"].append(F.poly_digests(mag, nb, extra=neg))
    res = {f"c3pipe_{k}": np.concatenate(v) for k, v in out.items()}
    res["c3pipe_W"] = np.array([W])
    return res


def main():
    """No arguments: every configuration.  With names (e.g. `c4shard`): only those, merged into the committed
    digests.npz / digests.json (the other entries are kept as they are)."""
    only = set(sys.argv[1:])
    res, meta = {}, {}
    if only:
        with np.load(HERE / "digests.npz") as z:
            res = {k: z[k] for k in z.files}
        meta = json.loads((HERE / "digests.json").read_text())
    for name, cfg in F.NTT_CONFIGS.items():
        if only and name not in only:
            continue
        t = time.time()
        d = ntt_digests(name, cfg)
        res.update(d)
        meta[name] = {k: F.top_digest(v) for k, v in d.items()}
        print(f"{name}: {time.time() - t:.1f} s", meta[name], flush=True)
    if not only or "c3pipe" in only:
        t = time.time()
        d = c3_pipeline()
        res.update(d)
        meta["c3pipe"] = {k: F.top_digest(v) for k, v in d.items() if k != "c3pipe_W"}
        print(f"c3pipe: {time.time() - t:.1f} s", meta["c3pipe"], flush=True)
    np.savez_compressed(HERE / "digests.npz", **res)
    (HERE / "digests.json").write_text(json.dumps(meta, indent=1) + "\n")


if __name__ == "__main__":
    main()
