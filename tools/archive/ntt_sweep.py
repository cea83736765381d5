#!/usr/bin/env python3
"""Sweep NTT launch options (prefetch, workgroups/CU, chunk bytes) across shapes; HIP-event timing. Dev tool.

usage: tools/ntt_sweep.py [logN,L,batch ...]   (one JSON line per configuration)
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "matrix-fhe-gpu_amd"))
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import mfhe  # noqa: E402
from bench import gen_moduli  # noqa: E402

OPT_WG, OPT_PF, OPT_FUSED, OPT_LAG = 4, 5, 6, 7


def t_call(fn, reps=8):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    shapes = [(16, 8, 1024), (14, 4, 256), (17, 32, 128), (12, 1, 4096), (6, 11, 32768)]
    if len(sys.argv) > 1:
        shapes = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]]
    for log_n, L, batch in shapes:
        N = 1 << log_n
        mods = mfhe.RNS_MODULI if (log_n == 6 and L == 11) else gen_moduli(50, 1 << (log_n + 2), L)
        ctx = mfhe.Context(mods, log_n)
        q = torch.tensor(mods, dtype=torch.int64, device="cuda").repeat_interleave(N).repeat(batch)
        d = torch.randint(0, 2 ** 62, (batch * L * N,), dtype=torch.int64, device="cuda") % q
        ref = d.clone()
        chunks = [192 << 20, 0] if log_n > 14 else [192 << 20]
        import os
        if os.environ.get("CHUNKS"):
            chunks = [int(x) << 20 for x in os.environ["CHUNKS"].split(",")]
        if log_n >= 15 and not os.environ.get("NOFUSED"):
            for lag in (1, 2, 3, 4, 6):
                ctx.set_option(OPT_FUSED, 1)
                ctx.set_option(OPT_LAG, lag)
                ctx.ntt_fwd(d, batch=batch)
                ctx.ntt_inv(d, batch=batch)
                torch.cuda.synchronize()
                ok = bool(torch.equal(d, ref)) and ctx.get_option(8) == 0
                f = t_call(lambda: ctx.ntt_fwd(d, batch=batch))
                i = t_call(lambda: ctx.ntt_inv(d, batch=batch))
                ntts = batch * L
                print(json.dumps({"logN": log_n, "L": L, "batch": batch, "fused": 1, "lag": lag, "fwd_ms": round(f, 4),
                                  "fwd_NTT_s": round(ntts / f * 1e3), "fwd_alg_GBps": round(16 * N * ntts / f / 1e6, 1),
                                  "inv_ms": round(i, 4), "inv_NTT_s": round(ntts / i * 1e3), "roundtrip_ok": ok}),
                      flush=True)
            ctx.set_option(OPT_FUSED, 0)
        import os
        quick = os.environ.get("QUICK") == "1"
        for pf in ((0,) if quick else (0, 1)):
            for wg in ((16,) if os.environ.get("WG16") else (0, 16) if quick else (0, 1, 2, 3, 4, 16)):
                for cb, plan, ov in [(c, p, o) for c in chunks for p in [int(x) for x in os.environ.get("PLANS", "0").split(",")]
                                     for o in [int(x) for x in os.environ.get("OVERLAP", "0").split(",")]]:
                    ctx.set_option(2, plan)
                    if os.environ.get("OVERLAP"):
                        ctx.set_option(10, ov)
                    ctx.set_option(OPT_PF, pf)
                    ctx.set_option(OPT_WG, wg)
                    ctx.set_option(mfhe.OPT_NTT_CHUNK_BYTES, cb)
                    ctx.ntt_fwd(d, batch=batch)
                    ctx.ntt_inv(d, batch=batch)
                    torch.cuda.synchronize()
                    ok = bool(torch.equal(d, ref))
                    f = t_call(lambda: ctx.ntt_fwd(d, batch=batch))
                    i = t_call(lambda: ctx.ntt_inv(d, batch=batch))
                    ntts = batch * L
                    print(json.dumps({"logN": log_n, "L": L, "batch": batch, "prefetch": pf, "wg_per_cu": wg,
                                      "chunk_MiB": cb >> 20, "plan": plan, "overlap": ov, "fwd_ms": round(f, 4), "fwd_NTT_s": round(ntts / f * 1e3),
                                      "fwd_alg_GBps": round(16 * N * ntts / f / 1e6, 1), "inv_ms": round(i, 4),
                                      "inv_NTT_s": round(ntts / i * 1e3), "roundtrip_ok": ok}), flush=True)
        del d, ref, q


if __name__ == "__main__":
    main()
