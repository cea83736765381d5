#!/usr/bin/env python3
"""Sweep the fused (single-launch, L2 hand-off) NTT over workgroups/CU and pass-2 lag; HIP-event timing.
Dev tool.  usage: tools/fused_sweep.py logN,L,batch [...]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "matrix-fhe-gpu_amd"))
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
import torch  # noqa: E402

import mfhe  # noqa: E402
from bench import gen_moduli  # noqa: E402
from ntt_sweep import t_call  # noqa: E402

OPT_WG, OPT_FUSED, OPT_LAG, OPT_ERR = 4, 6, 7, 8


def main():
    shapes = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]] or [(16, 8, 1024)]
    for log_n, L, batch in shapes:
        N = 1 << log_n
        ctx = mfhe.Context(gen_moduli(50, 1 << (log_n + 2), L), log_n)
        q = torch.tensor(ctx.moduli, dtype=torch.int64, device="cuda").repeat_interleave(N).repeat(batch)
        d = torch.randint(0, 2 ** 62, (batch * L * N,), dtype=torch.int64, device="cuda") % q
        ref = d.clone()
        import os
        mode = int(os.environ.get("FUSED_MODE", "1"))
        ctx.set_option(OPT_FUSED, mode)
        wgs = [int(x) for x in os.environ.get("FUSED_WGS", "1,2,3,4").split(",")]
        lags = [int(x) for x in os.environ.get("FUSED_LAGS", "1,2,3,4,6,8").split(",")]
        for wg in wgs:
            for lag in (lags if mode >= 1 else (1,)):
                ctx.set_option(OPT_WG, wg)
                ctx.set_option(OPT_LAG, lag)
                ctx.ntt_fwd(d, batch=batch)
                ctx.ntt_inv(d, batch=batch)
                torch.cuda.synchronize()
                ok = bool(torch.equal(d, ref)) and ctx.get_option(OPT_ERR) == 0
                f = t_call(lambda: ctx.ntt_fwd(d, batch=batch))
                i = t_call(lambda: ctx.ntt_inv(d, batch=batch))
                ntts = batch * L
                print(json.dumps({"lib": os.path.basename(os.environ.get("MFHE_LIB", "libmfhe.so")), "logN": log_n, "L": L, "batch": batch, "mode": mode, "wg": wg, "lag": lag, "fwd_ms": round(f, 4),
                                  "fwd_NTT_s": round(ntts / f * 1e3), "inv_NTT_s": round(ntts / i * 1e3),
                                  "ok": ok}), flush=True)


if __name__ == "__main__":
    main()
