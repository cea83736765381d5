#!/usr/bin/env python3
"""Dev tool: fused NTT at C3, forward and inverse checked separately (error word after each, forward output vs
the two-pass plan's), over workgroups/CU x lag; then `cycles` back-to-back forward+inverse pairs with no host sync in between (the
bench's timed-loop shape) checked once at the end.  usage: tools/fused_diag.py mode wg,wg lag,lag [cycles [stress]]
(stress: that many forward calls on fresh input, each checked word for word)"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matrix-fhe-gpu_amd"), str(ROOT)]
import torch  # noqa: E402

import mfhe  # noqa: E402
from bench import gen_moduli  # noqa: E402

mode = int(sys.argv[1])
wgs = [int(x) for x in sys.argv[2].split(",")]
lags = [int(x) for x in sys.argv[3].split(",")]
cycles = int(sys.argv[4]) if len(sys.argv) > 4 else 0
stress = int(sys.argv[5]) if len(sys.argv) > 5 else 0
import os  # noqa: E402
log_n = 16
L, batch = int(os.environ.get("FD_L", 8)), int(os.environ.get("FD_BATCH", 1024))   # C3 unless set
N = 1 << log_n
ctx = mfhe.Context(gen_moduli(50, 1 << (log_n + 2), L), log_n)
q = torch.tensor(ctx.moduli, dtype=torch.int64, device="cuda").repeat_interleave(N).repeat(batch)
ref = torch.randint(0, 2 ** 62, (batch * L * N,), dtype=torch.int64, device="cuda") % q
del q
want = ref.clone()
ctx.ntt_fwd(want, batch=batch)          # two-pass plan
d = torch.empty_like(ref)
for wg in wgs:
    for lag in lags:
        ctx.set_option(mfhe.OPT_NTT_FUSED, mode)
        ctx.set_option(mfhe.OPT_NTT_WG_PER_CU, wg)
        ctx.set_option(mfhe.OPT_NTT_FUSED_LAG, lag)
        d.copy_(ref)
        ctx.ntt_fwd(d, batch=batch)
        torch.cuda.synchronize()
        ef = ctx.get_option(mfhe.OPT_NTT_FUSED_ERRORS)
        fok = bool(torch.equal(d, want))
        nbad = int((d != want).sum().item()) if not fok else 0
        ctx.ntt_inv(d, batch=batch)
        torch.cuda.synchronize()
        ei = ctx.get_option(mfhe.OPT_NTT_FUSED_ERRORS)
        iok = bool(torch.equal(d, ref))
        rec = {"mode": mode, "wg": wg, "lag": lag, "fwd_ok": fok, "fwd_bad_words": nbad, "fwd_err": ef,
               "inv_ok": iok, "inv_err": ei}
        if cycles:
            d.copy_(ref)
            for _ in range(cycles):
                ctx.ntt_fwd(d, batch=batch)
                ctx.ntt_inv(d, batch=batch)
            torch.cuda.synchronize()
            rec.update(cycles=cycles, cycles_ok=bool(torch.equal(d, ref)),
                       cycles_bad_words=int((d != ref).sum().item()),
                       cycles_err=ctx.get_option(mfhe.OPT_NTT_FUSED_ERRORS))
        # stress: forward only, fresh input each time, every output checked; where the bad words sit
        bad = []
        for rep in range(stress):
            d.copy_(ref)
            ctx.ntt_fwd(d, batch=batch)
            torch.cuda.synchronize()
            if not torch.equal(d, want):
                idx = torch.nonzero(d != want).flatten()
                poly, off = idx // N, idx % N
                row, col = off // 256, off % 256
                bad.append({"rep": rep, "n": int(idx.numel()), "polys": sorted(set(poly.tolist()))[:8],
                            "rows": [int(row.min()), int(row.max())], "cols": [int(col.min()), int(col.max())],
                            "raw_fp64": int((d[idx] > (1 << 62)).sum().item())})
        if stress:
            rec.update(stress=stress, stress_fail=len(bad), stress_first=bad[:4],
                       stress_err=ctx.get_option(mfhe.OPT_NTT_FUSED_ERRORS))
        print(rec, flush=True)
        ctx.set_option(mfhe.OPT_NTT_FUSED, 0)
