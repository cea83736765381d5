#!/usr/bin/env python3
"""Dev tool: fused NTT at C3, forward and inverse checked separately (error word after each, forward output vs
the two-pass plan's), over workgroups/CU x lag.  usage: tools/fused_diag.py mode wg,wg lag,lag"""
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
log_n, L, batch = 16, 8, 1024
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
        print({"mode": mode, "wg": wg, "lag": lag, "fwd_ok": fok, "fwd_bad_words": nbad, "fwd_err": ef,
               "inv_ok": iok, "inv_err": ei}, flush=True)
        ctx.set_option(mfhe.OPT_NTT_FUSED, 0)
