#!/usr/bin/env python3
"""Run one NTT configuration a few times (for rocprofv3 counter passes). Dev tool.
usage: tools/ntt_once.py logN L batch fused lag wg [reps] [inv]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "matrix-fhe-gpu_amd"))
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import mfhe  # noqa: E402
from bench import gen_moduli  # noqa: E402

log_n, L, batch, fused, lag, wg = (int(x) for x in sys.argv[1:7])
reps = int(sys.argv[7]) if len(sys.argv) > 7 else 3
inv = len(sys.argv) > 8 and sys.argv[8] == "inv"
N = 1 << log_n
ctx = mfhe.Context(gen_moduli(50, 1 << (log_n + 2), L), log_n)
ctx.set_option(6, fused)
ctx.set_option(7, lag)
ctx.set_option(4, wg)
q = torch.tensor(ctx.moduli, dtype=torch.int64, device="cuda").repeat_interleave(N).repeat(batch)
d = torch.randint(0, 2 ** 62, (batch * L * N,), dtype=torch.int64, device="cuda") % q
del q
for _ in range(reps):
    (ctx.ntt_inv if inv else ctx.ntt_fwd)(d, batch=batch)
torch.cuda.synchronize()
print("done", log_n, L, batch, fused, lag, wg)
