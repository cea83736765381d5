#!/usr/bin/env python3
"""C3 forward NTT/s under MFHE_OPT_NTT_PLAN 0 (two passes) and 5 (one launch, XCD-L2 hand-off, ntt_xl2.hpp),
alternating, one resident 4 GiB batch, HIP events; the plan-5 output is checked against plan 0's on every round and
the timeout word is reported.  usage: tools/xl2_rate.py [rounds] [reps]   (MFHE_LIB selects a variant build)"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "matrix-fhe-gpu_amd"))
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402
import mfhe  # noqa: E402
from bench import gen_moduli  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
log_n, L, batch = 16, 8, 1024
N = 1 << log_n
moduli = gen_moduli(50, 1 << (log_n + 2), L)
ctx = mfhe.Context(moduli, log_n, mfhe.CONV_PHANTOM)
src = torch.empty(batch * L * N, dtype=torch.int64, device="cuda")
qt = torch.tensor(moduli, dtype=torch.int64, device="cuda").repeat_interleave(N).repeat(batch)
src.random_(0, 2 ** 62).remainder_(qt)
del qt
d = torch.empty_like(src)
lib = os.path.basename(os.environ.get("MFHE_LIB", "libmfhe.so"))
for r in range(rounds):
    outs = {}
    for plan in (0, 5):
        ctx.set_option(mfhe.OPT_NTT_PLAN, plan)
        for _ in range(3):
            ctx.ntt_fwd(d, batch=batch)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            ctx.ntt_fwd(d, batch=batch)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        rate = batch * L / (ms * 1e-3)
        d.copy_(src)
        ctx.ntt_fwd(d, batch=batch)
        torch.cuda.synchronize()
        outs[plan] = d.clone() if plan == 0 else d
        line = {"lib": lib, "round": r, "plan": plan, "ms": round(ms, 4), "fwd_NTT_s": round(rate),
                "frac": round(16 * N * rate / 8e12, 4)}
        if plan == 5:
            line["timeout"] = ctx.get_option(mfhe.OPT_NTT_XL2_TIMEOUT)
            line["equal_to_plan0"] = bool(torch.equal(outs[0], outs[5]))
        print(json.dumps(line), flush=True)
    del outs
