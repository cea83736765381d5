#!/usr/bin/env python3
"""C3 forward + inverse NTT on the U64 path (60-bit primes; NTTP_BITS=50 for the FP64 path), `reps` calls each,
for a rocprofv3 kernel trace.  Dev tool.  usage: tools/u64_prof.py [reps] [prefetch]"""
import os
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matrix-fhe-gpu_amd"), str(ROOT)]
import torch  # noqa: E402

import mfhe  # noqa: E402
from bench import gen_moduli  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
log_n, L, batch = (int(v) for v in os.environ.get("NTTP_SHAPE", "16,8,1024").split(","))   # C3 unless set
N = 1 << log_n
moduli = gen_moduli(int(os.environ.get("NTTP_BITS", 60)), 1 << (log_n + 2), L)
ctx = mfhe.Context(moduli, log_n, mfhe.CONV_PHANTOM)
if len(sys.argv) > 2:
    ctx.set_option(mfhe.OPT_NTT_PREFETCH, int(sys.argv[2]))
d = torch.empty(batch * L * N, dtype=torch.int64, device="cuda")
qt = torch.tensor(moduli, dtype=torch.int64, device="cuda").repeat_interleave(N).repeat(batch)
d.random_(0, 2 ** 62).remainder_(qt)
ref = d.clone()
del qt
res = {}
for kind, fn in (("fwd", ctx.ntt_fwd), ("inv", ctx.ntt_inv)):
    fn(d, batch=batch)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn(d, batch=batch)
    e1.record()
    torch.cuda.synchronize()
    res[f"{kind}_NTT_per_s"] = round(batch * L / (e0.elapsed_time(e1) / reps * 1e-3))
ctx.ntt_fwd(d, batch=batch)   # (reps + 1) forward, (reps + 1) inverse: one more forward restores the input
ctx.ntt_inv(d, batch=batch)
torch.cuda.synchronize()
res["arith"] = "u64" if ctx.info().arith == mfhe.ARITH_U64 else "f64"
res["roundtrip_ok"] = bool(torch.equal(d, ref))
print(json.dumps(res))
