#!/usr/bin/env python3
"""One NTT timing line (HIP events, forward and inverse, in-place on one resident batch) for A/B runs across
library builds (tools/lib_ab.py sets MFHE_LIB).  usage: tools/ntt_rate.py log_n L batch bits [arith] [reps] [u60]
(u60: MFHE_OPT_NTT_U60 for the forward, default the context's)"""
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

log_n, L, batch, bits = (int(x) for x in sys.argv[1:5])
arith = int(sys.argv[5]) if len(sys.argv) > 5 else 0
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 20
u60 = int(sys.argv[7]) if len(sys.argv) > 7 else -1
N = 1 << log_n
moduli = gen_moduli(bits, 1 << (log_n + 2), L)
ctx = mfhe.Context(moduli, log_n, mfhe.CONV_PHANTOM)
if arith:
    ctx.set_arith(arith)
if u60 >= 0:
    ctx.set_option(mfhe.OPT_NTT_U60, u60)
d = torch.empty(batch * L * N, dtype=torch.int64, device="cuda")
qt = torch.tensor(moduli, dtype=torch.int64, device="cuda").repeat_interleave(N).repeat(batch)
d.random_(0, 2 ** 62).remainder_(qt)
ref = d.clone()
out = {"lib": os.path.basename(os.environ.get("MFHE_LIB", "libmfhe.so")), "log_n": log_n, "L": L, "batch": batch,
       "bits": bits, "arith": "u64" if ctx.info().arith == mfhe.ARITH_U64 else "f64",
       "u60": ctx.get_option(mfhe.OPT_NTT_U60)}
for kind, fn in (("fwd", ctx.ntt_fwd), ("inv", ctx.ntt_inv)):
    for _ in range(3):
        fn(d, batch=batch)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn(d, batch=batch)
    e1.record()
    torch.cuda.synchronize()
    r = batch * L / (e0.elapsed_time(e1) / reps * 1e-3)
    out[f"{kind}_NTT_s"] = round(r)
    out[f"{kind}_frac"] = round(16 * N * r / 8e12, 4)
# round trip check: (3 + reps) forward and as many inverse transforms
out["roundtrip_ok"] = bool(torch.equal(d, ref))
print(json.dumps(out), flush=True)
