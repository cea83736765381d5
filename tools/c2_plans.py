#!/usr/bin/env python3
"""C2 (N = 2^14, L = 4, batch 256) forward / inverse NTT/s per MFHE_OPT_NTT_PLAN, HBM figure: 8 rotating buffers
of 128 MiB (1 GiB, each evicted before its next use), as bench.py other_configs_line; plans alternate, 3 rounds.
usage: tools/c2_plans.py [plans, default 0,2,1]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "matrix-fhe-gpu_amd"))
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402
import mfhe  # noqa: E402
from bench import gen_moduli  # noqa: E402

plans = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,2,1").split(",")]
log_n, L, batch, nbuf, reps = 14, 4, 256, 8, 20
N = 1 << log_n
moduli = gen_moduli(50, 1 << (log_n + 2), L)
ctx = mfhe.Context(moduli, log_n, mfhe.CONV_PHANTOM)
qt = torch.tensor(moduli, dtype=torch.int64, device="cuda").repeat_interleave(N).repeat(batch)
bufs = [torch.empty(batch * L * N, dtype=torch.int64, device="cuda").random_(0, 2 ** 62).remainder_(qt) for _ in range(nbuf)]


def rate(fn, nb):
    for k in range(nb):
        fn(bufs[k], batch=batch)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    n = reps * nb
    for k in range(n):
        fn(bufs[k % nb], batch=batch)
    e1.record()
    torch.cuda.synchronize()
    return batch * L / (e0.elapsed_time(e1) / n * 1e-3)


for rnd in range(3):
    for plan in plans:
        ctx.set_option(mfhe.OPT_NTT_PLAN, plan)
        f, i = rate(ctx.ntt_fwd, nbuf), rate(ctx.ntt_inv, nbuf)
        fc = rate(ctx.ntt_fwd, 1)
        print(json.dumps({"round": rnd, "plan": plan, "fwd_NTT_s": round(f), "inv_NTT_s": round(i),
                          "frac_fwd": round(16 * N * f / 8e12, 4), "frac_inv": round(16 * N * i / 8e12, 4),
                          "cache_resident_fwd_NTT_s": round(fc)}), flush=True)
