#!/usr/bin/env python3
"""Time mfhe NTT / CRT calls across shapes (device-resident data, HIP events). Dev tool."""
import sys, json, time
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "matrix-fhe-gpu_amd"))
sys.path.insert(0, str(ROOT))
import torch
import mfhe
from bench import gen_moduli


def t_call(fn, reps=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    shapes = [(6, 11, 32768), (12, 1, 4096), (14, 4, 256), (14, 4, 2048), (15, 8, 1024), (16, 8, 1024), (16, 8, 256), (17, 32, 128)]
    if len(sys.argv) > 1:
        shapes = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]]
    for log_n, L, batch in shapes:
        N = 1 << log_n
        mods = mfhe.RNS_MODULI if (log_n == 6 and L == 11) else gen_moduli(50, 1 << (log_n + 2), L)
        ctx = mfhe.Context(mods, log_n)
        d = torch.randint(0, 2 ** 40, (batch * L * N,), dtype=torch.int64, device="cuda")
        for arith in (1, 2):
            ctx.set_arith(arith)
            f = t_call(lambda: ctx.ntt_fwd(d, batch=batch))
            i = t_call(lambda: ctx.ntt_inv(d, batch=batch))
            nt = batch * L
            gb = 16.0 * N * nt / 1e9
            print(json.dumps({"logN": log_n, "L": L, "batch": batch, "arith": "f64" if arith == 1 else "u64",
                              "fwd_ms": round(f, 4), "fwd_NTT_s": round(nt / f * 1e3), "fwd_alg_GBps": round(gb / f * 1e3, 1),
                              "inv_ms": round(i, 4), "inv_NTT_s": round(nt / i * 1e3)}), flush=True)
        del d
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
