#!/usr/bin/env python3
"""Sweep NTT plan / chunk options on the device (dev tool)."""
import sys, json
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "matrix-fhe-gpu_amd")); sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tools"))
import torch
import mfhe
from bench import gen_moduli
from ntt_perf import t_call

MiB = 1 << 20
cases = [((16, 8, 1024), [(0, c) for c in (0, 16 * MiB, 32 * MiB, 64 * MiB, 96 * MiB, 128 * MiB, 192 * MiB)]),
         ((15, 8, 1024), [(0, c) for c in (0, 32 * MiB, 64 * MiB, 128 * MiB)]),
         ((17, 32, 128), [(0, c) for c in (0, 32 * MiB, 64 * MiB, 128 * MiB)]),
         ((14, 4, 256), [(1, 0), (2, 0), (2, 32 * MiB), (2, 64 * MiB)]),
         ((14, 4, 2048), [(1, 0), (2, 0), (2, 32 * MiB), (2, 64 * MiB), (2, 128 * MiB)]),
         ((13, 4, 2048), [(1, 0), (2, 32 * MiB), (2, 64 * MiB)]),
         ((12, 1, 4096), [(1, 0), (2, 0), (2, 32 * MiB)])]
for (log_n, L, batch), opts in cases:
    N = 1 << log_n
    ctx = mfhe.Context(gen_moduli(50, 1 << (log_n + 2), L), log_n)
    d = torch.randint(0, 2 ** 40, (batch * L * N,), dtype=torch.int64, device="cuda")
    for plan, chunk in opts:
        ctx.set_option(mfhe.OPT_NTT_PLAN, plan)
        ctx.set_option(mfhe.OPT_NTT_CHUNK_BYTES, chunk)
        f = t_call(lambda: ctx.ntt_fwd(d, batch=batch))
        i = t_call(lambda: ctx.ntt_inv(d, batch=batch))
        nt = batch * L
        print(json.dumps({"logN": log_n, "L": L, "batch": batch, "plan": plan, "chunk_MiB": chunk // MiB,
                          "fwd_ms": round(f, 4), "fwd_NTT_s": round(nt / f * 1e3),
                          "fwd_alg_GBps": round(16.0 * N * nt / f / 1e6, 1), "inv_ms": round(i, 4)}), flush=True)
    del d
    torch.cuda.empty_cache()
