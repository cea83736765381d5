#!/usr/bin/env python3
"""Reference-geometry pipeline timing (src/main.cu:31-157 flow): n = 64, phi = 512 W-lanes, the 11
reference moduli.  encode -> encrypt_pair -> decrypt_and_decode, HIP-event timed per stage, plus the
main.cu 1e-4 check.  Dev / profiling tool (run under rocprofv3 --kernel-trace --stats for the split).

usage: tools/pipeline_bench.py [reps]"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "matrix-fhe-gpu_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mfhe  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    t0 = time.perf_counter()
    ctx = mfhe.Context(mfhe.RNS_MODULI, 6, mfhe.CONV_PHANTOM | mfhe.CONV_WCRT)
    ctx.reserve_workspace()
    import os
    if os.environ.get("MFHE_WCRT_MODE"):
        ctx.set_option(9, int(os.environ["MFHE_WCRT_MODE"]))   # MFHE_OPT_WCRT_MFMA
    if os.environ.get("MFHE_WCRT_PIPE"):
        ctx.set_option(14, int(os.environ["MFHE_WCRT_PIPE"]))  # MFHE_OPT_WCRT_PIPE
    if os.environ.get("MFHE_HE_STREAMS"):
        ctx.set_option(18, int(os.environ["MFHE_HE_STREAMS"]))  # MFHE_OPT_HE_STREAMS
    if os.environ.get("MFHE_ENC_A_DIRECT"):
        ctx.set_option(19, int(os.environ["MFHE_ENC_A_DIRECT"]))  # MFHE_OPT_ENC_A_DIRECT
    if os.environ.get("MFHE_ENC_E_SMALL"):
        ctx.set_option(21, int(os.environ["MFHE_ENC_E_SMALL"]))  # MFHE_OPT_ENC_E_SMALL
    if os.environ.get("MFHE_CGEMM_MODE"):
        ctx.set_option(10, int(os.environ["MFHE_CGEMM_MODE"]))  # MFHE_OPT_CGEMM_MFMA
    t_ctx = time.perf_counter() - t0
    n2 = 64 * 64
    ell, i = np.meshgrid(np.arange(512), np.arange(n2), indexing="ij")
    msg = ((ell + i * 1e-5) + 1j * (ell - i * 1e-5)).ravel()          # main.cu:62-69
    mt = torch.from_numpy(msg.view(np.float64).copy()).cuda()
    words = 512 * 11 * n2
    sk = torch.empty(512 * 11 * 64, dtype=torch.int64, device="cuda")
    re_, im_ = (torch.empty(words, dtype=torch.int64, device="cuda") for _ in range(2))
    cre, cim = (torch.empty(2 * words, dtype=torch.int64, device="cuda") for _ in range(2))
    out = torch.empty_like(mt)
    ev = torch.empty(words, dtype=torch.int64, device="cuda")
    stages = {
        "keygen": lambda: ctx.keygen(sk),
        "encode": lambda: ctx.encode(mt, re_, im_),
        "encrypt_pair": lambda: ctx.encrypt_pair(re_, im_, sk, cre, cim),
        "decrypt_and_decode": lambda: ctx.decrypt_and_decode(cre, cim, sk, out),
        "decrypt_to_eval": lambda: ctx.decrypt_to_eval(cre, sk, ev),   # not in the total (dec_ring_kernel alone)
    }
    for f in stages.values():   # warm-up (workspace, lazy tables)
        f()
    torch.cuda.synchronize()
    res = {"geometry": "n=64 (4096 slots per lane) x 512 W-lanes, L=11 reference moduli", "ctx_create_s": t_ctx}
    for name, f in stages.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        res[f"{name}_ms"] = e0.elapsed_time(e1) / reps
    res["encode_encrypt_decrypt_decode_ms"] = sum(res[f"{k}_ms"] for k in ("encode", "encrypt_pair", "decrypt_and_decode"))

    # the three stages back to back, eager and as one captured HIP graph (same kernels, same stream)
    def chain():
        stages["encode"]()
        stages["encrypt_pair"]()
        stages["decrypt_and_decode"]()
    for mode in ("eager", "graph"):
        if mode == "graph":
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                chain()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                chain()
            step = g.replay
        else:
            step = chain
        step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            step()
        e1.record()
        torch.cuda.synchronize()
        res[f"chain_{mode}_ms"] = e0.elapsed_time(e1) / reps
    err = float(np.max(np.abs(out.cpu().numpy().view(np.complex128) - msg)))
    res["max_err"] = err
    res["main_cu_check_1e-4"] = err < 1e-4
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
