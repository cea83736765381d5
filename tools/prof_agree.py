#!/usr/bin/env python3
"""Check the bench's HIP-event time per forward transform against rocprofv3's kernel trace of the same
command (tools/gpu_check.sh: bench.py --steps S --warmup W under --kernel-trace --stats).

One mfhe_ntt_fwd call at the bench shape = C chunks x (column pass + block pass) launches.  The bench
runs its forward calls first (W warm-up + S timed), so the first (W + S) * 2C forward-pass dispatches
in timestamp order are those calls.  Reports per-call kernel time (sum of its dispatch durations) and
wall span (first start -> last end), and the bench's own event time from the same run.

usage: tools/prof_agree.py <prof dir> <prof.log> <steps> <warmup> <out.json>
"""
import csv
import json
import statistics
import sys
from pathlib import Path


def main():
    d, log, S, W, out = Path(sys.argv[1]), sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    bench = next(json.loads(l) for l in open(log) if l.startswith("{"))
    rows = [r for r in csv.DictReader(open(d / "run_kernel_trace.csv"))
            if "ntt_pass_kernel" in r["Kernel_Name"] or "ntt_col_db_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # forward pass kernels: the DMA-prefetch column pass (forward only), and ntt_pass_kernel with template
    # argument INV (7th) == false
    fwd = [r for r in rows if "ntt_col_db_kernel" in r["Kernel_Name"]
           or r["Kernel_Name"].split("<")[1].split(",")[6].strip() == "false"]
    N, L, B = bench["config"]["N"], bench["config"]["limbs"], bench["config"]["batch_per_gpu"]
    # chunks per call as the bench reports them ("mfhe_ntt_fwd call = C chunks x ..."), i.e. from the context's
    # MFHE_OPT_NTT_CHUNK_BYTES
    import re
    C = int(re.search(r"= (\d+) chunks", bench["roofline"]["kernel"]).group(1))
    per = 2 * C
    calls = [fwd[i * per:(i + 1) * per] for i in range(W + S)][W:]
    kern_ms = [sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in c) / 1e6 for c in calls]
    span_ms = [(int(c[-1]["End_Timestamp"]) - int(c[0]["Start_Timestamp"])) / 1e6 for c in calls]
    names = sorted({r["Kernel_Name"] for c in calls for r in c})
    per_kernel = {}
    for n in names:
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for c in calls for r in c if r["Kernel_Name"] == n]
        per_kernel[n] = {"dispatches_in_timed_calls": len(durs), "avg_us": statistics.mean(durs) / 1e3}
    res = {
        "shape": {"N": N, "limbs": L, "batch": B, "chunks_per_call": C, "launches_per_call": per},
        "bench_event_ms_per_transform": bench["roofline"]["event_ms_per_transform"],
        "rocprof_kernel_ms_per_transform": statistics.mean(kern_ms),
        "rocprof_span_ms_per_transform": statistics.mean(span_ms),
        "kernel_over_event": statistics.mean(kern_ms) / bench["roofline"]["event_ms_per_transform"],
        "per_kernel": per_kernel,
        "note": "span - kernel time = dispatch gaps between the call's launches; bench event time brackets the "
                "whole call on the launch stream",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
