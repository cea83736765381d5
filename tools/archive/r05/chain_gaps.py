#!/usr/bin/env python3
"""Inter-kernel idle time in one iteration of the pipeline chain (encode -> encrypt_pair -> decrypt_and_decode) from a
rocprofv3 kernel trace of tools/pipeline_bench.py: the iteration before the chain's last one in the eager section,
kernel by kernel, with the idle gap before each (negative = overlaps the previous kernel) and the iteration's busy
(union of kernel intervals) vs span.  usage: tools/r05/chain_gaps.py <trace dir>"""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/run_kernel_trace.csv", recursive=True)[0]
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f)))
names = [n for _, _, n in rows]
# the eager chain section: the 12 iterations (1 warm + 10 timed + ...) before the graph capture; an iteration starts at
# the encode's first XY-IDFT GEMM (cgemm<0> followed by cgemm<0> then cwdft_inv_dots)
starts = [i for i in range(len(rows) - 2) if "cwdft_inv_dots" in names[i + 2] and "cgemm_mfma_kernel<0>" in names[i]
          and "cgemm_mfma_kernel<0>" in names[i + 1]]
# pick the third-to-last eager iteration: starts are encode beginnings across all sections; the chain section comes
# after the per-stage loops, so take a start whose next start is also an encode start 1 iteration later
a, b = starts[-14], starts[-13]
seg = rows[a:b]
t0, t1 = seg[0][0], seg[-1][1]
busy, cs, ce = 0, None, None
prev_end = t0
for s, e, n in seg:
    print(f"{(s - prev_end) / 1e3:8.1f} gap {(e - s) / 1e3:8.1f} us  {n[:70]}")
    prev_end = max(prev_end, e)
    if ce is None or s > ce:
        if ce is not None:
            busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
print(f"iteration: {len(seg)} kernels, span {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us")
