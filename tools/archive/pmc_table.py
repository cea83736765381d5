#!/usr/bin/env python3
"""Per-kernel mean of rocprofv3 counter_collection CSVs from tools/pmc_sq.sh passes. Dev tool.

usage: tools/pmc_table.py <dir> [kernel substring]
"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "ntt_pass_kernel"
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if sub not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].split("<", 1)[-1][:70]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print(k)
    for c in sorted(m):
        print(f"   {c:28s} {m[c]:.4e}")
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                  "SQ_ACTIVE_INST_ANY"):
            if c in m:
                print(f"   {c + '/WAVE_CYCLES':40s} {m[c] / wc:.3f}")
    if "SQ_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
        pass
