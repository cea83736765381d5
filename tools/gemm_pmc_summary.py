#!/usr/bin/env python3
"""Per-kernel sums of one rocprofv3 --pmc pass (counter_collection CSV): MFMA busy over SIMD-cycles
(SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)) and wait / LDS fractions of SQ_WAVE_CYCLES.
Dev tool.  usage: tools/gemm_pmc_summary.py <pmc dir> [kernel substring]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "gemm"
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sub not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].replace("void mfhe::", "")[:60]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for k, m in sorted(tot.items()):
    simd = m.get("GRBM_GUI_ACTIVE", 0) / 8 * 1024
    wc = m.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k}: dispatches {len(disp[k])}; MFMA busy / SIMD-cycles {m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / simd if simd else 0:.3f}; "
          f"wait_any/wave {m.get('SQ_WAIT_ANY', 0) / wc:.3f}; wait_lds/wave {m.get('SQ_WAIT_INST_LDS', 0) / wc:.3f}; "
          f"lds_active/wave {m.get('SQ_ACTIVE_INST_LDS', 0) / wc:.3f}; valu_active/wave {m.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f}")
