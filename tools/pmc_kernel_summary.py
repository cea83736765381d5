#!/usr/bin/env python3
"""Per-kernel SQ counter summary over one or more rocprofv3 --pmc passes (counter_collection CSVs).

Prints, per kernel name containing the substring: dispatches, average duration, and for each counter its per-dispatch
average. Then the derived figures:
* VALU instructions per wave (SQ_INSTS_VALU / SQ_WAVES);
* per-wave fractions of SQ_WAVE_CYCLES: VALU active, wait_any (s_waitcnt / barrier parked), wait_inst_any (issue
  stall), any instruction active;
* SIMD VALU busy = 4 SQ_ACTIVE_INST_VALU / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs). SQ_ACTIVE_INST_* and
  SQ_WAVE_CYCLES count quad-cycles (MI355X_MICROARCH.md).
Dev tool. usage: tools/pmc_kernel_summary.py <kernel substring> <pmc dir> [<pmc dir> ...]"""
import collections
import csv
import glob
import sys

sub = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
nd = collections.defaultdict(lambda: collections.defaultdict(set))
dur = collections.defaultdict(dict)
for d in sys.argv[2:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if sub not in r["Kernel_Name"]:
                continue
            k = r["Kernel_Name"].replace("void mfhe::", "")[:70]
            c = r["Counter_Name"]
            key = (f, r["Dispatch_Id"])
            tot[k][c] += float(r["Counter_Value"])
            nd[k][c].add(key)
            dur[k][key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for k, m in sorted(tot.items()):
    avg = {c: v / max(1, len(nd[k][c])) for c, v in m.items()}
    ds = list(dur[k].values())
    print(f"## {k}: dispatches (per pass) {max(len(s) for s in nd[k].values())}, avg duration {sum(ds) / len(ds):.1f} us")
    for c in sorted(avg):
        print(f"  {c:28s} {avg[c]:.4g}")
    wc = avg.get("SQ_WAVE_CYCLES", 0) or float("nan")
    der = []
    if "SQ_INSTS_VALU" in avg and avg.get("SQ_WAVES"):
        der.append(f"VALU instructions / wave {avg['SQ_INSTS_VALU'] / avg['SQ_WAVES']:.0f}")
    for c, lab in (("SQ_ACTIVE_INST_VALU", "valu_active"), ("SQ_WAIT_ANY", "wait_any"),
                   ("SQ_WAIT_INST_ANY", "wait_inst_any"), ("SQ_ACTIVE_INST_ANY", "active_any"),
                   ("SQ_ACTIVE_INST_LDS", "lds_active"), ("SQ_ACTIVE_INST_SCA", "scalar_active")):
        if c in avg:
            der.append(f"{lab}/wave {avg[c] / wc:.3f}")
    if "SQ_ACTIVE_INST_VALU" in avg and avg.get("GRBM_GUI_ACTIVE"):
        der.append(f"SIMD VALU busy {4 * avg['SQ_ACTIVE_INST_VALU'] / (avg['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
    print("  derived: " + "; ".join(der))
