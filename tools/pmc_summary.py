#!/usr/bin/env python3
"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/pmc_run.sh) into per-transform HBM bytes.

Corrections (MI355X_MICROARCH.md §HBM, confirmed by tools/microbench/pmc_calib.hip on this box):
counters are in KiB; FETCH_SIZE reports exactly half of the bytes read by coalesced 8 B/lane and
16 B/lane streaming loads, so it is doubled; WRITE_SIZE is exact.  Memory-side counters include
Infinity-Cache hits, so "traffic" is L2<->fabric bytes (HBM + MALL).

usage: tools/pmc_summary.py <pmc dir> <fwd transforms> <inv transforms> <algorithmic bytes/transform> <out.json>
       [N L batch [command]]   (the shape bench.py measured; bench.py only uses a file whose config matches its run)
"""
import collections
import csv
import json
import sys
from pathlib import Path


def load(path):
    agg = collections.defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(path)):
        a = agg[r["Kernel_Name"]]
        a[0] += float(r["Counter_Value"])
        a[1] += 1
    return agg


def main():
    d = Path(sys.argv[1])
    nf, ni, alg = int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4])
    fetch = load(d / "ntt_FETCH_SIZE" / "run_counter_collection.csv")
    write = load(d / "ntt_WRITE_SIZE" / "run_counter_collection.csv")
    cf = load(d / "calib_FETCH_SIZE" / "run_counter_collection.csv")
    cw = load(d / "calib_WRITE_SIZE" / "run_counter_collection.csv")
    calib = {}
    for k in cf:
        if k.startswith("copy"):
            name = k.split("(")[0]
            calib[name] = {"known_bytes": 2 ** 31, "fetch_kib_raw": cf[k][0] / cf[k][1],
                           "write_kib": cw[k][0] / cw[k][1],
                           "fetch_ratio_raw": cf[k][0] / cf[k][1] * 1024 / 2 ** 31,
                           "write_ratio": cw[k][0] / cw[k][1] * 1024 / 2 ** 31}
    kernels = {}
    tot = {"fwd": [0.0, 0.0], "inv": [0.0, 0.0]}
    for k in fetch:
        if "ntt_col_db_kernel" in k:
            targs = [a.strip() for a in k.split("<", 1)[1].split(">(")[0].split(",")]
            inv = len(targs) >= 3 and targs[2] == "true"   # <A, TS, INV>: the inverse's last pass
        elif "ntt_pass_kernel" in k:
            inv = k.split("<")[1].split(",")[6].strip() == "true"   # template arg INV
        else:
            continue
        rb = fetch[k][0] * 2 * 1024          # corrected read bytes, all dispatches
        wb = write[k][0] * 1024
        kernels[k] = {"dispatches": fetch[k][1], "read_bytes_per_dispatch": rb / fetch[k][1],
                      "write_bytes_per_dispatch": wb / write[k][1], "inverse": inv}
        t = tot["inv" if inv else "fwd"]
        t[0] += rb
        t[1] += wb
    out = {}
    if len(sys.argv) > 8:
        out["config"] = {"N": int(sys.argv[6]), "limbs": int(sys.argv[7]), "batch": int(sys.argv[8]),
                         "command": sys.argv[9] if len(sys.argv) > 9 else
                         "tools/pmc_run.sh (bench.py --only ntt --steps 2 --warmup 1)"}
    out.update({"calibration": calib, "kernels": kernels, "algorithmic_bytes_per_transform": alg})
    for key, n in (("fwd", nf), ("inv", ni)):
        r, w = tot[key][0] / n, tot[key][1] / n
        out[f"{key}_traffic_bytes_per_transform"] = r + w
        out[f"{key}_read_bytes_per_transform"] = r
        out[f"{key}_write_bytes_per_transform"] = w
        out[f"{key}_traffic_over_algorithmic"] = (r + w) / alg
    json.dump(out, open(sys.argv[5], "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k not in ("kernels",)}, indent=1))


if __name__ == "__main__":
    main()
