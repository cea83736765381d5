#!/usr/bin/env python3
"""Print the headline-trace and traffic sentences DESIGN.md §3.1 / §6 quote, straight from the committed profiles
(a DESIGN number that cites a profiles/ file must be that file's number).  The latest round's
files are used unless a round is given:

    python3 tools/design_numbers.py [rNN]

tests/test_design_numbers.py checks that DESIGN.md contains exactly these sentences."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PROF = ROOT / "profiles"


def latest(pattern):
    files = sorted(PROF.glob(pattern))
    return files[-1] if files else None


def trace_sentence(path=None):
    path = Path(path) if path else latest("r*_ntt_rocprof_vs_event.json")
    d = json.loads(path.read_text())
    col = blk = None
    for k, v in d["per_kernel"].items():
        if "ntt_col_db_kernel" in k:
            col = v["avg_us"]
        elif "ntt_pass_kernel" in k:
            blk = v["avg_us"]
    s = (f"`profiles/{path.name}`: {d['rocprof_kernel_ms_per_transform']:.4f} ms of kernels per call against "
         f"{d['bench_event_ms_per_transform']:.4f} ms by events (kernel/event {d['kernel_over_event']:.4f})")
    if col is not None and blk is not None:
        s += f", column pass {col:.2f} µs, block pass {blk:.2f} µs per chunk"
    return s


def traffic_sentence(path=None):
    path = Path(path) if path else latest("r*_pmc_ntt_traffic.json")
    d = json.loads(path.read_text())
    return (f"`profiles/{path.name}`: {d['fwd_traffic_over_algorithmic']:.3f} × the algorithmic bytes forward, "
            f"{d['inv_traffic_over_algorithmic']:.3f} × inverse")


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else None
    tr = PROF / f"{rnd}_ntt_rocprof_vs_event.json" if rnd else None
    pm = PROF / f"{rnd}_pmc_ntt_traffic.json" if rnd else None
    print(trace_sentence(tr))
    print(traffic_sentence(pm))


if __name__ == "__main__":
    main()
