#!/bin/bash
# r05a: per-XCD L2 hand-off floor (tools/microbench/l2_handoff_floor): short stress check, then the sweep
set -o pipefail
cd tools/microbench
O=../../gpurun_out
timeout -k 10 120 ./l2_handoff_floor stress 2 1 2 18 0 20 > $O/r05a_stress.txt 2>&1 || exit $?
timeout -k 10 400 ./l2_handoff_floor sweep > $O/r05a_sweep.txt 2>&1 || exit $?
