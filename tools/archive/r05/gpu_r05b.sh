#!/bin/bash
# r05b: L2 hand-off floor, schedule E (LDS-DMA pipelined): stress check, then the E sweep
set -o pipefail
cd tools/microbench
O=../../gpurun_out
timeout -k 10 120 ./l2_handoff_floor stress E 2 1 1 0 0 20 > $O/r05b_stress.txt 2>&1 || exit $?
timeout -k 10 400 ./l2_handoff_floor sweep E > $O/r05b_sweep.txt 2>&1 || exit $?
