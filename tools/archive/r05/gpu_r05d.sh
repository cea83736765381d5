#!/bin/bash
# r05d: L2 hand-off floor E sweep + the plan-5 (XL2) kernel's tests and first timing
set -o pipefail
O=gpurun_out
export PYTHONUNBUFFERED=1
( cd tools/microbench && timeout -k 10 120 ./l2_handoff_floor stress E 2 1 1 0 0 20 > ../../$O/r05d_stress.txt 2>&1 ) || exit $?
( cd tools/microbench && timeout -k 10 300 ./l2_handoff_floor sweep E > ../../$O/r05d_sweep.txt 2>&1 ) || exit $?
timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py -x -v --timeout 120 --timeout-method thread -k "xl2 and not stress" > $O/r05d_xl2_tests.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/xl2_rate.py 3 20 > $O/r05d_xl2_rate.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py -x -v --timeout 280 --timeout-method thread -k "xl2 and stress" > $O/r05d_xl2_stress.txt 2>&1 || exit $?
