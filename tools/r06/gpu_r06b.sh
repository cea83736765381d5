#!/bin/bash
# r06b: world-1 recombine short-cut + compose-only flag (dist tests), W-CRT modulus sizes, C5 line with overlap_frac
set -o pipefail
O=gpurun_out
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_dist_gpu.py \
    tests/test_wcrt_sizes_gpu.py tests/test_c4_gpu.py > $O/r06b_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/r06b_tests.log; exit 1; }
tail -3 $O/r06b_tests.log
timeout -k 10 400 python -u bench.py --only c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/r06b_c5.json 2> $O/r06b_c5.err || { echo "c5 rc=$?"; tail -20 $O/r06b_c5.err; exit 2; }
tail -c 3000 $O/r06b_c5.json
