#!/bin/bash
# r06c: lazy U60 inverse parity (modulus sweep, U60 tests, full-shape digests), W-CRT sizes, dist / C4, then the C5 line
# (overlap_frac) and the U64 line (U60 vs Harvey, both directions)
set -o pipefail
O=gpurun_out
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_modsize_sweep_gpu.py \
    tests/test_ntt_gpu.py tests/test_wcrt_sizes_gpu.py tests/test_dist_gpu.py tests/test_c4_gpu.py \
    "tests/test_fullshape_gpu.py::test_c3_60bit_primes_full_shape" "tests/test_fullshape_gpu.py::test_c3_full_shape" \
    > $O/r06c_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/r06c_tests.log; exit 1; }
tail -3 $O/r06c_tests.log
timeout -k 10 300 python -u bench.py --only u64 --steps 2 --warmup 1 --no-cpu-baseline > $O/r06c_u64.json 2> $O/r06c_u64.err || { echo "u64 rc=$?"; tail -20 $O/r06c_u64.err; exit 2; }
tail -c 1500 $O/r06c_u64.json
timeout -k 10 400 python -u bench.py --only c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/r06c_c5.json 2> $O/r06c_c5.err || { echo "c5 rc=$?"; tail -20 $O/r06c_c5.err; exit 3; }
tail -c 3000 $O/r06c_c5.json
