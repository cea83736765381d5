#!/bin/bash
# One gpurun session: fused-NTT stress (mode 1; small and C3 shapes) -> GPU
# parity tests -> bench (all lines, incl. the U64 C3 line) -> two-pass floor microbenchmark.  Each GPU step has
# its own limit; stop at the first failure.
# usage: tools/r03_u64.sh <tag>
set -u
TAG=${1:-r03u}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for M in 1; do
  FD_BATCH=9 FD_L=4 timeout -k 10 150 python tools/fused_diag.py $M 2 7,4 0 300 > "$OUT/stress_small_m$M.txt" 2>&1; rc=$?
  cat "$OUT/stress_small_m$M.txt"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 python tools/fused_diag.py $M 2 6,12 20 100 > "$OUT/stress_c3_m$M.txt" 2>&1; rc=$?
  cat "$OUT/stress_c3_m$M.txt"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread --durations 15 \
    > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -5 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed rc=$?"; tail -20 "$OUT/bench.err"; exit 3; }
cat "$OUT/bench.json"
timeout -k 10 120 tools/microbench/twopass_floor > "$OUT/twopass_floor.txt" 2>&1; rc=$?
cat "$OUT/twopass_floor.txt"; exit $rc
