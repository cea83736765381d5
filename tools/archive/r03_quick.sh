#!/bin/bash
# One gpurun session: GPU parity tests, then the U64 C3 timing (60-bit primes) and the FP64 C3 timing.
# usage: tools/r03_quick.sh <tag> [skip-tests]
set -u
TAG=${1:-r03q}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread --durations 10 \
      > "$OUT/pytest_gpu.log" 2>&1; rc=$?
  tail -4 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
fi
timeout -k 10 120 python tools/u64_prof.py 10 > "$OUT/u64.json" 2>&1 || { tail -5 "$OUT/u64.json"; exit 3; }
tail -1 "$OUT/u64.json"
NTTP_BITS=50 timeout -k 10 120 python tools/u64_prof.py 10 > "$OUT/f64.json" 2>&1 || { tail -5 "$OUT/f64.json"; exit 3; }
tail -1 "$OUT/f64.json"
