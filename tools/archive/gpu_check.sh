#!/bin/bash
# One gpurun session: GPU parity tests -> bench -> rocprofv3 kernel trace.
# Stops at the first crash / timeout (exit codes other than 0 and 1 from pytest).
# usage: tools/gpu_check.sh <tag> [pytest selection...]
set -u
TAG=${1:-run}
shift || true
SEL=${*:-tests}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"

timeout -k 10 900 python -u -m pytest $SEL -m gpu -v -rf --timeout 400 --durations 15 > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -25 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi

timeout -k 10 300 python bench.py --steps 10 --warmup 2 > "$OUT/bench.log" 2>&1 || { echo "bench failed rc=$?"; tail -20 "$OUT/bench.log"; exit 3; }
cat "$OUT/bench.log"

cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || { echo "rocprof failed rc=$?"; tail -20 "$OUT/prof.log"; exit 4; }
find "$OUT/prof" -name "*kernel_stats.csv" -exec cat {} \; | head -20
exit 0
