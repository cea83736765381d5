#!/bin/bash
# One gpurun session (round 3): GPU parity tests -> the driver's bench command -> rocprofv3 kernel trace of the
# same command (NTT part) -> FETCH_SIZE / WRITE_SIZE passes with the same steps.  Every GPU step has its own
# time limit and the chain stops at the first failure.
# usage: tools/r03_check.sh <tag> [skip-tests]
set -u
TAG=${1:-r03}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
STEPS=20
WARM=5

if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread --durations 15 \
      > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  tail -5 "$OUT/pytest_gpu.log"
  [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
fi

timeout -k 10 400 python bench.py --gpus 1 --steps $STEPS --warmup $WARM > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed rc=$?"; tail -20 "$OUT/bench.err"; exit 3; }
cat "$OUT/bench.json"

cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --gpus 1 --steps $STEPS --warmup $WARM --only ntt --no-cpu-baseline \
    > "$OUT/prof.log" 2>&1 || { echo "rocprof failed rc=$?"; tail -20 "$OUT/prof.log"; exit 4; }
P=$(find "$OUT/prof" -name "run_kernel_trace.csv" | head -1)
python3 "$ROOT/tools/prof_agree.py" "$(dirname "$P")" "$OUT/prof.log" $STEPS $WARM "$OUT/ntt_rocprof_vs_event.json" \
    > "$OUT/prof_agree.out" 2>&1 || { echo "prof_agree failed"; tail -5 "$OUT/prof_agree.out"; exit 5; }
grep -E "ms_per_transform|kernel_over_event" "$OUT/prof_agree.out" || true

for C in FETCH_SIZE WRITE_SIZE; do
  if [ -x "$ROOT/tools/microbench/pmc_calib" ]; then
    timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/calib_$C" -o run --output-format csv -- \
        "$ROOT/tools/microbench/pmc_calib" > "$OUT/calib_$C.log" 2>&1 || { echo "calib $C failed rc=$?"; exit 6; }
  fi
  timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/ntt_$C" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --gpus 1 --only ntt --steps $STEPS --warmup $WARM --no-cpu-baseline \
      > "$OUT/ntt_$C.log" 2>&1 || { echo "pmc $C failed rc=$?"; tail -5 "$OUT/ntt_$C.log"; exit 6; }
  echo "pmc $C done"
done
exit 0
