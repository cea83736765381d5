#!/bin/bash
# The headline's evidence in one gpurun session: GPU parity tests (optional) -> the driver's bench command ->
# rocprofv3 kernel trace of the same command's NTT part (tools/prof_agree.py: per-call kernel time vs the bench's
# HIP-event time) -> FETCH_SIZE / WRITE_SIZE passes, each in its own run, calibrated on known byte counts
# (tools/microbench/pmc_calib) -> tools/pmc_summary.py.  Every GPU step has its own time limit; the chain stops at
# the first failure.  Outputs: gpurun_out/<tag>/{bench.json, ntt_rocprof_vs_event.json, pmc_ntt_traffic.json,
# prof/.../run_kernel_stats.csv}; the round's copies under profiles/ are named <round>_*.
# usage: tools/profile_headline.sh <tag> [tests]
set -u
TAG=${1:-prof}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
STEPS=20
WARM=5

if [ "${2:-}" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread --durations 15 \
      > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  tail -5 "$OUT/pytest_gpu.log"
  [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
fi

timeout -k 10 400 python bench.py --gpus 1 --steps $STEPS --warmup $WARM > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed rc=$?"; tail -20 "$OUT/bench.err"; exit 3; }
python3 -c "import json,sys; d=json.load(open('$OUT/bench.json')); print({k: d[k] for k in ('value', 'ms_per_step')}, d['roofline']['frac'])"

cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --gpus 1 --steps $STEPS --warmup $WARM --only ntt --no-cpu-baseline \
    > "$OUT/prof.log" 2>&1 || { echo "rocprof failed rc=$?"; tail -20 "$OUT/prof.log"; exit 4; }
P=$(find "$OUT/prof" -name "run_kernel_trace.csv" | head -1)
python3 "$ROOT/tools/prof_agree.py" "$(dirname "$P")" "$OUT/prof.log" $STEPS $WARM "$OUT/ntt_rocprof_vs_event.json" \
    > "$OUT/prof_agree.out" 2>&1 || { echo "prof_agree failed"; tail -5 "$OUT/prof_agree.out"; exit 5; }
grep -E "ms_per_transform|kernel_over_event" "$OUT/prof_agree.out" || true

for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/pmc/calib_$C" -o run --output-format csv -- \
      "$ROOT/tools/microbench/pmc_calib" > "$OUT/calib_$C.log" 2>&1 || { echo "calib $C failed rc=$?"; exit 6; }
  timeout -s KILL 180 rocprofv3 --pmc $C -d "$OUT/pmc/ntt_$C" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --gpus 1 --only ntt --steps 2 --warmup 1 --no-cpu-baseline \
      > "$OUT/ntt_$C.log" 2>&1 || { echo "pmc $C failed rc=$?"; tail -5 "$OUT/ntt_$C.log"; exit 6; }
  echo "pmc $C done"
done
# rocprofv3 writes <dir>/<host>/<pid>/run_counter_collection.csv: flatten for pmc_summary
for D in calib_FETCH_SIZE calib_WRITE_SIZE ntt_FETCH_SIZE ntt_WRITE_SIZE; do
  F=$(find "$OUT/pmc/$D" -name "run_counter_collection.csv" | head -1)
  mkdir -p "$OUT/pmcflat/$D" && cp "$F" "$OUT/pmcflat/$D/run_counter_collection.csv"
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT/pmcflat" 3 3 $((16 * 65536 * 1024 * 8)) "$OUT/pmc_ntt_traffic.json" \
    65536 8 1024 "tools/profile_headline.sh (bench.py --only ntt --steps 2 --warmup 1)" > "$OUT/pmc_summary.out" 2>&1 \
    || { echo "pmc_summary failed"; tail -5 "$OUT/pmc_summary.out"; exit 7; }
grep -E "traffic_over" "$OUT/pmc_summary.out" || true
exit 0
