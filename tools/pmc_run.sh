#!/bin/bash
# rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs, MI355X_MICROARCH.md "rocprofv3 PMC
# slots"): first the calibration copy kernels (known bytes), then the NTT bench.  No trace domains are
# combined with --pmc.  usage: tools/pmc_run.sh <tag>
set -u
TAG=${1:-pmc}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
[ -x "$ROOT/tools/microbench/pmc_calib" ] || { echo "build tools/microbench/pmc_calib first (hipcc, in this container)"; exit 2; }
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $C -d "$OUT/calib_$C" -o run --output-format csv -- \
      "$ROOT/tools/microbench/pmc_calib" > "$OUT/calib_$C.log" 2>&1 || { echo "calib $C failed rc=$?"; tail -5 "$OUT/calib_$C.log"; exit 3; }
  echo "calib $C done"
  timeout -k 10 300 rocprofv3 --pmc $C -d "$OUT/ntt_$C" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --only ntt --steps 2 --warmup 1 --no-cpu-baseline --recombine-batch 0 > "$OUT/ntt_$C.log" 2>&1 || { echo "ntt $C failed rc=$?"; tail -5 "$OUT/ntt_$C.log"; exit 4; }
  echo "ntt $C done"
done
exit 0
