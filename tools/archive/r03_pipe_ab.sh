#!/bin/bash
# HE GPU tests under a variant library, then reference-geometry pipeline timing + kernel trace, base vs variant.
# usage: tools/r03_pipe_ab.sh <tag> <variant>   (matrix-fhe-gpu_amd/libmfhe_<variant>.so)
set -u
TAG=$1; V=$2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/libmfhe_$V.so timeout -k 10 400 python -u -m pytest tests/test_he_gpu.py tests/test_c4_gpu.py -x -q \
    --timeout 200 --timeout-method thread > "$OUT/pytest_$V.log" 2>&1; rc=$?
echo "$V parity: $(tail -1 "$OUT/pytest_$V.log")"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
for v in base $V; do
  if [ $v = base ]; then lib=$ROOT/matrix-fhe-gpu_amd/libmfhe.so; else lib=$ROOT/matrix-fhe-gpu_amd/libmfhe_$v.so; fi
  MFHE_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/kt_${v}_$rep" -o run --output-format csv -- \
      python3 "$ROOT/tools/pipeline_bench.py" 10 > "$OUT/pipe_${v}_$rep.json" 2>&1 || { echo "$v failed"; exit 3; }
  echo "$v $rep done"
done
done
