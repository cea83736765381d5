#!/bin/bash
# A tuning-variant library (matrix-fhe-gpu_amd/libmfhe_<v>.so): NTT parity under MFHE_LIB, then bench.py --only ntt
# A/B against libmfhe.so, alternating, 2 rounds.  usage: tools/r03_variant.sh <tag> <variant>
set -u
TAG=$1; V=$2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/libmfhe_$V.so timeout -k 10 500 python -u -m pytest tests/test_ntt_gpu.py \
    tests/test_fullshape_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_$V.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_$V.log"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for v in base $V; do
  if [ $v = base ]; then lib=$ROOT/matrix-fhe-gpu_amd/libmfhe.so; else lib=$ROOT/matrix-fhe-gpu_amd/libmfhe_$v.so; fi
  MFHE_LIB=$lib timeout -k 10 150 python bench.py --only ntt --steps 20 --warmup 5 --no-cpu-baseline \
      > "$OUT/$v.$rep.json" 2> "$OUT/$v.$rep.err" || { echo "bench $v failed"; tail -3 "$OUT/$v.$rep.err"; exit 3; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), 'inv', round(d['inverse_NTT_per_s']), 'ratio', d['inverse_over_forward'])" "$OUT/$v.$rep.json" $v
done
done
