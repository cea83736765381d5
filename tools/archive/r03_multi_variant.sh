#!/bin/bash
# NTT parity for each variant library (matrix-fhe-gpu_amd/libmfhe_<v>.so, under MFHE_LIB), then bench.py --only ntt
# A/B of base + variants, alternating, 2 rounds, 20 steps / 5 warm-up.  usage: tools/r03_multi_variant.sh <tag> <variant>...
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for V in "$@"; do
  MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/libmfhe_$V.so timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py \
      tests/test_fullshape_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
      > "$OUT/pytest_$V.log" 2>&1; rc=$?
  echo "$V parity: $(tail -1 "$OUT/pytest_$V.log")"; [ $rc -ne 0 ] && exit $rc
done
for rep in 1 2; do
for v in base "$@"; do
  if [ $v = base ]; then lib=$ROOT/matrix-fhe-gpu_amd/libmfhe.so; else lib=$ROOT/matrix-fhe-gpu_amd/libmfhe_$v.so; fi
  MFHE_LIB=$lib timeout -k 10 150 python bench.py --only ntt --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} \
      > "$OUT/$v.$rep.json" 2> "$OUT/$v.$rep.err" || { echo "bench $v failed"; tail -3 "$OUT/$v.$rep.err"; exit 3; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), 'inv', round(d['inverse_NTT_per_s']), 'ratio', d['inverse_over_forward'])" "$OUT/$v.$rep.json" $v
done
done
