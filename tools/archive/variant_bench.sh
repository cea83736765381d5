#!/bin/bash
# A/B NTT timing of tuning-variant libraries (make BUILD=build_X LIB=libmfhe_X.so EXTRA=...).
# usage: tools/variant_bench.sh <tag> <variant>... ("base" = libmfhe.so).  Dev tool.
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
for v in "$@"; do
  if [ "$v" = base ]; then lib=$ROOT/matrix-fhe-gpu_amd/libmfhe.so; else lib=$ROOT/matrix-fhe-gpu_amd/libmfhe_$v.so; fi
  MFHE_LIB=$lib timeout -k 10 120 python "$ROOT/bench.py" --only ntt --steps 10 --warmup 2 --no-cpu-baseline \
      --recombine-batch 0 ${BENCH_ARGS:-} > "$OUT/$v.$rep.json" 2> "$OUT/$v.$rep.err" || { echo "$v failed"; tail -3 "$OUT/$v.$rep.err"; exit 3; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), 'inv', round(d['inverse_NTT_per_s']), 'frac', d['roofline']['frac'])" "$OUT/$v.$rep.json" "$v"
done
done
