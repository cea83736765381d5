#!/bin/bash
# A/B of the two-pass chunk size (MFHE_OPT_NTT_CHUNK_BYTES) on the C3 headline, alternating, two rounds.  Dev tool.
# usage: tools/chunk_ab.sh <tag> <MiB>...
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
for m in "$@"; do
  timeout -k 10 120 python "$ROOT/bench.py" --only ntt --steps 20 --warmup 5 --no-cpu-baseline --recombine-batch 0 \
      --ntt-chunk $((m * 1048576)) > "$OUT/$m.$rep.json" 2> "$OUT/$m.$rep.err" || { echo "$m failed"; tail -3 "$OUT/$m.$rep.err"; exit 3; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('chunk_MiB', sys.argv[2], round(d['value']), 'inv', round(d['inverse_NTT_per_s']), 'frac', d['roofline']['frac'])" "$OUT/$m.$rep.json" "$m"
done
done
