#!/bin/bash
# A/B timing of the C3 NTT (tools/u64_prof.py) across variant libraries, alternating, 3 rounds.
# usage: tools/r03_ab.sh <tag> <bits> <variant>... ("base" = libmfhe.so)
set -u
TAG=$1; BITS=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for rep in 1 2 3; do
for v in "$@"; do
  if [ "$v" = base ]; then lib=$ROOT/matrix-fhe-gpu_amd/libmfhe.so; else lib=$ROOT/matrix-fhe-gpu_amd/libmfhe_$v.so; fi
  NTTP_BITS=$BITS NTTP_SHAPE=${NTTP_SHAPE:-16,8,1024} MFHE_LIB=$lib timeout -k 10 120 python tools/u64_prof.py 10 > "$OUT/$v.$rep.json" 2>&1 \
      || { echo "$v failed"; tail -3 "$OUT/$v.$rep.json"; exit 3; }
  echo "$v $rep $(tail -1 "$OUT/$v.$rep.json")"
done
done
