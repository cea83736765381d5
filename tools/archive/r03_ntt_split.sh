#!/bin/bash
# One gpurun session: per-kernel split of the C3 NTT on the U64 path (60-bit primes) and the FP64 inverse.
# usage: tools/r03_ntt_split.sh <tag>
set -u
TAG=${1:-r03s}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 120 python tools/u64_prof.py 10 > "$OUT/u64_pf2.json" 2>&1 || { tail -5 "$OUT/u64_pf2.json"; exit 3; }
tail -1 "$OUT/u64_pf2.json"
timeout -k 10 120 python tools/u64_prof.py 10 0 > "$OUT/u64_pf0.json" 2>&1 || { tail -5 "$OUT/u64_pf0.json"; exit 3; }
tail -1 "$OUT/u64_pf0.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/kt_u64" -o run --output-format csv -- \
    python3 "$ROOT/tools/u64_prof.py" 10 > "$OUT/kt_u64.log" 2>&1 || { echo "kt u64 failed"; exit 4; }
NTTP_BITS=50 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/kt_f64" -o run --output-format csv -- \
    python3 "$ROOT/tools/u64_prof.py" 10 > "$OUT/kt_f64.log" 2>&1 || { echo "kt f64 failed"; exit 4; }
echo traces done
exit 0
