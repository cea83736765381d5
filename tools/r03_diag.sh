#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-diag}
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 200 python tools/fused_diag.py 2 1,2 4,8,12 > "$OUT/diag2.txt" 2>&1; rc=$?
cat "$OUT/diag2.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/fused_diag.py 1 2,3 4,8,12 > "$OUT/diag1.txt" 2>&1; rc=$?
cat "$OUT/diag1.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 tools/microbench/twopass_floor > "$OUT/twopass_floor.txt" 2>&1; rc=$?
cat "$OUT/twopass_floor.txt"; exit $rc
