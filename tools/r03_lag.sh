#!/bin/bash
# Which fused plan fails at a long lag (tools/fused_sweep.py reported ok=false at mode 2, lag 8 / 12).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-lag}
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_fullshape_gpu.py -m gpu -v -k "long_lag" --timeout 200 \
    --timeout-method thread > "$OUT/pytest_lag.log" 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|assert" "$OUT/pytest_lag.log" | head -40
exit $rc
