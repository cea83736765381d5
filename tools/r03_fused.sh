#!/bin/bash
# Fused NTT with the LDS-DMA prefetch (MFHE_OPT_NTT_FUSED = 2): parity first, then the wg x lag sweep beside the
# two-pass default.  usage: tools/r03_fused.sh <tag>
set -u
TAG=${1:-fdb}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 "$OUT/pytest_gpu.log"; exit 2; }
tail -3 "$OUT/pytest_gpu.log"
FUSED_MODE=2 FUSED_WGS=1,2 FUSED_LAGS=2,3,4,6,8,12 timeout -k 10 300 python tools/fused_sweep.py 16,8,1024 \
    > "$OUT/sweep2.txt" 2>&1 || { echo "sweep failed rc=$?"; tail -5 "$OUT/sweep2.txt"; exit 4; }
cat "$OUT/sweep2.txt"
FUSED_MODE=1 FUSED_WGS=2 FUSED_LAGS=4,6 timeout -k 10 300 python tools/fused_sweep.py 16,8,1024 \
    > "$OUT/sweep1.txt" 2>&1 || { echo "sweep1 failed rc=$?"; exit 5; }
cat "$OUT/sweep1.txt"
timeout -k 10 200 python bench.py --only ntt --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_twopass.json" 2>/dev/null \
    || { echo "bench failed"; exit 6; }
python3 -c "import json;d=json.load(open('$OUT/bench_twopass.json'));print('two-pass', d['value'], d['inverse_NTT_per_s'])"
