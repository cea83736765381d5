#!/bin/bash
# One gpurun session: block-pass DMA (MFHE_OPT_NTT_PREFETCH = 3) parity, then bench A/B prefetch 2 vs 3.
set -u
TAG=${1:-r03b}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_ntt_gpu.py tests/test_fullshape_gpu.py -m gpu -x -v -rf --timeout 200 \
    --timeout-method thread -k "dma or c3_full_shape" > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && { grep -E "Error|assert" "$OUT/pytest.log" | head -20; exit $rc; }
for rep in 1 2; do
for pf in 2 3; do
  timeout -k 10 150 python bench.py --only ntt --steps 20 --warmup 5 --no-cpu-baseline --ntt-prefetch $pf \
      > "$OUT/pf$pf.$rep.json" 2> "$OUT/pf$pf.$rep.err" || { echo "bench pf=$pf failed"; tail -3 "$OUT/pf$pf.$rep.err"; exit 3; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('pf', sys.argv[2], round(d['value']), 'inv', round(d['inverse_NTT_per_s']), 'ratio', d['inverse_over_forward'])" "$OUT/pf$pf.$rep.json" $pf
done
done
