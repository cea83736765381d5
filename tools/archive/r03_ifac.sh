#!/bin/bash
# One gpurun session: HE / C4 / core-API GPU tests -> reference-geometry pipeline timing (W-CRT mode 1 = factored
# forward + inverse, mode 3 = dense) -> rocprofv3 kernel trace of mode 1.  usage: tools/r03_ifac.sh <tag>
set -u
TAG=${1:-r03f}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 500 python -u -m pytest tests/test_he_gpu.py tests/test_c4_gpu.py tests/test_core_api_gpu.py -x -v -rf \
    --timeout 200 --timeout-method thread > "$OUT/pytest_he.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_he.log"; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; grep -E "FAILED|Error|assert" "$OUT/pytest_he.log" | head -20; exit $rc; }
for m in 1 3 1 3; do
  MFHE_WCRT_MODE=$m timeout -k 10 150 python tools/pipeline_bench.py 20 > "$OUT/pipe_m$m.json" 2>&1 \
      || { echo "pipeline mode=$m failed"; tail -5 "$OUT/pipe_m$m.json"; exit 3; }
  echo "mode $m: $(tail -1 "$OUT/pipe_m$m.json")"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/kt1" -o run --output-format csv -- \
    python3 "$ROOT/tools/pipeline_bench.py" 5 > "$OUT/kt1.log" 2>&1 || { echo "kt failed rc=$?"; exit 4; }
echo "kernel trace done"
exit 0
