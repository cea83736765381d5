#!/bin/bash
# One gpurun session: W-CRT GEMM K-pipeline variants (MFHE_OPT_WCRT_PIPE 1 two-stage, 2 ring, 4 persistent ring): HE GPU tests -> reference-
# geometry pipeline timing per variant -> rocprofv3 kernel trace per variant -> one SQ counter pass per variant.
# usage: tools/r03_gemm.sh <tag>
set -u
TAG=${1:-r03g}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_he_gpu.py -x -v -rf --timeout 200 --timeout-method thread \
    > "$OUT/pytest_he.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_he.log"; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
for p in 1 2; do
  MFHE_WCRT_PIPE=$p timeout -k 10 150 python tools/pipeline_bench.py 20 > "$OUT/pipe$p.json" 2>&1 \
      || { echo "pipeline pipe=$p failed"; tail -5 "$OUT/pipe$p.json"; exit 3; }
  tail -1 "$OUT/pipe$p.json"
done
cd /tmp && export TMPDIR=/tmp
for p in 1 2; do
  MFHE_WCRT_PIPE=$p timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/kt$p" -o run --output-format csv -- \
      python3 "$ROOT/tools/pipeline_bench.py" 5 > "$OUT/kt$p.log" 2>&1 || { echo "kt pipe=$p failed rc=$?"; exit 4; }
  echo "kernel trace pipe=$p done"
done
for p in 1 2; do
  MFHE_WCRT_PIPE=$p timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
      SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d "$OUT/pmc$p" -o run \
      --output-format csv -- python3 "$ROOT/tools/pipeline_bench.py" 3 > "$OUT/pmc$p.log" 2>&1 \
      || { echo "pmc pipe=$p failed rc=$?"; exit 5; }
  echo "pmc pipe=$p done"
done
exit 0
