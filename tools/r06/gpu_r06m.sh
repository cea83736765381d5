#!/bin/bash
# r06m: the per-lane XY product in one launch (MFHE_OPT_CGEMM_MFMA 2, gemm.hip xy_fused_kernel) vs two launches (3):
# HE parity tests, the pipeline A/B on one box, then a kernel trace of mode 2.
set -o pipefail
O=gpurun_out/${TAG:-r06m}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_he_gpu.py \
    > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for v in 2 3; do
    MFHE_CGEMM_MODE=$v timeout -k 10 120 python -u tools/pipeline_bench.py 20 > $O/pipe_${v}_$r.json 2>&1 || { echo "pipe $v rc=$?"; tail -5 $O/pipe_${v}_$r.json; exit 2; }
    python3 -c "import json,sys; d=json.loads(open('$O/pipe_${v}_$r.json').read().strip().splitlines()[-1]); print('cgemm=$v round $r', {k: round(v, 4) for k, v in d.items() if k.endswith('_ms')})"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$O/pipe_prof -o run --output-format csv -- \
    python3 $ROOT/tools/pipeline_bench.py 10 > $ROOT/$O/pipe_prof.log 2>&1 || { echo "prof rc=$?"; exit 3; }
grep -h -E "xy_fused|cgemm_mfma_kernel<0>" $ROOT/$O/pipe_prof/run_kernel_stats.csv | cut -d, -f1-4
echo done
