#!/bin/bash
# r06h: the encrypt's ring kernel with the noise GEMM fused in (MFHE_OPT_ENC_E_SMALL 2): HE parity tests, then the
# pipeline A/B of options 2 / 1 on one box (tools/pipeline_bench.py), then a kernel trace of the default pipeline.
set -o pipefail
O=gpurun_out/${TAG:-r06h}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_he_gpu.py tests/test_c4_gpu.py \
    > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for v in 2 1; do
    MFHE_ENC_E_SMALL=$v timeout -k 10 120 python -u tools/pipeline_bench.py 20 > $O/pipe_${v}_$r.json 2>&1 || { echo "pipe $v rc=$?"; tail -5 $O/pipe_${v}_$r.json; exit 2; }
    python3 -c "import json,sys; d=json.loads(open('$O/pipe_${v}_$r.json').read().strip().splitlines()[-1]); print('e_small=$v round $r', {k: round(v, 4) for k, v in d.items() if k.endswith('_ms')})"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$O/pipe_prof -o run --output-format csv -- \
    python3 $ROOT/tools/pipeline_bench.py 10 > $ROOT/$O/pipe_prof.log 2>&1 || { echo "prof rc=$?"; exit 3; }
grep -h -E "smallb|enc_ring|gaussian_i8" $ROOT/$O/pipe_prof/run_kernel_stats.csv | cut -d, -f1-4
echo done
