#!/bin/bash
# r06d: the encrypt noise's small-operand W-CRT GEMM (MFHE_OPT_ENC_E_SMALL): HE parity tests, then the pipeline A/B
# (tools/pipeline_bench.py, the option alternating 1 / 0 on one box), then a kernel trace of the default pipeline
set -o pipefail
O=gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_he_gpu.py tests/test_c4_gpu.py \
    > $O/r06d_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/r06d_tests.log; exit 1; }
tail -2 $O/r06d_tests.log
for r in 1 2 3; do
  for v in 1 0; do
    MFHE_ENC_E_SMALL=$v timeout -k 10 120 python -u tools/pipeline_bench.py 20 > $O/r06d_pipe_${v}_$r.json 2>&1 || { echo "pipe $v rc=$?"; tail -5 $O/r06d_pipe_${v}_$r.json; exit 2; }
    python3 -c "import json,sys; d=json.loads(open('$O/r06d_pipe_${v}_$r.json').read().strip().splitlines()[-1]); print('e_small=$v round $r', {k: round(v, 4) for k, v in d.items() if k.endswith('_ms')})"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$O/r06d_pipe_prof -o run --output-format csv -- \
    python3 $ROOT/tools/pipeline_bench.py 10 > $ROOT/$O/r06d_pipe_prof.log 2>&1 || { echo "prof rc=$?"; exit 3; }
echo done
