#!/bin/bash
# r06j: decrypt_and_decode with the im chain forked after re's decrypt-fused digitize (MFHE_OPT_HE_STREAMS 4): HE / C4
# parity tests, then the pipeline A/B of modes 4 / 3 on one box, then a kernel trace of mode 4.
set -o pipefail
O=gpurun_out/${TAG:-r06j}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_he_gpu.py tests/test_c4_gpu.py \
    > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for v in 4 3; do
    MFHE_HE_STREAMS=$v timeout -k 10 120 python -u tools/pipeline_bench.py 20 > $O/pipe_${v}_$r.json 2>&1 || { echo "pipe $v rc=$?"; tail -5 $O/pipe_${v}_$r.json; exit 2; }
    python3 -c "import json,sys; d=json.loads(open('$O/pipe_${v}_$r.json').read().strip().splitlines()[-1]); print('streams=$v round $r', {k: round(v, 4) for k, v in d.items() if k.endswith('_ms')})"
  done
done
cd /tmp && export TMPDIR=/tmp
MFHE_HE_STREAMS=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$O/pipe_prof -o run --output-format csv -- \
    python3 $ROOT/tools/pipeline_bench.py 10 > $ROOT/$O/pipe_prof.log 2>&1 || { echo "prof rc=$?"; exit 3; }
echo done
