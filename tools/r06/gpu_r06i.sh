#!/bin/bash
# r06i: HE / C4 parity tests and the reference-geometry pipeline (two rounds) plus its kernel trace, for a build check.
set -o pipefail
O=gpurun_out/${TAG:-r06i}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_he_gpu.py tests/test_c4_gpu.py \
    > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  timeout -k 10 120 python -u tools/pipeline_bench.py 20 > $O/pipe_$r.json 2>&1 || { echo "pipe rc=$?"; tail -5 $O/pipe_$r.json; exit 2; }
  python3 -c "import json,sys; d=json.loads(open('$O/pipe_$r.json').read().strip().splitlines()[-1]); print('round $r', {k: round(v, 4) for k, v in d.items() if k.endswith('_ms')})"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$O/pipe_prof -o run --output-format csv -- \
    python3 $ROOT/tools/pipeline_bench.py 10 > $ROOT/$O/pipe_prof.log 2>&1 || { echo "prof rc=$?"; exit 3; }
echo done
