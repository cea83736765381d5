#!/bin/bash
# r06k: a build A/B on one box: HE / C4 parity tests on the current build, then tools/pipeline_bench.py alternating
# libmfhe.so and $LIBB (a copy of the previous build, MFHE_LIB), then a kernel trace of the current build.
set -o pipefail
O=gpurun_out/${TAG:-r06k}
LIBB=${LIBB:-libmfhe_prev.so}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_he_gpu.py tests/test_c4_gpu.py ${EXTRA_TESTS:-} \
    > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for lib in libmfhe.so $LIBB; do
    MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$lib timeout -k 10 120 python -u tools/pipeline_bench.py 20 > $O/pipe_${lib}_$r.json 2>&1 || { echo "pipe $lib rc=$?"; tail -5 $O/pipe_${lib}_$r.json; exit 2; }
    python3 -c "import json,sys; d=json.loads(open('$O/pipe_${lib}_$r.json').read().strip().splitlines()[-1]); print('$lib round $r', {k: round(v, 4) for k, v in d.items() if k.endswith('_ms')})"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$O/pipe_prof -o run --output-format csv -- \
    python3 $ROOT/tools/pipeline_bench.py 10 > $ROOT/$O/pipe_prof.log 2>&1 || { echo "prof rc=$?"; exit 3; }
echo done
