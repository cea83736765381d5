#!/bin/bash
# r06v: an experimental build (matrix-fhe-gpu_amd/$LIBX, default libmfhe_exp.so) against the tree's libmfhe.so:
# parity tests run ON the experimental build (MFHE_LIB), then tools/pipeline_bench.py alternating the two, then a
# kernel trace of the experimental build (BASE: the build compared against, default the tree's libmfhe.so).  The
# tree's libmfhe.so stays the one its sources build.
set -o pipefail
O=gpurun_out/${TAG:-r06v}
LIBX=${LIBX:-libmfhe_exp.so}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $O
export PYTHONUNBUFFERED=1
MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$LIBX timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
    tests/test_he_gpu.py tests/test_c4_gpu.py ${EXTRA_TESTS:-} > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for lib in $LIBX ${BASE:-libmfhe.so}; do
    MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$lib timeout -k 10 120 python -u tools/pipeline_bench.py 20 > $O/pipe_${lib}_$r.json 2>&1 || { echo "pipe $lib rc=$?"; tail -5 $O/pipe_${lib}_$r.json; exit 2; }
    python3 -c "import json,sys; d=json.loads(open('$O/pipe_${lib}_$r.json').read().strip().splitlines()[-1]); print('$lib round $r', {k: round(v, 4) for k, v in d.items() if k.endswith('_ms')})"
  done
done
cd /tmp && export TMPDIR=/tmp
MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$LIBX timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$O/pipe_prof -o run --output-format csv -- \
    python3 $ROOT/tools/pipeline_bench.py 10 > $ROOT/$O/pipe_prof.log 2>&1 || { echo "prof rc=$?"; exit 3; }
echo done
