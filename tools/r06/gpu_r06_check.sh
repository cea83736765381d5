#!/bin/bash
# r06: the whole GPU suite and smoke() on the tree's build (a final consistency check of the committed libmfhe.so)
set -o pipefail
O=gpurun_out/${TAG:-r06check}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { echo "pytest rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
