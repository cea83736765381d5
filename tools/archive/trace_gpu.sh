set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out/trace4
timeout -k 10 300 python -u -m pytest tests/test_trace.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/trace4/pytest.log 2>&1; rc=$?
tail -30 gpurun_out/trace4/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "
import sys, json; sys.path.insert(0,'matrix-fhe-gpu_amd'); sys.path.insert(0,'.')
import bench
print(json.dumps(bench.trace_line()))
" 2>&1 | tee gpurun_out/trace4/trace_line.json
