#!/bin/bash
# r05: HE parity after the workspace reservation change + graph capture of the pipeline
set -o pipefail
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_he_gpu.py tests/test_c4_gpu.py -x -v -rf --timeout 120 --timeout-method thread \
    > $O/pytest.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest.log | tail -8; exit $rc
