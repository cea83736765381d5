# r04: parity after the C2 late conversion -- the NTT / full-shape / HE GPU tests on HEAD's libmfhe.so
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ntt_gpu.py tests/test_fullshape_gpu.py tests/test_he_gpu.py tests/test_golden.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
