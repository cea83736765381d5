#!/bin/bash
# r05f: the reworked plan-5 kernel: parity tests + stress (256- and 512-thread builds), then timing of variants
set -o pipefail
O=gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py -x -v --timeout 120 --timeout-method thread -k "xl2" > $O/r05f_xl2_tests.txt 2>&1 || exit $?
MFHE_LIB=matrix-fhe-gpu_amd/libmfhe_r3.so timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py -x -v --timeout 120 --timeout-method thread -k "xl2" > $O/r05f_xl2_tests_r3.txt 2>&1 || exit $?
for v in "" r3 p2 p2r3 o18 m4; do
  lib=matrix-fhe-gpu_amd/libmfhe${v:+_$v}.so
  MFHE_LIB=$lib timeout -k 10 120 python -u tools/xl2_rate.py 2 20 >> $O/r05f_xl2_variants.txt 2>&1 || exit $?
done
