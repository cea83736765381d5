#!/bin/bash
# r05f: the reworked plan-5 kernel: parity tests + stress, then timing of variants (MFHE_LIB builds)
set -o pipefail
O=gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py -x -v --timeout 120 --timeout-method thread -k "xl2" > $O/r05f_xl2_tests.txt 2>&1 || exit $?
for v in "" p2 m1 l1 o18; do
  lib=matrix-fhe-gpu_amd/libmfhe${v:+_$v}.so
  MFHE_LIB=$lib timeout -k 10 120 python -u tools/xl2_rate.py 2 20 >> $O/r05f_xl2_variants.txt 2>&1 || exit $?
done
