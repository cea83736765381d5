#!/bin/bash
# r05e: plan-5 (XL2) timing probes and schedule variants (MFHE_LIB builds), one resident C3 batch each
set -o pipefail
O=gpurun_out
export PYTHONUNBUFFERED=1
for v in "" p1 p2 m1 l2 o18; do
  lib=matrix-fhe-gpu_amd/libmfhe${v:+_$v}.so
  MFHE_LIB=$lib timeout -k 10 120 python -u tools/xl2_rate.py 2 20 >> $O/r05e_xl2_variants.txt 2>&1 || exit $?
done
