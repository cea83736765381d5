#!/bin/bash
set -o pipefail
cd tools/microbench
O=../../gpurun_out
timeout -k 10 60 ./l2_nE one D 2 1 1 0 0 5 > $O/r05c_ne.txt 2>&1; echo "nE rc=$?" >> $O/r05c_ne.txt
exit 0
