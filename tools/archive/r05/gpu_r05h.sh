#!/bin/bash
# r05: per-kernel split of the C3 60-bit forward, lazy U60 vs Harvey (rocprofv3 kernel trace of tools/ntt_rate.py)
set -u
OUT=$PWD/gpurun_out/r05h; mkdir -p $OUT
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
for u in 1 0; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_u$u -o run --output-format csv -- \
      python3 $ROOT/tools/ntt_rate.py 16 8 1024 60 0 10 $u > $OUT/rate_u$u.log 2>&1 || { tail -5 $OUT/rate_u$u.log; exit 3; }
  cat $OUT/rate_u$u.log | tail -1
  F=$(find $OUT/prof_u$u -name "run_kernel_stats.csv" | head -1)
  cut -c1-200 $F | head -8
done
