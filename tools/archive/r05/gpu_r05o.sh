#!/bin/bash
# r05: C2 single pass vs batch (polynomials per CU): tools/ntt_rate.py 14 4 <batch> 50 on one resident batch
set -o pipefail
O=gpurun_out/r05o; mkdir -p $O
for b in 256 512 1024 4096 256; do
  timeout -k 10 120 python tools/ntt_rate.py 14 4 $b 50 0 20 >> $O/c2_batch.jsonl 2>> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
done
cat $O/c2_batch.jsonl
