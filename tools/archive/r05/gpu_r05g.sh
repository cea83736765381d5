#!/bin/bash
# r05: the lazy U60 forward schedule -- new parity tests, then C3 60-bit forward A/B (U60 vs Harvey, alternating)
set -u
OUT=gpurun_out/r05g; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ntt_gpu.py -x -v -rf --timeout 120 --timeout-method thread \
    -k "u60 or u64 or gl_and_cyclic or phantom_ntt" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for u in 1 0; do
    timeout -k 10 120 python tools/ntt_rate.py 16 8 1024 60 0 10 $u >> $OUT/rate.jsonl 2>> $OUT/rate.err || exit 4
  done
done
cat $OUT/rate.jsonl
