#!/bin/bash
# r05: MFHE_OPT_DEC_MM kernel variants (launch bound 2 / 1 workgroups per CU): parity, per-kernel time
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r05ac; mkdir -p $O
LP=$ROOT/matrix-fhe-gpu_amd
timeout -k 10 200 python -u -m pytest tests/test_he_gpu.py -x -q -k "dec_mm or fused_ring" --timeout 120 --timeout-method thread \
    > $O/pytest_mm.log 2>&1 || { tail -40 $O/pytest_mm.log; exit 1; }
tail -1 $O/pytest_mm.log
for v in k8 k8a1; do
  MFHE_LIB=$LP/libmfhe_$v.so timeout -k 10 200 python -u -m pytest tests/test_he_gpu.py -x -q -k "dec_mm" --timeout 120 \
      --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -40 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
cd /tmp && export TMPDIR=/tmp
for v in base k8 k8a1; do
  case $v in base) lib=$LP/libmfhe.so;; *) lib=$LP/libmfhe_$v.so;; esac
  MFHE_DEC_MM=1 MFHE_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof_$v" -o run --output-format csv -- \
      python3 "$ROOT/tools/pipeline_bench.py" 10 > "$O/prof_$v.log" 2>&1 || { echo "prof failed"; tail -5 $O/prof_$v.log; exit 4; }
  f=$(find $O/prof_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; grep -E "dec_mm|dec_colsum|ring56_kernel<2>|ifold_dec" $f | cut -d, -f1-4,6 | cut -c1-150
  python3 -c "import json,sys; d=json.load(open('$O/prof_$v.log'.replace('.log','.log'))) " 2>/dev/null || tail -1 $O/prof_$v.log | cut -c1-300
done
