#!/bin/bash
# r05: MFHE_OPT_DEC_MM timing diagnostics (variant libraries, wrong results by construction): d1 no digit-plane
# stores, d2 no MFMAs
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r05ab; mkdir -p $O
LP=$ROOT/matrix-fhe-gpu_amd
for r in 1 2; do for v in base0 base1 d1 d2; do
  case $v in base0) lib=$LP/libmfhe.so; mm=0;; base1) lib=$LP/libmfhe.so; mm=1;; *) lib=$LP/libmfhe_$v.so; mm=1;; esac
  MFHE_LIB=$lib MFHE_DEC_MM=$mm timeout -k 10 150 python tools/pipeline_bench.py 20 > $O/pipe.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 2; }
  python3 -c "import json; d=json.load(open('$O/pipe.json')); print('$v', {k: round(v, 4) for k, v in d.items() if k in ('decrypt_and_decode_ms','chain_eager_ms')})" | tee -a $O/ab.txt
done; done
