#!/bin/bash
# r05: enc_ring_kernel's row streams nontemporal (MFHE_ENC_NT variant library) vs default: parity, pipeline A/B
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r05ae; mkdir -p $O
LP=$ROOT/matrix-fhe-gpu_amd
MFHE_LIB=$LP/libmfhe_nt.so timeout -k 10 300 python -u -m pytest tests/test_he_gpu.py -x -q --timeout 120 --timeout-method thread \
    > $O/pytest_nt.log 2>&1 || { tail -30 $O/pytest_nt.log; exit 1; }
tail -1 $O/pytest_nt.log
for r in 1 2 3; do for v in base nt; do
  case $v in base) lib=$LP/libmfhe.so;; *) lib=$LP/libmfhe_$v.so;; esac
  MFHE_LIB=$lib timeout -k 10 150 python tools/pipeline_bench.py 20 > $O/pipe.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 2; }
  python3 -c "import json; d=json.load(open('$O/pipe.json')); print('$v', {k: round(v, 4) for k, v in d.items() if k in ('encode_ms','encrypt_pair_ms','decrypt_and_decode_ms','chain_eager_ms')})" | tee -a $O/ab.txt
done; done
