#!/bin/bash
# r05: pipeline A/B of library builds (MFHE_LIB), alternating: tools/r05/gpu_r05r.sh libA,libB [rounds]
set -o pipefail
O=gpurun_out/r05r; mkdir -p $O
IFS=, read -ra LIBS <<< "$1"
for r in $(seq 1 ${2:-3}); do for lib in "${LIBS[@]}"; do
  MFHE_LIB=$PWD/matrix-fhe-gpu_amd/$lib timeout -k 10 150 python tools/pipeline_bench.py 20 > $O/pipe.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 2; }
  python3 -c "import json; d=json.load(open('$O/pipe.json')); print('$lib', {k: round(v, 4) for k, v in d.items() if k.endswith('_ms')}, d['max_err'])" | tee -a $O/ab.txt
done; done
