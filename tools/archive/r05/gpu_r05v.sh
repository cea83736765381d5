#!/bin/bash
# r05: MFHE_OPT_HE_STREAMS modes 1 / 2 / 3 / 0, pipeline chain (tools/pipeline_bench.py 20), alternating, 3 rounds
set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
for r in 1 2 3; do for st in 1 2 3 0; do
  MFHE_HE_STREAMS=$st timeout -k 10 150 python tools/pipeline_bench.py 20 > $O/pipe.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 2; }
  python3 -c "import json; d=json.load(open('$O/pipe.json')); print('streams=$st', {k: round(v, 4) for k, v in d.items() if k in ('encode_ms','decrypt_and_decode_ms','chain_eager_ms')}, d['max_err'])" | tee -a $O/ab.txt
done; done
