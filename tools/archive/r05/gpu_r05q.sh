#!/bin/bash
# r05: pipeline eager vs one captured HIP graph (tools/pipeline_bench.py chain_eager_ms / chain_graph_ms), 3 runs
set -o pipefail
O=gpurun_out/r05q; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 150 python tools/pipeline_bench.py 20 > $O/pipe.$r.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 2; }
  python3 -c "import json; d=json.load(open('$O/pipe.$r.json')); print({k: round(v, 4) for k, v in d.items() if k.endswith('_ms')}, d['max_err'])"
done
