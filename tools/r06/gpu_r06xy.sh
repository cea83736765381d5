#!/bin/bash
# r06xy: the tree's build against libmfhe_head.so (the previous commit's build) on tools/pipeline_bench.py,
# alternating, then the whole final-evidence chain (gpu_r06_final.sh) on the tree's build.
set -o pipefail
O=gpurun_out/${XYTAG:-r06xy}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2 3; do
  for lib in libmfhe.so libmfhe_head.so; do
    MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$lib timeout -k 10 120 python -u tools/pipeline_bench.py 20 > $O/pipe_${lib}_$r.json 2>&1 || { echo "pipe $lib rc=$?"; tail -5 $O/pipe_${lib}_$r.json; exit 2; }
    python3 -c "import json,sys; d=json.loads(open('$O/pipe_${lib}_$r.json').read().strip().splitlines()[-1]); print('$lib round $r', {k: round(v, 4) for k, v in d.items() if k.endswith('_ms')})"
  done
done
R06TAG=${R06TAG:-r06final7} bash tools/r06/gpu_r06_final.sh
