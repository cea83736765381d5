#!/bin/bash
# Rehearsal of bench.py's N > 1 code path on a one-GPU box: 2 ranks on cuda:0 over gloo (RCCL refuses two ranks
# on one GPU, so the native-RCCL lines report themselves skipped), then the driver's default N = 1 command.
set -u
TAG=${1:-r03r}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
MFHE_BENCH_BACKEND=gloo MFHE_BENCH_SAME_DEVICE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 \
    > "$OUT/bench_n2.json" 2> "$OUT/bench_n2.err" || { echo "n2 rehearsal failed rc=$?"; tail -20 "$OUT/bench_n2.err"; exit 3; }
tail -c 3000 "$OUT/bench_n2.json"; echo
SECONDS=0; timeout -k 10 500 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" \
    || { echo "default bench failed"; tail -20 "$OUT/bench_default.err"; exit 4; }
echo "default bench wall: ${SECONDS} s"
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['steps'], d['warmup'], d['inverse_over_forward'], d.get('c4_sharded_pipeline',{}).get('exchange'))" "$OUT/bench_default.json"
