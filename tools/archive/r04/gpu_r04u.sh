# r04 final: rehearse the N > 1 bench path on the one-GPU box with the final bench.py -- plain `python3 bench.py --gpus 2`
# (self-launched ranks, gloo, both ranks on the same device), then the default single-GPU command
set -o pipefail
O=gpurun_out/r04u; mkdir -p $O
MFHE_BENCH_BACKEND=gloo MFHE_BENCH_SAME_DEVICE=1 timeout -k 10 500 python3 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_n2.json 2> $O/bench_n2.err || { tail -30 $O/bench_n2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_n2.json')); print(d['n_gpus'], d['value'], {k: (v if not isinstance(v, dict) else str(v)[:160]) for k, v in d.items() if k in ('c4_sharded_pipeline', 'c5_residue_shard')})"
