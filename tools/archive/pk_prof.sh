#!/bin/bash
# rocprofv3 kernel trace + FETCH/WRITE passes of the forward NTT with the packed intermediate on/off. Dev tool.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-pkprof}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for p in 0 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/kt$p" -o run --output-format csv -- python3 "$ROOT/bench.py" --only ntt --steps 5 --warmup 1 --no-cpu-baseline --recombine-batch 0 --ntt-pack $p > "$OUT/kt$p.log" 2>&1 || exit 3
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/$C$p" -o run --output-format csv -- python3 "$ROOT/bench.py" --only ntt --steps 2 --warmup 1 --no-cpu-baseline --recombine-batch 0 --ntt-pack $p > "$OUT/$C$p.log" 2>&1 || exit 4
  done
done
echo ok
