# r04: encode+CRT line (rns_decompose + crt_compose_f64 at C3, 256 polys per call): bench --only crt, then a
# rocprofv3 kernel trace of the same command for the per-kernel split
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04k; mkdir -p $O
timeout -k 10 300 python3 bench.py --only crt --no-cpu-baseline > $O/crt.json 2> $O/crt.err || { tail -20 $O/crt.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/crt.json')); print({k: d.get(k) for k in ('encode_crt_ops_per_s', 'encode_crt_GBps')})"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $ROOT/bench.py --only crt --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 2; }
F=$(find $O/prof -name "run_kernel_stats.csv" | head -1); head -6 "$F" | cut -c1-220
