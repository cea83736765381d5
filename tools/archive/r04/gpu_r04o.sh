# r04: the whole GPU suite on HEAD's libmfhe.so (drain-counter C2, U64 inverse twiddle prefetch), smoke(), the default bench command
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04o; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread --durations 10 > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -14 $O/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['reference_geometry_pipeline']['ms'], json.dumps(d['other_ntt_configs'])[:400], json.dumps(d['u64_path_c3_forward_ntt'])[:300])"
