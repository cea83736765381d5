# r04: two-coefficient CRT compose (crt_compose_f64_x2_kernel) -- CRT / full-shape / HE GPU tests, then the
# encode+CRT line alternating MFHE_CRT_X2=0 (one-coefficient kernel) / 1 (default), and a kernel trace
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04l; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_crt_gpu.py tests/test_fullshape_gpu.py tests/test_he_gpu.py tests/test_c4_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2 3; do for x in 0 1; do
  MFHE_CRT_X2=$x timeout -k 10 200 python3 bench.py --only crt --no-cpu-baseline > $O/crt_$x.json 2>> $O/crt.err || { tail -20 $O/crt.err; exit 2; }
  python3 -c "import json; d=json.load(open('$O/crt_$x.json')); print('x2=$x', round(d['encode_crt_ops_per_s']), round(d['encode_crt_GBps'], 1))" | tee -a $O/crt_ab.txt
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $ROOT/bench.py --only crt --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 3; }
F=$(find $O/prof -name "run_kernel_stats.csv" | head -1); head -4 "$F" | cut -c1-200
