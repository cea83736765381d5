# r04: is the CRT compose (crt_compose_f64_kernel) bound by its memory access pattern or by its arithmetic?  The
# encode+CRT line with the product vs a probe build whose compose only loads the limbs and stores (MFHE_EXP_CRT_COPY,
# wrong results), then the probe's kernel split
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04p; mkdir -p $O
for r in 1 2; do for lib in libmfhe.so libmfhe_cc.so; do
  MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$lib timeout -k 10 200 python3 bench.py --only crt --no-cpu-baseline > $O/crt.json 2>> $O/crt.err || { tail -20 $O/crt.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/crt.json')); print('$lib', round(d['encode_crt_ops_per_s']), round(d['encode_crt_GBps'], 1))" | tee -a $O/ab.txt
done; done
cd /tmp && export TMPDIR=/tmp
MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/libmfhe_cc.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $ROOT/bench.py --only crt --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 2; }
F=$(find $O/prof -name "run_kernel_stats.csv" | head -1); head -3 "$F" | cut -c1-200
