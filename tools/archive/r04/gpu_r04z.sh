# r04: evidence for the decrypt-fused inverse W-CRT digitize + the LDS-transpose ring in the encrypt / decrypt row
# kernels: the headline chain (GPU suite, the driver's bench command, kernel trace vs events, PMC passes), smoke(),
# the reference-geometry pipeline A/B against the HEAD~ build (libmfhe_prev.so), the product build's kernel split
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04z
bash tools/profile_headline.sh r04z tests || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 9; }
tail -1 $O/smoke.log
for r in 1 2 3; do for L in libmfhe_prev.so libmfhe.so; do
  echo "== $L" >> $O/ab.txt
  MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$L timeout -k 10 200 python3 tools/pipeline_bench.py 40 >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 2; }
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pprof -o run --output-format csv -- python3 $ROOT/tools/pipeline_bench.py 10 > $O/pprof.log 2>&1 || { tail -20 $O/pprof.log; exit 3; }
F=$(find $O/pprof -name "run_kernel_stats.csv" | head -1); cp $F $O/pipeline_kernel_stats.csv
