# r04: kernel split of the reference-geometry pipeline at HEAD (rocprofv3 kernel trace of tools/pipeline_bench.py 10)
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04t; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $ROOT/tools/pipeline_bench.py 10 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep -v amdgpu.ids $O/prof.log | tail -1 | cut -c1-400
F=$(find $O/prof -name "run_kernel_stats.csv" | head -1); cp $F $O/kernel_stats.csv
