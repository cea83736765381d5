# r04 final: the headline chain at the final HEAD (GPU suite, the driver's bench command, kernel trace vs events, PMC
# passes), smoke(), and the reference-geometry pipeline's kernel split
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04ac
bash tools/profile_headline.sh r04ac tests || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 9; }
tail -1 $O/smoke.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pprof -o run --output-format csv -- python3 $ROOT/tools/pipeline_bench.py 10 > $O/pprof.log 2>&1 || { tail -20 $O/pprof.log; exit 3; }
F=$(find $O/pprof -name "run_kernel_stats.csv" | head -1); cp $F $O/pipeline_kernel_stats.csv
grep -v amdgpu.ids $O/pprof.log | tail -1 | cut -c1-300
