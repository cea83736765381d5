# r04: U64 60-bit C3 -- does the block pass wait on its global twiddle loads?  Alternating the product with a probe
# build whose TwSrcU twiddles come from the index (MFHE_EXP_TWCONST, wrong results, no loads); then a kernel trace of
# the product's U64 forward + inverse for the per-pass split
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04m; mkdir -p $O
timeout -k 10 300 python3 tools/lib_ab.py 3 libmfhe.so,libmfhe_tw.so -- 16 8 1024 60 0 10 > $O/twab.txt 2>&1 || { tail -20 $O/twab.txt; exit 1; }
cat $O/twab.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $ROOT/tools/ntt_rate.py 16 8 1024 60 0 10 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 2; }
F=$(find $O/prof -name "run_kernel_stats.csv" | head -1); head -6 "$F" | cut -c1-200
