# r04: C2 single-pass probes + kernel trace + SQ pass, then the whole GPU suite, then the driver's bench command
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04d; mkdir -p $O
timeout -k 10 400 python3 tools/lib_ab.py 2 libmfhe.so,libmfhe_e1.so,libmfhe_e2.so,libmfhe_e3.so -- 14 4 256 50 1 40 > $O/probes.txt 2>&1 || { tail -20 $O/probes.txt; exit 1; }
cat $O/probes.txt
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $ROOT/tools/ntt_rate.py 14 4 256 50 1 40 > $O/trace.log 2>&1 ) || { tail -20 $O/trace.log; exit 2; }
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $O/pmc -o run --output-format csv -- python3 $ROOT/tools/ntt_rate.py 14 4 256 50 1 10 > $O/pmc.log 2>&1 ) || { tail -20 $O/pmc.log; exit 3; }
find $O/trace -name "*stats.csv" | head -1 | xargs -I{} sh -c 'head -4 {} | cut -c1-160'
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread --durations 10 > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 4; }
tail -15 $O/pytest_gpu.log
timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 5; }
echo bench ok
