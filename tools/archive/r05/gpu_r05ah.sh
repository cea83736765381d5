#!/bin/bash
# r05 (final build): reference-geometry pipeline kernel split (rocprofv3 kernel trace of tools/pipeline_bench.py 10) and one SQ
# counter pass (MFMA busy / VALU / waits per kernel, tools/gemm_pmc_summary.py)
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r05ah; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- \
    python3 "$ROOT/tools/pipeline_bench.py" 10 > "$O/trace.log" 2>&1 || { echo "trace failed rc=$?"; tail -5 "$O/trace.log"; exit 4; }
grep encode_encrypt "$O/trace.log" | cut -c1-400
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS \
    SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d "$O/pmc_pipe" -o run --output-format csv -- \
    python3 "$ROOT/tools/pipeline_bench.py" 3 > "$O/pmc_pipe.log" 2>&1 || { echo "pmc failed rc=$?"; tail -5 "$O/pmc_pipe.log"; exit 5; }
for k in ring56 ifold_dec enc_ring digitize_fold crt_compose cgemm colsum gaussian; do python3 "$ROOT/tools/gemm_pmc_summary.py" "$O/pmc_pipe" $k; done | tee "$O/pipe_sq.txt"
