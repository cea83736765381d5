# r04: SQ counters of the reference-geometry pipeline's row kernels (the decrypt-fused digitize, enc_ring / dec_ring
# with the LDS-transpose ring product), one pass with the r04f counter set, summarised by tools/gemm_pmc_summary.py
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04af; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS \
    SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d "$O/pmc_pipe" -o run --output-format csv -- \
    python3 "$ROOT/tools/pipeline_bench.py" 3 > "$O/pmc_pipe.log" 2>&1 || { echo "pmc failed rc=$?"; tail -5 "$O/pmc_pipe.log"; exit 5; }
for k in ifold_dec enc_ring dec_ring colsum; do python3 "$ROOT/tools/gemm_pmc_summary.py" "$O/pmc_pipe" $k; done | tee "$O/row_kernels_sq.txt"
