#!/bin/bash
# r06e: SQ counters of the small-operand noise GEMM (mod_gemm_mfma_smallb_kernel) and its neighbours in the
# reference-geometry pipeline: two rocprofv3 --pmc passes of tools/pipeline_bench.py 3 (no trace domains).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; O=$ROOT/gpurun_out/${TAG:-r06e}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS \
    SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d "$O/pmc1" -o run --output-format csv -- \
    python3 "$ROOT/tools/pipeline_bench.py" 3 > "$O/pmc1.log" 2>&1 || { echo "pmc1 failed rc=$?"; tail -5 "$O/pmc1.log"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVES \
    SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY -d "$O/pmc2" -o run --output-format csv -- \
    python3 "$ROOT/tools/pipeline_bench.py" 3 > "$O/pmc2.log" 2>&1 || { echo "pmc2 failed rc=$?"; tail -5 "$O/pmc2.log"; exit 2; }
for k in ${KERNELS:-smallb ring56 ifold_dec enc_ring gaussian_i8}; do python3 "$ROOT/tools/gemm_pmc_summary.py" "$O/pmc1" $k; done | tee "$O/sq1.txt"
python3 "$ROOT/tools/pmc_kernel_summary.py" ${SUMK:-smallb} "$O/pmc1" "$O/pmc2" | tee "$O/sq2.txt"
echo done
