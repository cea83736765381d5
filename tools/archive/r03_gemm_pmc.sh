#!/bin/bash
# One gpurun session: one SQ counter pass over the reference-geometry pipeline (tools/pipeline_bench.py 3), summarised
# per GEMM kernel by tools/gemm_pmc_summary.py.  usage: tools/r03_gemm_pmc.sh <tag>
set -u
TAG=${1:-r03gp}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS \
    SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d "$OUT/pmc" -o run --output-format csv -- \
    python3 "$ROOT/tools/pipeline_bench.py" 3 > "$OUT/pmc.log" 2>&1 || { echo "pmc failed rc=$?"; tail -5 "$OUT/pmc.log"; exit 5; }
python3 "$ROOT/tools/gemm_pmc_summary.py" "$OUT/pmc" gemm | tee "$OUT/summary.txt"
python3 "$ROOT/tools/gemm_pmc_summary.py" "$OUT/pmc" digitize | tee -a "$OUT/summary.txt"
python3 "$ROOT/tools/gemm_pmc_summary.py" "$OUT/pmc" ring_kernel | tee -a "$OUT/summary.txt"
python3 "$ROOT/tools/gemm_pmc_summary.py" "$OUT/pmc" cwdft | tee -a "$OUT/summary.txt"
exit 0
