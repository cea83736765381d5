#!/bin/bash
# SQ counters of the C3 NTT kernels, U64 (60-bit primes) and FP64: one --pmc pass each, no trace domains.
# usage: tools/r03_u64_pmc.sh <tag>
set -u
TAG=${1:-r03p}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for B in 60 50; do
  NTTP_BITS=$B timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
      SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE -d "$OUT/pmc$B" -o run \
      --output-format csv -- python3 "$ROOT/tools/u64_prof.py" 2 > "$OUT/pmc$B.log" 2>&1 || { echo "pmc $B failed rc=$?"; tail -5 "$OUT/pmc$B.log"; exit 3; }
  echo "pmc $B done"
done
