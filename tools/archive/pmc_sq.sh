#!/bin/bash
# SQ / TCC counter passes over the NTT bench (one --pmc group per run, no trace domains).
# usage: tools/pmc_sq.sh <tag> [extra bench args]
set -u
TAG=${1:-sq}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for G in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $G -d "$OUT/p$i" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --only ntt --steps 1 --warmup 0 --no-cpu-baseline --recombine-batch 0 "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 3; }
  echo "pass $i done"
done
exit 0
