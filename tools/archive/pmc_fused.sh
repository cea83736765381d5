#!/bin/bash
# Counter passes (one rocprofv3 --pmc run per counter group) over fused vs two-pass NTT. Dev tool.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-pmcf}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
IFS=";" read -ra CFGS <<< "${PMC_CFGS:-16 8 1024 1 4 2;16 8 1024 1 8 3;16 8 1024 0 2 16}"
for cfg in "${CFGS[@]}"; do
  for C in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/p$i" -o run --output-format csv -- python3 "$ROOT/tools/ntt_once.py" $cfg 3 > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($cfg / $C) failed rc=$?"; tail -3 "$OUT/p$i.log"; exit 3; }
    echo "p$i: $cfg : $C" >> "$OUT/index.txt"
  done
done
echo ok
