#!/bin/bash
# r05: lazy U60 forward -- parity subset, then SQ counters of the C3 60-bit forward (U60 default and Harvey) in one
# --pmc pass each (tools/gemm_pmc_summary.py: VALU busy / wait fractions per kernel)
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r05j; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ntt_gpu.py tests/test_fullshape_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "u60 or u64 or gl_and_cyclic or phantom or c3u60 or fullshape" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cd /tmp && export TMPDIR=/tmp
for u in 1 0; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS \
      SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d "$O/pmc_u$u" -o run --output-format csv -- \
      python3 "$ROOT/tools/ntt_rate.py" 16 8 1024 60 0 3 $u > "$O/pmc_u$u.log" 2>&1 || { echo "pmc failed rc=$?"; tail -5 "$O/pmc_u$u.log"; exit 3; }
  python3 "$ROOT/tools/gemm_pmc_summary.py" "$O/pmc_u$u" ArithU6 | tee "$O/sq_u$u.txt"
done
