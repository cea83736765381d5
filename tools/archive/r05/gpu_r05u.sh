#!/bin/bash
# r05: kernel traces of the pipeline (tools/pipeline_bench.py 10, whose last eager section is the back-to-back chain)
# with MFHE_OPT_HE_STREAMS 1 and 0, for the inter-kernel gap analysis (tools/r05/chain_gaps.py)
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r05u; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for st in 1 0; do
  MFHE_HE_STREAMS=$st timeout -k 10 200 rocprofv3 --kernel-trace -d "$O/trace_s$st" -o run --output-format csv -- \
      python3 "$ROOT/tools/pipeline_bench.py" 10 > "$O/trace_s$st.log" 2>&1 || { echo "trace failed rc=$?"; tail -5 "$O/trace_s$st.log"; exit 4; }
  grep -o '"chain_eager_ms": [0-9.]*' "$O/trace_s$st.log"
done
