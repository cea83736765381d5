#!/bin/bash
# r05: any-order pair launches (MFHE_OPT_HE_STREAMS 2): HE parity, pipeline A/B 1 / 2 / 0, chain trace of mode 2
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r05w; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_he_gpu.py tests/test_c4_gpu.py -x -q --timeout 120 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2 3; do for st in 1 2 0; do
  MFHE_HE_STREAMS=$st timeout -k 10 150 python tools/pipeline_bench.py 20 > $O/pipe.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 2; }
  python3 -c "import json; d=json.load(open('$O/pipe.json')); print('streams=$st', {k: round(v, 4) for k, v in d.items() if k in ('encode_ms','decrypt_and_decode_ms','chain_eager_ms')}, d['max_err'])" | tee -a $O/ab.txt
done; done
cd /tmp && export TMPDIR=/tmp
MFHE_HE_STREAMS=2 timeout -k 10 200 rocprofv3 --kernel-trace -d "$O/trace_s2" -o run --output-format csv -- \
    python3 "$ROOT/tools/pipeline_bench.py" 10 > "$O/trace_s2.log" 2>&1 || { echo "trace failed"; exit 4; }
python3 "$ROOT/tools/r05/chain_gaps.py" "$O/trace_s2" | tail -28
