#!/bin/bash
# r05: two-stream HE chains (MFHE_OPT_HE_STREAMS) -- HE / C4 / core-API parity, then pipeline A/B (1 vs 0, alternating)
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r05m; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_he_gpu.py tests/test_c4_gpu.py tests/test_core_api_gpu.py -x -q -k "fused_ring or streams or encrypt or kat or pipeline or c4" \
    --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2 3; do for st in 1 0; do
  MFHE_ENC_A_DIRECT=$st MFHE_HE_STREAMS=$st timeout -k 10 120 python tools/pipeline_bench.py 10 > $O/pipe_$st.$r.json 2> $O/pipe.err || { tail -20 $O/pipe.err; exit 2; }
  python3 -c "import json; d=json.load(open('$O/pipe_$st.$r.json')); print('streams=$st', {k: round(v, 4) for k, v in d.items() if k.endswith('_ms')}, d['max_err'])"
done; done
