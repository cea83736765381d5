#!/bin/bash
# r05: MFHE_OPT_DEC_MM (the decrypt's ring product on the matrix cores): parity, pipeline A/B, kernel stats
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r05aa; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_he_gpu.py -x -q -k dec_mm --timeout 120 --timeout-method thread \
    > $O/pytest_mm.log 2>&1 || { tail -40 $O/pytest_mm.log; exit 1; }
tail -2 $O/pytest_mm.log
timeout -k 10 500 python -u -m pytest tests/test_he_gpu.py tests/test_c4_gpu.py -x -q --timeout 120 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2 3; do for mm in 0 1; do
  MFHE_DEC_MM=$mm timeout -k 10 150 python tools/pipeline_bench.py 20 > $O/pipe.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 2; }
  python3 -c "import json; d=json.load(open('$O/pipe.json')); print('dec_mm=$mm', {k: round(v, 4) for k, v in d.items() if k in ('encode_ms','decrypt_and_decode_ms','chain_eager_ms')}, d['max_err'])" | tee -a $O/ab.txt
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- \
    python3 "$ROOT/tools/pipeline_bench.py" 10 > "$O/prof.log" 2>&1 || { echo "prof failed"; exit 4; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -14 {} | cut -c1-160'
