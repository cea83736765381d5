# r04: the decrypt-fused digitize split over G workgroups per (row, limb) + dec_colsum_kernel: parity on the product
# build (G = 4), then the pipeline A/B against G = 1 (HEAD 4b79632, prev), G = 2, G = 8, then the kernel split
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04aa; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_he_gpu.py tests/test_c4_gpu.py tests/test_core_api_gpu.py tests/test_multigpu_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do for L in libmfhe_prev.so libmfhe_s2.so libmfhe.so libmfhe_s8.so; do
  echo "== $L" >> $O/ab.txt
  MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$L timeout -k 10 200 python3 tools/pipeline_bench.py 40 >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 2; }
done; done
python3 - <<'PY'
import json
cur=None
for line in open("gpurun_out/r04aa/ab.txt"):
    if line.startswith("=="): cur=line.split()[1]; continue
    if line.startswith("{"):
        d=json.loads(line); print(cur.ljust(18), "enc_pair %.4f dec_dec %.4f total %.4f" % (d["encrypt_pair_ms"], d["decrypt_and_decode_ms"], d["encode_encrypt_decrypt_decode_ms"]))
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pprof -o run --output-format csv -- python3 $ROOT/tools/pipeline_bench.py 10 > $O/pprof.log 2>&1 || { tail -20 $O/pprof.log; exit 3; }
F=$(find $O/pprof -name "run_kernel_stats.csv" | head -1); cp $F $O/pipeline_kernel_stats.csv
