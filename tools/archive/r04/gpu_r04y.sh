# r04: decrypt-fused digitize variants (one-substep-ahead ct prefetch at 3 / 2 workgroups per CU, shuffle / LDS ring
# product) against the unfused build and the first fused builds: parity on the product build, the pipeline A/B,
# then the kernel split of the product build and of pf2
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04y; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_he_gpu.py tests/test_c4_gpu.py tests/test_core_api_gpu.py tests/test_multigpu_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do for L in libmfhe_prev.so libmfhe_fs.so libmfhe_lds.so libmfhe.so libmfhe_pf2.so libmfhe_fl.so; do
  echo "== $L" >> $O/ab.txt
  MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$L timeout -k 10 200 python3 tools/pipeline_bench.py 40 >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 2; }
done; done
python3 - <<'PY'
import json
cur=None
for line in open("gpurun_out/r04y/ab.txt"):
    if line.startswith("=="): cur=line.split()[1]; continue
    if line.startswith("{"):
        d=json.loads(line); print(cur.ljust(18), "enc_pair %.4f dec_dec %.4f total %.4f" % (d["encrypt_pair_ms"], d["decrypt_and_decode_ms"], d["encode_encrypt_decrypt_decode_ms"]))
PY
cd /tmp && export TMPDIR=/tmp
for L in libmfhe.so libmfhe_pf2.so; do
MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$L -o run --output-format csv -- python3 $ROOT/tools/pipeline_bench.py 10 > $O/prof_$L.log 2>&1 || { tail -20 $O/prof_$L.log; exit 3; }
F=$(find $O/prof_$L -name "run_kernel_stats.csv" | head -1); cp $F $O/kernel_stats_$L.csv
done
