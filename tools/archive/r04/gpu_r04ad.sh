# r04: decrypt-fused digitize with ring_mul_row64_lds fed by 32-byte layout-C loads (MFHE_DEC_RING_C): rc (184 VGPRs),
# rc3 (bounded to 3 WG/CU, 3 spilled) against the product build (prev); A/B only, plus the main.cu 1e-4 check inside
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04ad; mkdir -p $O
for r in 1 2; do for L in libmfhe_prev.so libmfhe_rc.so libmfhe_rc3.so; do
  echo "== $L" >> $O/ab.txt
  MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$L timeout -k 10 200 python3 tools/pipeline_bench.py 40 >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 2; }
done; done
python3 - <<'PY'
import json
cur=None
for line in open("gpurun_out/r04ad/ab.txt"):
    if line.startswith("=="): cur=line.split()[1]; continue
    if line.startswith("{"):
        d=json.loads(line); print(cur.ljust(18), "enc_pair %.4f dec_dec %.4f total %.4f ok %s" % (d["encrypt_pair_ms"], d["decrypt_and_decode_ms"], d["encode_encrypt_decrypt_decode_ms"], d["main_cu_check_1e-4"]))
PY
