# r04: decrypt-fused digitize occupancy variants (G = 4): prod (149 VGPRs, 3 WG/CU), w4 (4 WG/CU, 2-substep loads,
# 20 spills), sb2 (2-substep loads), tl (twiddles in LDS), tl4 (tl at 4 WG/CU, 29 spills); no parity step (A/B only)
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04ab; mkdir -p $O
for r in 1 2; do for L in libmfhe.so libmfhe_w4.so libmfhe_sb2.so libmfhe_tl.so libmfhe_tl4.so; do
  echo "== $L" >> $O/ab.txt
  MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$L timeout -k 10 200 python3 tools/pipeline_bench.py 40 >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 2; }
done; done
python3 - <<'PY'
import json
cur=None
for line in open("gpurun_out/r04ab/ab.txt"):
    if line.startswith("=="): cur=line.split()[1]; continue
    if line.startswith("{"):
        d=json.loads(line); print(cur.ljust(18), "enc_pair %.4f dec_dec %.4f total %.4f" % (d["encrypt_pair_ms"], d["decrypt_and_decode_ms"], d["encode_encrypt_decrypt_decode_ms"]))
PY
cd /tmp && export TMPDIR=/tmp
