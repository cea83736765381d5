# r04: U64 60-bit C3 block-pass variants, alternating (tools/lib_ab.py): product (4-row block tiles, no prefetch),
# v1 8-row tiles, v2 16-row tiles (MFHE_NTT_NGB16), v3 the next tile's loads issued before the butterflies
# (MFHE_NTT_U64_BLOCK_PF), v4 the inverse block pass's first-stage twiddles loaded before its entry exchange (MFHE_NTT_U64_INV_TWPRE),
# v5 the U64 block passes held to 128 VGPRs, 4 waves per SIMD (MFHE_NTT_U64_BLOCK_W4; the inverse first pass spills 8)
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04n; mkdir -p $O
timeout -k 10 400 python3 tools/lib_ab.py 2 libmfhe.so,libmfhe_v1.so,libmfhe_v2.so,libmfhe_v3.so,libmfhe_v4.so,libmfhe_v5.so -- 16 8 1024 60 0 10 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
