# r04: C2 single pass with two barriers per polynomial (forward stores from L1, inverse loads L1) -- NTT parity subset,
# then alternating C2 A/B: HEAD~ r03-style (libmfhe_base.so), three-barrier r04 (libmfhe_prev.so), two-barrier (libmfhe.so),
# two-barrier with plain (c0) and nt-only (c2) output stores
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04h2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py tests/test_fullshape_gpu.py -x -q --timeout 120 --timeout-method thread -k "14 or c2 or phantom" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do for lib in libmfhe_base.so libmfhe_prev.so libmfhe.so libmfhe_c0.so libmfhe_c2.so; do
  echo "== $lib" >> $O/c2ab.txt
  MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$lib timeout -k 10 120 python3 tools/c2_plans.py 0 >> $O/c2ab.txt 2>&1 || { tail -20 $O/c2ab.txt; exit 2; }
done; done
grep -v amdgpu.ids $O/c2ab.txt
