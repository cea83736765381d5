# r04: C2 single pass, the loop carrying converted doubles (conversion after the stores, MFHE_S14_LATE_CVT=1,
# libmfhe_lc.so) vs the product, alternating tools/c2_plans.py 0 (8 rotating 128 MiB buffers)
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04q; mkdir -p $O
for r in 1 2; do for lib in libmfhe.so libmfhe_lc.so; do
  echo "== $lib" >> $O/c2ab.txt
  MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$lib timeout -k 10 120 python3 tools/c2_plans.py 0 >> $O/c2ab.txt 2>&1 || { tail -20 $O/c2ab.txt; exit 2; }
done; done
grep -v amdgpu.ids $O/c2ab.txt
