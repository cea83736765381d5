# r04: C2 exchange rewrite + U64 mulhi64 + D = 6 ring GEMM at 2 workgroups/CU -- whole GPU suite on the new
# libmfhe.so, then alternating A/Bs against the HEAD build (libmfhe_base.so): C2 (tools/c2_plans.py plan 0),
# U64 60-bit C3 (tools/lib_ab.py + ntt_rate.py), reference-geometry pipeline (tools/pipeline_bench.py)
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for r in 1 2; do for lib in libmfhe_base.so libmfhe.so; do
  echo "== $lib" >> $O/c2ab.txt
  MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$lib timeout -k 10 120 python3 tools/c2_plans.py 0 >> $O/c2ab.txt 2>&1 || { tail -20 $O/c2ab.txt; exit 2; }
  echo "== $lib" >> $O/pipe.txt
  MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$lib timeout -k 10 120 python3 tools/pipeline_bench.py 20 >> $O/pipe.txt 2>&1 || { tail -20 $O/pipe.txt; exit 3; }
done; done
grep -v amdgpu.ids $O/c2ab.txt
grep -v amdgpu.ids $O/pipe.txt | cut -c1-400
timeout -k 10 300 python3 tools/lib_ab.py 2 libmfhe_base.so,libmfhe.so -- 16 8 1024 60 0 10 > $O/u64ab.txt 2>&1 || { tail -20 $O/u64ab.txt; exit 4; }
cat $O/u64ab.txt
