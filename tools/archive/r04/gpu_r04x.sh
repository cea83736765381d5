# r04: decrypt-fused digitize with the LDS-transpose ring product (ring_mul_row64_lds): parity, then the pipeline
# A/B unfused (prev) vs fused with the shuffle ring (fs) vs fused LDS ring, then the kernel split
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04x; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_he_gpu.py tests/test_c4_gpu.py tests/test_core_api_gpu.py tests/test_multigpu_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do for L in libmfhe_prev.so libmfhe_fs.so libmfhe.so; do
  echo "== $L" >> $O/ab.txt
  MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$L timeout -k 10 200 python3 tools/pipeline_bench.py 40 >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 2; }
done; done
grep -v amdgpu.ids $O/ab.txt | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $ROOT/tools/pipeline_bench.py 10 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 3; }
F=$(find $O/prof -name "run_kernel_stats.csv" | head -1); cp $F $O/kernel_stats.csv
