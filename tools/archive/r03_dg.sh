set -u
cd /tmp && export TMPDIR=/tmp
for v in base dg; do
  if [ $v = base ]; then lib=$GRAFT_REPO_ROOT/matrix-fhe-gpu_amd/libmfhe.so; else lib=$GRAFT_REPO_ROOT/matrix-fhe-gpu_amd/libmfhe_$v.so; fi
  MFHE_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03dg/$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/pipeline_bench.py 5 > $GRAFT_REPO_ROOT/gpurun_out/r03dg/$v.log 2>&1 || { echo "$v failed"; exit 3; }
  grep -h "ring_kernel<5, 2" $(find $GRAFT_REPO_ROOT/gpurun_out/r03dg/$v -name "*kernel_stats.csv") | cut -d, -f1-4
done
