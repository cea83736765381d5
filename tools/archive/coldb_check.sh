set -o pipefail
mkdir -p gpurun_out/coldb
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_ntt_gpu.py -k "column_pass_dma" tests/test_fullshape_gpu.py > gpurun_out/coldb/pytest.log 2>&1 || { tail -30 gpurun_out/coldb/pytest.log; exit 3; }
tail -3 gpurun_out/coldb/pytest.log
for rep in 1 2; do for pf in 0 2; do
timeout -k 10 120 python bench.py --only ntt --steps 20 --warmup 5 --no-cpu-baseline --recombine-batch 0 --ntt-prefetch $pf > gpurun_out/coldb/b$pf.$rep.json 2>/dev/null || exit 4
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('pf',sys.argv[2], round(d['value']), 'inv', round(d['inverse_NTT_per_s']), 'frac', d['roofline']['frac'])" gpurun_out/coldb/b$pf.$rep.json $pf
done; done
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/coldb/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --only ntt --steps 10 --warmup 2 --no-cpu-baseline --recombine-batch 0 --ntt-prefetch 2 > $GRAFT_REPO_ROOT/gpurun_out/coldb/prof.log 2>&1 || exit 5
grep -h "ntt_" $(find $GRAFT_REPO_ROOT/gpurun_out/coldb/prof -name "*kernel_stats.csv") | cut -c1-220
