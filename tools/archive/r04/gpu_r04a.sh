set -o pipefail
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dist_gpu.py tests/test_ntt_gpu.py::test_fused_option_removed tests/test_c4_gpu.py "tests/test_he_gpu.py::test_encode_quantize_near_int64_limit" "tests/test_he_gpu.py::test_wcrt_mfma_matches_valu_and_oracle" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
MFHE_BENCH_BACKEND=gloo MFHE_BENCH_SAME_DEVICE=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_n2.json 2> $O/bench_n2.err || { tail -30 $O/bench_n2.err; exit 1; }
timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo done
