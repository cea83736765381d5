# r04: N = 2^14 pipelined single pass -- parity, then C2 timing (bench other_ntt_configs) per plan
set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "tests/test_ntt_gpu.py::test_single_pass_14_matches_oracle_and_other_plans" "tests/test_ntt_gpu.py::test_phantom_ntt_matches_oracle" "tests/test_fullshape_gpu.py::test_c2_full_shape" "tests/test_fullshape_gpu.py::test_c4_shard_full_shape" "tests/test_he_gpu.py::test_encrypt_decrypt_vs_oracle_c4_moduli" "tests/test_he_gpu.py::test_encrypt_decrypt_vs_oracle" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python3 tools/c2_plans.py > $O/c2_plans.txt 2>&1 || { tail -30 $O/c2_plans.txt; exit 1; }
cat $O/c2_plans.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_ntt_gpu.py::test_phantom_ntt_matches_oracle" "tests/test_ntt_gpu.py::test_extreme_moduli_and_values_u64" "tests/test_fullshape_gpu.py::test_c3_60bit_primes_full_shape" "tests/test_fullshape_gpu.py::test_c3_full_shape" > $O/pytest_u64.log 2>&1 || { tail -40 $O/pytest_u64.log; exit 1; }
tail -2 $O/pytest_u64.log
timeout -k 10 600 python3 tools/lib_ab.py 3 libmfhe.so,libmfhe_w3.so,libmfhe_sb0.so -- 16 8 1024 60 > $O/u64_ab.txt 2>&1 || { tail -20 $O/u64_ab.txt; exit 1; }
cat $O/u64_ab.txt
