# r04: the factored W-CRT's D = 5 and D = 6 limbs in one grid (mod_gemm_mfma_ring56_kernel) -- HE / C4 / core-API /
# full-shape GPU tests, pipeline A/B against the HEAD build (libmfhe_base.so), the N = 2^14 single-pass timing probes
# (MFHE_S14_EXP 1: no memory traffic, 2: exchanges only, 3: neither), and one SQ counter pass each over the pipeline
# (GEMM kernels) and over C2 (ntt14_kernel), summarised by tools/gemm_pmc_summary.py
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04f; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_he_gpu.py tests/test_c4_gpu.py tests/test_core_api_gpu.py tests/test_fullshape_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do for lib in libmfhe_base.so libmfhe.so; do
  echo "== $lib" >> $O/pipe.txt
  MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$lib timeout -k 10 120 python3 tools/pipeline_bench.py 20 >> $O/pipe.txt 2>&1 || { tail -20 $O/pipe.txt; exit 3; }
done; done
grep -v amdgpu.ids $O/pipe.txt | cut -c1-420
timeout -k 10 300 python3 tools/lib_ab.py 2 libmfhe.so,libmfhe_e1.so,libmfhe_e2.so,libmfhe_e3.so -- 14 4 256 50 0 40 > $O/probes.txt 2>&1 || { tail -20 $O/probes.txt; exit 4; }
cat $O/probes.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS \
    SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d "$O/pmc_pipe" -o run --output-format csv -- \
    python3 "$ROOT/tools/pipeline_bench.py" 3 > "$O/pmc_pipe.log" 2>&1 || { echo "pmc failed rc=$?"; tail -5 "$O/pmc_pipe.log"; exit 5; }
python3 "$ROOT/tools/gemm_pmc_summary.py" "$O/pmc_pipe" gemm | tee "$O/gemm_summary.txt"
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS \
    SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d "$O/pmc_c2" -o run --output-format csv -- \
    python3 "$ROOT/tools/ntt_rate.py" 14 4 256 50 0 10 > "$O/pmc_c2.log" 2>&1 || { echo "pmc c2 failed rc=$?"; tail -5 "$O/pmc_c2.log"; exit 6; }
python3 "$ROOT/tools/gemm_pmc_summary.py" "$O/pmc_c2" ntt14 | tee "$O/c2_summary.txt"
exit 0
