# r04: C2 single pass with the LDS drain counter in place of the per-polynomial first barrier -- NTT parity subset,
# then alternating C2 A/B against the two-barrier build (libmfhe_prev.so)
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04j; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py tests/test_fullshape_gpu.py -x -q --timeout 120 --timeout-method thread -k "14 or c2 or phantom" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do for lib in libmfhe_prev.so libmfhe.so; do
  echo "== $lib" >> $O/c2ab.txt
  MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$lib timeout -k 10 120 python3 tools/c2_plans.py 0 >> $O/c2ab.txt 2>&1 || { tail -20 $O/c2ab.txt; exit 2; }
done; done
grep -v amdgpu.ids $O/c2ab.txt
# U64 (60-bit primes) SQ counters, one pass (tools/gemm_pmc_summary.py: VALU / LDS / wait fractions per kernel)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS \
    SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d "$O/pmc_u64" -o run --output-format csv -- \
    python3 "$ROOT/tools/ntt_rate.py" 16 8 1024 60 0 3 > "$O/pmc_u64.log" 2>&1 || { echo "pmc u64 failed rc=$?"; tail -5 "$O/pmc_u64.log"; exit 3; }
python3 "$ROOT/tools/gemm_pmc_summary.py" "$O/pmc_u64" ArithU64 | tee "$O/u64_summary.txt"
