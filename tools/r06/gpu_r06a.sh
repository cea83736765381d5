#!/bin/bash
# r06a: modulus-size sweep (U60 canon fix), plan-5 (XL2) SQ counters of the product and probe builds, and the
# existing XL2 stress test on an M = 1 build of the final kernel
set -o pipefail
O=gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 420 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_modsize_sweep_gpu.py \
    tests/test_ntt_gpu.py -k "sweep or size or u60 or gl_and" > $O/r06a_sweep.log 2>&1 || { echo "sweep rc=$?"; tail -30 $O/r06a_sweep.log; exit 1; }
tail -3 $O/r06a_sweep.log
timeout -s KILL 60 rocprofv3 -L > $O/r06a_counters.txt 2>&1 || echo "counter list rc=$?"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA"
P3=""
for c in SQ_WAIT_BARRIER SQ_BARRIER_CYCLES SQ_SLEEP_CYCLES SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_INSTS_FLAT; do
  grep -qw "$c" $O/r06a_counters.txt && P3="$P3 $c"
done
echo "pass3: $P3"
cd /tmp && export TMPDIR=/tmp
for v in "" p2; do
  export MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/libmfhe${v:+_$v}.so
  k=1
  for P in "$P1" "$P2" "SQ_WAVE_CYCLES $P3"; do
    timeout -s KILL 120 rocprofv3 --pmc $P -d $ROOT/$O/r06a_pmc_${v:-prod}_$k -o run --output-format csv -- \
        python3 $ROOT/tools/xl2_rate.py 1 3 > $ROOT/$O/r06a_pmc_${v:-prod}_$k.log 2>&1 || { echo "pmc $v $k rc=$?"; tail -5 $ROOT/$O/r06a_pmc_${v:-prod}_$k.log; exit 2; }
    k=$((k+1))
  done
done
unset MFHE_LIB
cd $ROOT
MFHE_LIB=matrix-fhe-gpu_amd/libmfhe_m1.so timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py -x -v --timeout 200 \
    --timeout-method thread -k "xl2" > $O/r06a_xl2_m1_tests.log 2>&1 || { echo "m1 rc=$?"; tail -20 $O/r06a_xl2_m1_tests.log; exit 3; }
tail -3 $O/r06a_xl2_m1_tests.log
MFHE_LIB=matrix-fhe-gpu_amd/libmfhe_m1.so timeout -k 10 120 python -u tools/xl2_rate.py 2 20 > $O/r06a_xl2_m1_rate.txt 2>&1 || { echo "m1 rate rc=$?"; exit 4; }
cat $O/r06a_xl2_m1_rate.txt
