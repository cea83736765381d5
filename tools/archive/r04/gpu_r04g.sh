# r04: C2 store / load probes (MFHE_S14_EXP 4: no stores, 5: no loads after the first) beside the product and e1 / e3,
# and the VALU issue-rate microbenchmark (tools/microbench/valu_rate.hip)
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r04g; mkdir -p $O
timeout -k 10 60 tools/microbench/valu_rate > $O/valu_rate.txt 2>&1 || { cat $O/valu_rate.txt; exit 1; }
cat $O/valu_rate.txt
timeout -k 10 300 python3 tools/lib_ab.py 2 libmfhe.so,libmfhe_e1.so,libmfhe_e3.so,libmfhe_e4.so,libmfhe_e5.so -- 14 4 256 50 0 40 > $O/probes.txt 2>&1 || { tail -20 $O/probes.txt; exit 2; }
cat $O/probes.txt
