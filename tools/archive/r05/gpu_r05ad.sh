#!/bin/bash
# r05: SQ counters of dec_mm_digitize_kernel (MFHE_OPT_DEC_MM 1) against mfma_digitize_ifold_dec_kernel (0)
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r05ad; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for mm in 1 0; do
  MFHE_DEC_MM=$mm timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS \
      SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d "$O/pmc1_$mm" -o run --output-format csv -- \
      python3 "$ROOT/tools/pipeline_bench.py" 3 > "$O/pmc1_$mm.log" 2>&1 || { echo "pmc failed rc=$?"; tail -5 "$O/pmc1_$mm.log"; exit 5; }
  MFHE_DEC_MM=$mm timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVES \
      SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY -d "$O/pmc2_$mm" -o run --output-format csv -- \
      python3 "$ROOT/tools/pipeline_bench.py" 3 > "$O/pmc2_$mm.log" 2>&1 || { echo "pmc2 failed rc=$?"; tail -5 "$O/pmc2_$mm.log"; exit 6; }
  for k in dec_mm ifold_dec; do python3 "$ROOT/tools/gemm_pmc_summary.py" "$O/pmc1_$mm" $k; done
  python3 - "$O/pmc2_$mm" <<'PY'
import collections, csv, glob, sys
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "dec_mm" in k or "ifold_dec" in k:
            tot[k[:50]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, m in tot.items():
    w = m.get("SQ_WAVES", 1) or 1
    print(k, {c: round(v / w, 1) for c, v in sorted(m.items())}, "per wave; waves", w)
PY
done
