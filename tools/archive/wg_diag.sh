#!/bin/bash
# Per-pass NTT kernel time vs resident workgroups per CU (MFHE_OPT_NTT_WG_PER_CU cap), C3 forward + inverse.
# One rocprofv3 kernel trace per setting; prints the average duration of each ntt_pass_kernel instantiation.
# usage: tools/wg_diag.sh <tag> [wg...]   Dev tool.
set -u
TAG=$1; shift
WGS=${*:-1 2 3 4}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for wg in $WGS; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/wg$wg" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --only ntt --steps 10 --warmup 2 --no-cpu-baseline --recombine-batch 0 \
      --ntt-wg "$wg" > "$OUT/wg$wg.log" 2>&1 || { echo "wg $wg failed rc=$?"; tail -5 "$OUT/wg$wg.log"; exit 3; }
  python3 - "$OUT/wg$wg" "$wg" <<'EOF'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "ntt_pass_kernel" in r["Name"]:
        n = r["Name"]
        targs = n[n.index("<"):n.index(">(")] if "<" in n else n
        print("wg", sys.argv[2], "avg_us", round(float(r["AverageNs"]) / 1e3, 1), "calls", r["Calls"], targs[:160])
EOF
done
