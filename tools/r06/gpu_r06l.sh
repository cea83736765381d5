#!/bin/bash
# r06l: the wide compose with every limb of a >= 11-word Q in registers (C5: 32 limbs): CRT / recombine / full-shape
# parity tests, then bench.py --only c5 alternating libmfhe.so and libmfhe_prev.so (MFHE_LIB) on one box.
set -o pipefail
O=gpurun_out/${TAG:-r06l}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_crt_gpu.py tests/test_dist_gpu.py \
    tests/test_fullshape_gpu.py tests/test_c4_gpu.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for lib in libmfhe.so libmfhe_prev.so; do
    MFHE_LIB=$ROOT/matrix-fhe-gpu_amd/$lib timeout -k 10 300 python -u bench.py --only c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_${lib}_$r.json 2> $O/c5_${lib}_$r.err || { echo "c5 $lib rc=$?"; tail -5 $O/c5_${lib}_$r.err; exit 2; }
    python3 -c "
import json; d=json.loads(open('$O/c5_${lib}_$r.json').read().strip().splitlines()[-1]); c=d.get('c5_residue_shard', d)
print('$lib round $r', {k: c['local'][k] for k in ('ms','recombine_ms')}, {k: c['alltoall'].get(k) for k in ('recombine_only_ms','compose_only_ms')})"
  done
done
echo done
