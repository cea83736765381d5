#!/bin/bash
# r06 final evidence in one session: the whole GPU suite, smoke(), the driver's default bench command, then the
# headline kernel trace + PMC traffic (tools/profile_headline.sh), the pipeline kernel trace and the U64 line's
# kernel trace (U60 vs Harvey).  Each GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
O=gpurun_out/${R06TAG:-r06final}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread --durations 15 \
    > $O/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench rc=$?"; tail -20 $O/bench_default.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print(d['value'], d['roofline']['frac'], d.get('reference_geometry_pipeline',{}).get('ms'))"
bash tools/profile_headline.sh ${R06TAG:-r06final}_prof || { echo "profile_headline rc=$?"; exit 4; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$O/pipe_prof -o run --output-format csv -- \
    python3 $ROOT/tools/pipeline_bench.py 10 > $ROOT/$O/pipe_prof.log 2>&1 || { echo "pipe prof rc=$?"; tail -10 $ROOT/$O/pipe_prof.log; exit 5; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$O/u64_prof -o run --output-format csv -- \
    python3 $ROOT/bench.py --only u64 --steps 2 --warmup 1 --no-cpu-baseline > $ROOT/$O/u64_prof.log 2>&1 || { echo "u64 prof rc=$?"; tail -10 $ROOT/$O/u64_prof.log; exit 6; }
echo done
