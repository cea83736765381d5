# r04 final: the headline evidence at HEAD (tools/profile_headline.sh: GPU suite, the driver's bench command, kernel
# trace vs HIP events, FETCH_SIZE / WRITE_SIZE passes), then smoke()
set -o pipefail
ROOT=$(pwd)
bash tools/profile_headline.sh r04s tests || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04s/smoke.log 2>&1 || { tail -20 gpurun_out/r04s/smoke.log; exit 9; }
tail -1 gpurun_out/r04s/smoke.log
