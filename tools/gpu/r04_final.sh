#!/bin/bash
# Round-4 final measurement set (one gpurun call) on the final sources: the GPU test suite, the three
# bench workloads, the rocprof kernel statistics of the Base bench, the Base PMC traffic record (for
# bench.py's roofline.traffic) and the LvT-B parity-stage split.  Every GPU step has its own time limit;
# the set stops at the first failing step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r04z}
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n start"; timeout -k 10 "$t" "$@"; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step tests 1000 bash -c "python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1"
step bench_base 300 bash -c "python -u bench.py > gpurun_out/${T}_bench_base.log 2>&1"
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_rocprof -o run -- python3 bench.py --no-cpu-baseline
step pmc_base 600 bash tools/pmc_traffic.sh gpurun_out/${T}_pmc_base base
step bench_base2 300 bash -c "python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench_base2.log 2>&1"
step bench_large 300 bash -c "python -u bench.py --workload large --no-cpu-baseline > gpurun_out/${T}_bench_large.log 2>&1"
step bench_lvt 400 bash -c "python -u bench.py --workload lvt_large > gpurun_out/${T}_bench_lvt_large.log 2>&1"
step stages 300 bash -c "python -u tools/parity_stages.py --json gpurun_out/${T}_stages.json > gpurun_out/${T}_stages.log 2>&1"
cp profiles/traffic_r04_base.json gpurun_out/ 2>/dev/null
exit 0
