#!/bin/bash
# Round-5 measurement set (one gpurun call) on the committed sources: the GPU test suite, smoke(), the
# three bench workloads, the rocprof kernel statistics of the Base bench, the PMC traffic records of the three
# workloads (for bench.py's roofline.traffic), the extended SQ / LDS counter passes of the Base bench and the LvT-B
# parity-stage split.  Every GPU step has its own time limit; the set stops at the first failing step
# (failing tests excepted: pytest rc 1 is recorded and the set goes on).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05f}
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n start"; timeout -k 10 "$t" "$@"; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
echo "[$(date +%T)] tests start"
timeout -k 10 1500 bash -c "python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1"
rc=$?; echo "[$(date +%T)] tests rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
step smoke 300 bash -c "python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/${T}_smoke.log 2>&1"
step bench_base 300 bash -c "python -u bench.py > gpurun_out/${T}_bench_base.log 2>&1"
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_rocprof -o run -- python3 bench.py --no-cpu-baseline
step pmc_base 600 bash tools/pmc_traffic.sh gpurun_out/${T}_pmc_base base profiles/traffic_r05_base.json
cp profiles/traffic_r05_base.json gpurun_out/ 2>/dev/null
step bench_base2 300 bash -c "python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench_base2.log 2>&1"
step pmc_large 600 bash tools/pmc_traffic.sh gpurun_out/${T}_pmc_large large profiles/traffic_r05_large.json
step pmc_lvt 600 bash tools/pmc_traffic.sh gpurun_out/${T}_pmc_lvt lvt_large profiles/traffic_r05_lvt_large.json
cp profiles/traffic_r05_large.json profiles/traffic_r05_lvt_large.json gpurun_out/ 2>/dev/null
step bench_large 300 bash -c "python -u bench.py --workload large --no-cpu-baseline > gpurun_out/${T}_bench_large.log 2>&1"
step bench_lvt 400 bash -c "python -u bench.py --workload lvt_large > gpurun_out/${T}_bench_lvt_large.log 2>&1"
step stages 400 bash -c "python -u tools/parity_stages.py --json gpurun_out/${T}_stages.json > gpurun_out/${T}_stages.log 2>&1"
step pmc_sq 900 bash tools/pmc_passes.sh gpurun_out/${T}_pmc_sq -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
step pmc_sq_sum 120 bash -c "python3 tools/pmc_summary.py gpurun_out/${T}_pmc_sq > gpurun_out/${T}_pmc_sq_summary.txt 2>&1"
exit 0
