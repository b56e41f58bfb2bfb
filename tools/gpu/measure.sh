#!/bin/bash
# One GPU measurement set on the gpurun box.  Usage (from the repo root, through gpurun):
#   bash tools/gpu/measure.sh TAG STEP [STEP ...]
# STEP: tests | tests_k=<pytest -k expr> | bench_base | bench_large | bench_lvt | rocprof |
#       pmc_base | pmc_large | bench_base2 | ab=<python tools/... args>
# Every GPU step runs under its own time limit; the set stops at the first failing step (no
# retries), and everything is written under gpurun_out/<TAG>_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1
shift
step() {  # name timeout cmd...
  local name=$1 t=$2
  shift 2
  echo "[$(date +%T)] $name start"
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
for S in "$@"; do
  case "$S" in
    tests) step tests 1000 bash -c "python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1" ;;
    tests_k=*) step tests_k 600 bash -c "python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k '${S#tests_k=}' > gpurun_out/${TAG}_gputest_k.log 2>&1" ;;
    bench_base) step bench_base 300 bash -c "python -u bench.py > gpurun_out/${TAG}_bench_base.log 2>&1" ;;
    bench_base2) step bench_base2 300 bash -c "python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench_base2.log 2>&1" ;;
    bench_large) step bench_large 300 bash -c "python -u bench.py --workload large > gpurun_out/${TAG}_bench_large.log 2>&1" ;;
    bench_lvt) step bench_lvt 400 bash -c "python -u bench.py --workload lvt_large > gpurun_out/${TAG}_bench_lvt_large.log 2>&1" ;;
    rocprof) step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_rocprof -o run -- python3 bench.py --no-cpu-baseline ;;
    pmc_base) step pmc_base 600 bash tools/pmc_traffic.sh gpurun_out/${TAG}_pmc_base base ;;
    pmc_large) step pmc_large 600 bash tools/pmc_traffic.sh gpurun_out/${TAG}_pmc_large large ;;
    ab=*) step ab 600 bash -c "python -u ${S#ab=} > gpurun_out/${TAG}_ab.log 2>&1" ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
done
cp profiles/traffic_r0*_base.json profiles/traffic_r0*_large.json gpurun_out/ 2>/dev/null
exit 0
