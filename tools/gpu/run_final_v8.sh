# Round-2 final measurement set (v8: final round-2 build; v7 code with updated kernel comments): GPU tests, bench lines (base / large / lvt_large), rocprof
# kernel stats of the base bench, PMC traffic records (base, large) for bench.py's roofline.traffic,
# then the base bench again with the fresh traffic record.  Stops at the first failing GPU step.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 900 bash -c 'python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v8_gputest.log 2>&1'
step bench_base 300 bash -c 'python -u bench.py > gpurun_out/v8_bench_base.log 2>&1'
step bench_large 300 bash -c 'python -u bench.py --workload large > gpurun_out/v8_bench_large.log 2>&1'
step bench_lvt 400 bash -c 'python -u bench.py --workload lvt_large > gpurun_out/v8_bench_lvt_large.log 2>&1'
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v8_rocprof -o run -- python3 bench.py --no-cpu-baseline
step pmc_base 600 bash tools/pmc_traffic.sh gpurun_out/v8_pmc_base base
step pmc_large 600 bash tools/pmc_traffic.sh gpurun_out/v8_pmc_large large
cp profiles/traffic_r02_base.json profiles/traffic_r02_large.json gpurun_out/
step bench_base2 300 bash -c 'python -u bench.py > gpurun_out/v8_bench_base2.log 2>&1'
step bench_large2 300 bash -c 'python -u bench.py --workload large > gpurun_out/v8_bench_large2.log 2>&1'
