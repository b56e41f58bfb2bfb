# Round-2 measurement set: GPU tests, bench lines (base / large / lvt_large), rocprof kernel stats
# of the base bench, PMC traffic records (base, large) for bench.py's roofline.traffic.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_gputest.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python -u bench.py > gpurun_out/final_bench_base.log 2>&1 && echo bench-base-ok
timeout -k 10 300 python -u bench.py --workload large > gpurun_out/final_bench_large.log 2>&1 && echo bench-large-ok
timeout -k 10 400 python -u bench.py --workload lvt_large > gpurun_out/final_bench_lvt_large.log 2>&1 && echo bench-lvt-ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final_rocprof -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/final_bench_under_rocprof.log 2>&1 && echo rocprof-ok
timeout -k 10 600 bash tools/pmc_traffic.sh gpurun_out/final_pmc_base base && echo pmc-base-ok
timeout -k 10 600 bash tools/pmc_traffic.sh gpurun_out/final_pmc_large large && echo pmc-large-ok
cp profiles/traffic_r02_base.json profiles/traffic_r02_large.json gpurun_out/ 2>/dev/null
timeout -k 10 300 python -u bench.py > gpurun_out/final_bench_base2.log 2>&1 && echo bench-base2-ok
