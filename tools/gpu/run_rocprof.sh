set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final_rocprof_csv -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/final_bench_under_rocprof.log 2>&1 && echo rocprof-ok
