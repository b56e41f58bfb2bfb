set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r03ab_on_$i.log 2>&1 || exit 1
VP_NO_TATTN=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r03ab_off_$i.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03ab_rocprof -o run -- python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/r03ab_rocprof.log 2>&1 || exit 1
