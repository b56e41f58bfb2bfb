#!/bin/bash
# Small-M text-tower GEMM: its kernel tests and the LvT / CLIP parity tests, then the LvT-Large bench and
# its rocprof kernel statistics.  Every GPU step has its own time limit; the set stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05s}
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n start"; timeout -k 10 "$t" "$@"; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step tests 900 bash -c "python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_clip.py tests/test_gpu_lvt_large.py tests/test_gpu_long_clips.py -m gpu -v -s --timeout 600 --timeout-method thread -k 'small_m or clip or lvt or text' > gpurun_out/${T}_gputest.log 2>&1"
step bench_lvt 400 bash -c "python -u bench.py --workload lvt_large --no-cpu-baseline > gpurun_out/${T}_bench_lvt_large.log 2>&1"
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_rocprof_lvt -o run -- python3 bench.py --workload lvt_large --no-cpu-baseline
exit 0
