#!/bin/bash
# The sequence-packed attention (16 < S <= 256): kernel tests, every forward test that reaches it (long clips,
# padded frames, other patch grids, encoder, CLIP), then the long-clip benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${1:-r05q}
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n start"; timeout -k 10 "$t" "$@"; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step tests 900 bash -c "python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_long_clips.py tests/test_gpu_geometry.py tests/test_gpu_encoder.py tests/test_gpu_clip.py tests/test_gpu_boundary.py -m gpu -v -s --timeout 600 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1"
step t64 300 bash -c "python -u bench.py --frames 64 --batch 8 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/${T}_bench_t64.log 2>&1"
step t32 300 bash -c "python -u bench.py --frames 32 --batch 16 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/${T}_bench_t32.log 2>&1"
exit 0
