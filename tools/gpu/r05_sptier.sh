#!/bin/bash
# Tiered capped numerator in the spatial attention: parity tests that reach it (kernel tests, full-size
# Base / Large, LvT), then the whole-forward A/B against the previous revision (.ab/pre), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${1:-r05v}
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n start"; timeout -k 10 "$t" "$@"; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step tests 900 bash -c "python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_clip.py tests/test_gpu_lvt_large.py tests/test_gpu_encoder.py -m gpu -v -s --timeout 600 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1"
step ab 900 bash -c "bash tools/gpu/ab_bench.sh pre 3 > gpurun_out/${T}_ab.txt 2>&1"
exit 0
