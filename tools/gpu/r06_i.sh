#!/bin/bash
# Round-6: spatial attention with its 8 tiles written out (immediate V offsets) vs the committed kernel: kernel-level
# bitwise A/B (tools/ab_lib.py spatial), whole-forward alternating A/B, and the attention / encoder tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06i
mkdir -p $O
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n start"; timeout -k 10 "$t" "$@"; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
test -f videoprism-mlx_amd/videoprism/libvideoprism_hip.so || { echo "product library missing"; exit 9; }
step ab_lib 300 bash -c "python -u tools/ab_lib.py spatial .ab/unroll_base/videoprism-mlx_amd/videoprism/libvideoprism_hip.so > $O/ab_lib.log 2>&1"
step ab 600 bash -c "bash tools/gpu/ab_bench.sh unroll_base 3 > $O/ab.log 2>&1"
echo "[$(date +%T)] tests start"
timeout -k 10 900 bash -c "python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_encoder.py tests/test_gpu_geometry.py -m gpu -v -s --timeout 600 --timeout-method thread > $O/gputest.log 2>&1"
rc=$?; echo "[$(date +%T)] tests rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
exit 0
