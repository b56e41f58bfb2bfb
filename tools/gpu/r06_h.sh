#!/bin/bash
# Round-6: aux attention VAR 1024 (stage-unrolled chunk loop, immediate LDS offsets) vs the product kernel,
# bitwise; the product library's restructured (lambda) loop: forward hash vs round 5 and the LvT / long-attention tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06h
mkdir -p $O
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n start"; timeout -k 10 "$t" "$@"; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
test -f videoprism-mlx_amd/videoprism/libvideoprism_hip.so || { echo "product library missing"; exit 9; }
step attn_long 400 bash -c "VP_ATTN_VARIANTS=0,1024 python -u tools/attn_bench.py long > $O/attn_long.log 2>&1"
step hash_new 300 bash -c "python -u tools/ab_forward_hash.py > $O/hash_new.json 2>$O/hash_new.err"
step hash_r05 300 bash -c "python -u tools/ab_forward_hash.py .ab/r05 > $O/hash_r05.json 2>$O/hash_r05.err"
echo "[$(date +%T)] tests start"
timeout -k 10 900 bash -c "python -u -m pytest tests/test_gpu_lvt_frames.py tests/test_gpu_clip.py -m gpu -v -s --timeout 600 --timeout-method thread > $O/gputest.log 2>&1"
rc=$?; echo "[$(date +%T)] tests rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
exit 0
