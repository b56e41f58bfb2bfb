#!/bin/bash
# Round-6: the GEMM epilogue waits (ffn1's LN-fold constants of all columns in LDS; the first K-tile after a
# row-blocked epilogue leaves that epilogue's 32 stores in flight) -- the whole GPU suite, the bitwise forward
# hash against round 5's library, the ffn1 split, and an alternating whole-forward A/B against the previous tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06f
mkdir -p $O
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n start"; timeout -k 10 "$t" "$@"; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
test -f videoprism-mlx_amd/videoprism/libvideoprism_hip.so || { echo "product library missing"; exit 9; }
step hash_new 300 bash -c "python -u tools/ab_forward_hash.py > $O/hash_new.json 2>$O/hash_new.err"
step hash_r05 300 bash -c "python -u tools/ab_forward_hash.py .ab/r05 > $O/hash_r05.json 2>$O/hash_r05.err"
step ffn1_split 300 bash -c "python -u tools/ffn1_split.py > $O/ffn1_split.log 2>&1"
step ab_pre 600 bash -c "bash tools/gpu/ab_bench.sh pre 3 > $O/ab_pre.log 2>&1"
step ab_blk 600 bash -c "bash tools/gpu/ab_bench.sh blk 3 > $O/ab_blk.log 2>&1"
echo "[$(date +%T)] tests start"
timeout -k 10 900 bash -c "python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > $O/gputest.log 2>&1"
rc=$?; echo "[$(date +%T)] tests rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
exit 0
