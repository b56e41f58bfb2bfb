#!/bin/bash
# Round-6: the auxiliary attention's A/B builds (one-wave kernel: packed linear tier 128, static priority for waves
# 4-7 256; the two-waves-per-SIMD alternating kernel 512 (+128 / +256)) at the LvT-Large shape, bitwise against
# the product kernel; then the bench line with the fixed MFMA peak microbenchmark.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06b
export TMPDIR=/tmp
O=gpurun_out/r06b
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n start"; timeout -k 10 "$t" "$@"; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step attn_long 400 bash -c "VP_ATTN_VARIANTS=0,128,256,384,512,640,768 python -u tools/attn_bench.py long > $O/attn_long.log 2>&1"
step bench 300 bash -c "python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1"
exit 0
