#!/bin/bash
# degree-5 GELU polynomial (product library) vs degree 6 (the diag library, built from the previous
# sources): bf16 full-depth parity printouts for both, the full GPU suite, forward A/B alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-g5}
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n start"; timeout -k 10 "$t" "$@"; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
K="full_depth_t16_bf16 or full_base_b1_bf16 or lvt_large_full_depth or clip_full_lvt_base or base_dims_bf16 or fused_vs_unfused"
step par5 600 bash -c "python -u -m pytest tests -m gpu -q -s -k '$K' --timeout 300 --timeout-method thread > gpurun_out/${T}_par5.log 2>&1"
step par6 600 bash -c "VP_DIAG_LIB=1 python -u -m pytest tests -m gpu -q -s -k '$K' --timeout 300 --timeout-method thread > gpurun_out/${T}_par6.log 2>&1"
for i in 1 2; do
  step d5_$i 200 bash -c "python -u bench.py --no-cpu-baseline > gpurun_out/${T}_d5_$i.log 2>&1"
  step d6_$i 200 bash -c "VP_DIAG_LIB=1 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_d6_$i.log 2>&1"
done
step tests 900 bash -c "python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1"
