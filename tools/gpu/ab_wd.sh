#!/bin/bash
# W-direct GEMM (gemm_bf16_w4.hip WD): isolated A/B + bitwise check, GPU tests with WD on, then
# the forward with and without it (VP_W4_WD=1), alternating on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-wd}
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n start"; timeout -k 10 "$t" "$@"; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step gemm 300 bash -c "python -u tools/gemm_bench.py wd > gpurun_out/${T}_gemm.log 2>&1"
step tests 900 bash -c "VP_W4_WD=1 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1"
for i in 1 2; do
  step on$i 200 bash -c "VP_W4_WD=1 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_on_$i.log 2>&1"
  step off$i 200 bash -c "python -u bench.py --no-cpu-baseline > gpurun_out/${T}_off_$i.log 2>&1"
done
