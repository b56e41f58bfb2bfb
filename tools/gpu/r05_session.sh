#!/bin/bash
# Round-5 GPU session: the GPU test suite, the auxiliary-attention variants (linear tier A/B), and the
# LvT-Large bench.  Every GPU step has its own time limit; the set stops at the first failing step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r05d}
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n start"; timeout -k 10 "$t" "$@"; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
# failing tests (pytest rc 1) do not stop the set; anything else (a crash, a time limit) does
echo "[$(date +%T)] tests start"
timeout -k 10 1200 bash -c "python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1"
rc=$?; echo "[$(date +%T)] tests rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
step attn_long 300 bash -c "VP_DIAG_LIB=1 python -u tools/attn_bench.py long > gpurun_out/${T}_attn_long.log 2>&1"
step bench_lvt 400 bash -c "python -u bench.py --workload lvt_large --no-cpu-baseline > gpurun_out/${T}_bench_lvt_large.log 2>&1"
exit 0
