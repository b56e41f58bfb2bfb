#!/bin/bash
# Round-4 second measurement set (one gpurun call): the other bench workloads, the auxiliary-attention
# scalar/packed A/B (diag library), the Base PMC traffic record and the Base parity-stage split.
# Every GPU step has its own time limit; the set stops at the first failing step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r04b}
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n start"; timeout -k 10 "$t" "$@"; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step tests_patch 300 bash -c "python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ingest.py tests/test_gpu_fullsize.py -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/${T}_tests_patch.log 2>&1"
step bench_large 300 bash -c "python -u bench.py --workload large --no-cpu-baseline > gpurun_out/${T}_bench_large.log 2>&1"
step bench_lvt 400 bash -c "python -u bench.py --workload lvt_large > gpurun_out/${T}_bench_lvt_large.log 2>&1"
step attn_long 200 bash -c "python -u tools/attn_bench.py long > gpurun_out/${T}_attn_long.log 2>&1"
step tattn 200 bash -c "VP_DIAG_LIB=1 python -u tools/gemm_bench.py tattn > gpurun_out/${T}_tattn.log 2>&1"
step stages_base 300 bash -c "python -u tools/parity_stages.py --base --json gpurun_out/${T}_stages_base.json > gpurun_out/${T}_stages_base.log 2>&1"
step pmc_base 600 bash tools/pmc_traffic.sh gpurun_out/${T}_pmc_base base
cp profiles/traffic_r04_base.json gpurun_out/ 2>/dev/null
exit 0
