#!/bin/bash
# 8-wave ffn_layer1 GEMM (gemm_bf16_w8b.hip): bitwise tests, isolated A/B, (forward A/B: it ran as ffn_layer1 under VP_FFN1_W8B=1 in the session that measured it; DESIGN)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-w8b}
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n start"; timeout -k 10 "$t" "$@"; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step test 300 bash -c "python -u tools/ab_tests.py > gpurun_out/${T}_test.log 2>&1"
step gemm 300 bash -c "python -u tools/gemm_bench.py w8b > gpurun_out/${T}_gemm.log 2>&1"




