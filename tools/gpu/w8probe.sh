#!/bin/bash
# 4-wave vs 8-wave GEMM kernels at the forward's shapes (epilogue and no-epilogue builds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/gemm_bench.py w8epi > gpurun_out/w8_epi.log 2>&1 || exit $?
