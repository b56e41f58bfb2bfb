#!/bin/bash
# Round-3 experiment set (one gpurun call): parity of the fused temporal attention, fused/unfused
# A/B in the forward, spatial-attention ablations + the pipelined loop, ffn_layer1 tile orders.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu/measure.sh r03x "tests_k=temporal_attention_fused or full_depth_t16 or lvt_large_full" || exit $?
bash tools/gpu/ab_tattn.sh || exit $?
timeout -k 10 150 python -u tools/attn_bench.py 1003 1008 1011 1067 1131 1195 > gpurun_out/r03x_attn.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/gemm_bench.py grouped > gpurun_out/r03x_grouped.log 2>&1 || exit $?
