#!/bin/bash
# PMC FETCH / WRITE and kernel timings of the three ffn_layer1 tile orders (tools/gemm_bench.py
# grouped_pmc), one rocprofv3 pass each, outputs under gpurun_out/$1_*.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r03grp}
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o run -- python3 tools/gemm_bench.py grouped_pmc > gpurun_out/${T}_kt.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_p1 -o pmc -- python3 tools/gemm_bench.py grouped_pmc > gpurun_out/${T}_p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_p2 -o pmc -- python3 tools/gemm_bench.py grouped_pmc > gpurun_out/${T}_p2.log 2>&1
echo done
