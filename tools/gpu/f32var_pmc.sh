#!/bin/bash
# fp32 GEMM variants (tools/gemm_f32_var.py) timed, then their HBM traffic in two rocprofv3 --pmc passes
# (FETCH_SIZE, WRITE_SIZE: separate passes) summarised per kernel symbol by tools/pmc_summary.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${REC:-f32var_pmc}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/gemm_f32_var.py ${B:-8} > $O/time.txt 2>&1 || exit $?
i=0
for P in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o pmc -- python3 tools/gemm_f32_var.py ${B:-8} > $O/p$i.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py $O > $O/summary.txt
