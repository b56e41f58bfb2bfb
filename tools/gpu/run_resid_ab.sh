set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/gemm_bench.py resid > gpurun_out/r2s2_resid_ab.log 2>&1
