set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/gemm_bench.py early > gpurun_out/r2s2_early.log 2>&1
