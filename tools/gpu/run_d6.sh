set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VP_DIAG_LIB=1 timeout -k 10 300 python -u tools/gemm_bench.py grouped > gpurun_out/r2s4_d6.log 2>&1; echo "d6 rc=$?"
