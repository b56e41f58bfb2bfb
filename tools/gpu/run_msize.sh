set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/gemm_bench.py msize 2>&1 | grep -v amdgpu.ids > gpurun_out/r2s2_msize.log
