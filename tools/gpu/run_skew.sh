set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_bench.py $1 2>&1 | grep -v amdgpu.ids > gpurun_out/r2s3_$1.log
