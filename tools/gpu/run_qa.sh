set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "qkv_attention" --timeout 120 --timeout-method thread > gpurun_out/r2s2_qa_test.log 2>&1
