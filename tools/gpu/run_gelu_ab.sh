set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/keep_ab.py > gpurun_out/r2s2_keep_ab.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py fold > gpurun_out/r2s2_gemm_fold2.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_encoder.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2s2_gputest2.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r2s2_bench2.log 2>&1
