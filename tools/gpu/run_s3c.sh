set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_encoder.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2s4_s3c_tests.log 2>&1; echo "tests rc=$?"
VP_DIAG_LIB=1 timeout -k 10 300 python -u tools/gemm_bench.py s3 > gpurun_out/r2s4_s3c.log 2>&1; echo "s3 rc=$?"
for i in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r2s4_s3c_new$i.log 2>&1 && echo new-ok
done
