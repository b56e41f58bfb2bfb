set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/verify_clip_models.py --layers 1 --frames 4 > gpurun_out/r2s2_verify_bf16.log 2>&1; echo "verify bf16 rc=$?"
timeout -k 10 300 python -u tools/verify_clip_models.py --layers 1 --frames 4 --dtype f32 > gpurun_out/r2s2_verify_f32.log 2>&1; echo "verify f32 rc=$?"
timeout -k 10 300 python -u tools/benchmark_performance.py --framework both --runs 5 --warmup 2 --num-frames 8 --layers 2 --oracle-runs 1 > gpurun_out/r2s2_harness.log 2>&1; echo "bench rc=$?"
