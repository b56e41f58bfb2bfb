set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2s2_gputest3.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/r2s2_bench4.log 2>&1
