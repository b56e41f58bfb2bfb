set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT/tools:$PYTHONPATH
timeout -k 10 200 python -u tools/qa_bench.py 512 2>&1 | grep -v amdgpu.ids > gpurun_out/r2s2_qa_bench2.log
