set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/graph_probe.py 2>&1 | grep -v amdgpu.ids > gpurun_out/r2s3_graph.log
