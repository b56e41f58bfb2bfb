set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/graph_probe.py > gpurun_out/r2s4_graph.log 2>&1; echo "graph rc=$?"
timeout -k 10 300 python -u tools/gemm_bench.py epilds > gpurun_out/r2s4_epilds.log 2>&1 && echo epilds-ok && \
timeout -k 10 400 python -u tools/gemm_bench.py skew > gpurun_out/r2s4_skew.log 2>&1 && echo skew-ok
