set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/attn_bench.py 1003 1008 1011 1067 1131 1195 3 > gpurun_out/r2s4_attnmem.log 2>&1; echo "attn rc=$?"
