#!/bin/bash
# Round-6: bench line with the measured MFMA peak; the aux attention's static-priority build again; the ffn_layer1
# K-loop / epilogue split with PMC counters (the close-out of the ping-pong GEMM question); PMC of the aux
# attention's one-wave vs alternating kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06d
mkdir -p $O
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n start"; timeout -k 10 "$t" "$@"; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
test -f videoprism-mlx_amd/videoprism/libvideoprism_hip.so || { echo "product library missing"; exit 9; }
step bench 300 bash -c "python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1"
step ffn1_split 300 bash -c "python -u tools/ffn1_split.py > $O/ffn1_split.log 2>&1"
step pmc_ffn1 600 bash tools/pmc_passes.sh $O/pmc_ffn1 -- python3 tools/ffn1_split.py
step pmc_ffn1_sum 120 bash -c "python3 tools/pmc_summary.py $O/pmc_ffn1 > $O/pmc_ffn1_summary.txt 2>&1"
step pmc_attn 600 env VP_ATTN_VARIANTS=0,512,256 bash tools/pmc_passes.sh $O/pmc_attn -- python3 tools/attn_bench.py long
step pmc_attn_sum 120 bash -c "python3 tools/pmc_summary.py $O/pmc_attn > $O/pmc_attn_summary.txt 2>&1"
exit 0
