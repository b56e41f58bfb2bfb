#!/bin/bash
# Round-6: ffn_layer2's K-loop / epilogue split (ablation builds) with PMC counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06g
mkdir -p $O
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n start"; timeout -k 10 "$t" "$@"; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
test -f videoprism-mlx_amd/videoprism/libvideoprism_hip.so || { echo "product library missing"; exit 9; }
step ffn2_split 300 bash -c "python -u tools/ffn1_split.py ffn2 > $O/ffn2_split.log 2>&1"
step pmc_ffn2 600 bash tools/pmc_passes.sh $O/pmc_ffn2 -- python3 tools/ffn1_split.py ffn2
step pmc_ffn2_sum 120 bash -c "python3 tools/pmc_summary.py $O/pmc_ffn2 > $O/pmc_ffn2_summary.txt 2>&1"
exit 0
