#!/bin/bash
# Round-6 check: the whole GPU suite on the current sources, then smoke().
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06e
mkdir -p $O
export TMPDIR=/tmp
test -f videoprism-mlx_amd/videoprism/libvideoprism_hip.so || { echo "product library missing"; exit 9; }
echo "[$(date +%T)] tests start"
timeout -k 10 1500 bash -c "python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > $O/gputest.log 2>&1"
rc=$?; echo "[$(date +%T)] tests rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 bash -c "python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1"; echo "smoke rc=$?"
exit 0
