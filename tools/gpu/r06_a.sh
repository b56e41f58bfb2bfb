#!/bin/bash
# Round-6 first check: the new tests (LvT at other frame sizes, attention beyond 256 keys with paddings,
# temporal T > 256, concurrent handles), the LvT / clip / long-clip suites, the production gate's worst-ulp
# print, the forward-hash A/B against round 5's library, and one bench line with the measured MFMA peak.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06a
export TMPDIR=/tmp
O=gpurun_out/r06a
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n start"; timeout -k 10 "$t" "$@"; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
echo "[$(date +%T)] tests start"
timeout -k 10 900 bash -c "python -u -m pytest tests/test_gpu_lvt_frames.py tests/test_gpu_threads.py tests/test_gpu_clip.py tests/test_gpu_lvt_large.py 'tests/test_gpu_fullsize.py::test_production_shape_layers_vs_wbf16_oracle' -v -s --timeout 600 --timeout-method thread > $O/pytest.log 2>&1"
rc=$?; echo "[$(date +%T)] tests rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
step hash_new 300 bash -c "python -u tools/ab_forward_hash.py > $O/hash_new.json 2>$O/hash_new.err"
step hash_r05 300 bash -c "python -u tools/ab_forward_hash.py .ab/r05 > $O/hash_r05.json 2>$O/hash_r05.err"
step bench 300 bash -c "python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1"
exit 0
