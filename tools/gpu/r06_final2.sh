#!/bin/bash
# Round-6 final record on the committed sources (REC=name, default r06x): the GPU test suite, smoke(), the Base bench
# (with the CPU baseline), rocprof kernel statistics of the Base and LvT-Large benches, the PMC traffic records of
# the three workloads (bench.py's roofline.traffic, keyed on the source fingerprint), the three benches with
# those records in place, and the fp32 benches with theirs.  Every GPU step has its own limit; failing tests are
# recorded and the set goes on.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${REC:-r06x}
mkdir -p $O
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n start"; timeout -k 10 "$t" "$@"; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
test -f videoprism-mlx_amd/videoprism/libvideoprism_hip.so || { echo "product library missing"; exit 9; }
# three gpurun calls (each within the 20-minute limit): PHASE 1 = tests, smoke, the Base bench and the rocprof runs;
# PHASE 2 = the PMC traffic records and the benches that quote them; PHASE 3 = the same for --dtype f32
PHASE=${1:-1}
if [ "$PHASE" = 1 ]; then
echo "[$(date +%T)] tests start"
timeout -k 10 1000 bash -c "python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > $O/gputest.log 2>&1"
rc=$?; echo "[$(date +%T)] tests rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
step smoke 300 bash -c "python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1"
step bench_base 300 bash -c "python -u bench.py > $O/bench_base.log 2>&1"
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rocprof -o run -- python3 bench.py --no-cpu-baseline --no-peak
step rocprof_lvt 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rocprof_lvt -o run -- python3 bench.py --workload lvt_large --no-peak
exit 0
fi
if [ "$PHASE" = 2 ]; then
step pmc_base 600 bash tools/pmc_traffic.sh $O/pmc_base base profiles/traffic_r06_base.json
step pmc_large 600 bash tools/pmc_traffic.sh $O/pmc_large large profiles/traffic_r06_large.json
step pmc_lvt 600 bash tools/pmc_traffic.sh $O/pmc_lvt lvt_large profiles/traffic_r06_lvt_large.json
cp profiles/traffic_r06_base.json profiles/traffic_r06_large.json profiles/traffic_r06_lvt_large.json $O/ 2>/dev/null
step bench_base2 300 bash -c "python -u bench.py > $O/bench_base2.log 2>&1"
step bench_large 300 bash -c "python -u bench.py --workload large --no-cpu-baseline > $O/bench_large.log 2>&1"
step bench_lvt 400 bash -c "python -u bench.py --workload lvt_large > $O/bench_lvt_large.log 2>&1"
exit 0
fi
if [ "$PHASE" = 3 ]; then  # the fp32 benches (bench.py --dtype f32) with their own PMC traffic record
step pmc_f32 600 bash tools/pmc_traffic.sh $O/pmc_base_f32 base - f32
cp profiles/traffic_r06_base_f32.json $O/ 2>/dev/null
step bench_f32 600 bash -c "python -u bench.py --dtype f32 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_base_f32.log 2>&1"
step bench_large_f32 400 bash -c "python -u bench.py --dtype f32 --workload large --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_large_f32.log 2>&1"
step bench_lvt_f32 500 bash -c "python -u bench.py --dtype f32 --workload lvt_large --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_lvt_large_f32.log 2>&1"
exit 0
fi
