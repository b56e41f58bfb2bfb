#!/bin/bash
# HBM traffic (+ clock / MFMA-busy) counters of the bench's kernels, one rocprofv3 --pmc pass per
# group (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass), then the per-symbol
# traffic record bench.py reads for roofline.traffic.
# Usage (on the GPU box, from the repo root): tools/pmc_traffic.sh OUTDIR WORKLOAD [RECORD]
#   RECORD defaults to profiles/traffic_r06_WORKLOAD.json
set -e
OUT=$(realpath -m "$1")
WL=${2:-base}
REC=${3:-profiles/traffic_r06_${WL}.json}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o pmc -- \
    python3 "$ROOT/bench.py" --workload "$WL" --steps 2 --warmup 1 --no-cpu-baseline --no-peak > "$OUT/p$i.log" 2>&1
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT" --json "$REC" "$WL" > "$OUT/summary.txt"
cat "$OUT/summary.txt"
