#!/bin/bash
# HBM traffic (+ clock / MFMA-busy) counters of the bench's kernels, one rocprofv3 --pmc pass per
# group (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass), then the per-symbol
# traffic record bench.py reads for roofline.traffic.
# Usage (on the GPU box, from the repo root): tools/pmc_traffic.sh OUTDIR WORKLOAD [RECORD] [DTYPE]
#   RECORD defaults to profiles/traffic_r06_WORKLOAD.json (DTYPE f32: traffic_r06_WORKLOAD_f32.json,
#   the bench's `--dtype f32` kernels; the record's workload label is WORKLOAD_f32)
set -e
OUT=$(realpath -m "$1")
WL=${2:-base}
DT=${4:-bf16}
LABEL=$WL
[ "$DT" = f32 ] && LABEL=${WL}_f32
REC=${3:-profiles/traffic_r06_${LABEL}.json}
[ -n "$3" ] && [ "$3" != - ] || REC=profiles/traffic_r06_${LABEL}.json
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o pmc -- \
    python3 "$ROOT/bench.py" --workload "$WL" --dtype "$DT" --steps 2 --warmup 1 --no-cpu-baseline --no-peak > "$OUT/p$i.log" 2>&1
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT" --json "$REC" "$LABEL" > "$OUT/summary.txt"
cat "$OUT/summary.txt"
