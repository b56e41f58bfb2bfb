#!/bin/bash
# Separate rocprofv3 --pmc passes (MI355X_MICROARCH.md: TCC slots limit FETCH/WRITE to
# their own passes; at most 8 SQ counters per pass).  Usage (from the repo root):
#   tools/pmc_passes.sh OUTDIR -- python3 script args...
set -e
OUT=$(realpath -m "$1"); shift; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM" \
         "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o pmc -- "$@" > "$OUT/p$i.log" 2>&1
done
