#!/bin/bash
# Separate rocprofv3 --pmc passes (MI355X_MICROARCH.md: TCC slots limit FETCH/WRITE to
# their own passes).  Usage: tools/pmc_passes.sh OUTDIR -- python3 script args...
set -e
OUT=$1; shift; shift
mkdir -p $OUT; cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o pmc -- "$@" > $OUT/p$i.log 2>&1
done
