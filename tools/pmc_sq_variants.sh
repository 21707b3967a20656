#!/bin/bash
# SQ wave-state counters (one pass per leaf variant) over C2:
# tools/pmc_sq_variants.sh OUTDIR "1 4 6 14"
set -u
OUT=${1:-gpurun_out/pmc_sq}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
for V in $2; do
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
     SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD -d $R/$OUT/v$V -o v$V --output-format csv \
     -- python $R/tools/ab_leaf.py --rounds 1 --reps 2 --variants $V > $R/$OUT/v$V.log 2>&1) || exit 1
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS \
     SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS -d $R/$OUT/g$V -o g$V --output-format csv \
     -- python $R/tools/ab_leaf.py --rounds 1 --reps 2 --variants $V > $R/$OUT/g$V.log 2>&1) || exit 1
done
