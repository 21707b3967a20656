#!/bin/bash
# SQ instruction / wave-state counters of leaf variants of the ABLATION
# library, per workload, two counter groups per run (the VALU mix; cycles,
# LDS, SALU): tools/pmc_sq_ab.sh OUTDIR "67 78" "c2:1000000 c5:6250000"
# Summarise with tools/pmc_sq_ab_summary.py OUTDIR.
set -u
OUT=${1:-gpurun_out/pmc_sq_ab}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
for V in ${2:-67 78}; do
  for WN in ${3:-c2:1000000 c5:6250000}; do
    W=${WN%%:*}; N=${WN##*:}
    PROG="python $R/tools/ab_leaf.py --rounds 1 --reps 2 --variants $V --workload $W --files $N"
    (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
       SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD -d $R/$OUT/s_${W}_$V -o s --output-format csv \
       -- $PROG > $R/$OUT/s_${W}_$V.log 2>&1) || exit 1
    (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS \
       SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS -d $R/$OUT/g_${W}_$V -o g --output-format csv \
       -- $PROG > $R/$OUT/g_${W}_$V.log 2>&1) || exit 2
    find $R/$OUT/s_${W}_$V $R/$OUT/g_${W}_$V -type f ! -name "*counter_collection.csv" -delete
    echo "$V $W done"
  done
done
