#!/bin/bash
# SQ instruction / wave-state counters and HBM read bytes of the default leaf
# kernel (product library) on each leaf workload, one counter group per run:
#   tools/pmc_sq_workloads.sh OUTDIR "c2:1000000 c3:1250000 c5:6250000"
# Summarise with tools/pmc_sq_workloads_summary.py.
set -u
OUT=${1:-gpurun_out/pmc_sq_workloads}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
for WN in ${2:-c2:1000000 c3:1250000 c5:6250000}; do
  W=${WN%%:*}; N=${WN##*:}
  PROG="python $R/tools/ab_leaf.py --product --rounds 1 --reps 2 --variants ${VARIANT:-67} --workload $W --files $N"
  (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
     SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD -d $R/$OUT/s_$W -o s_$W --output-format csv \
     -- $PROG > $R/$OUT/s_$W.log 2>&1) || exit 1
  (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS \
     SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS -d $R/$OUT/g_$W -o g_$W --output-format csv \
     -- $PROG > $R/$OUT/g_$W.log 2>&1) || exit 2
  (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $R/$OUT/f_$W -o f_$W --output-format csv \
     -- $PROG > $R/$OUT/f_$W.log 2>&1) || exit 3
  (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $R/$OUT/w_$W -o w_$W --output-format csv \
     -- $PROG > $R/$OUT/w_$W.log 2>&1) || exit 4
  echo "$W done"
done
