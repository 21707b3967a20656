#!/bin/bash
# SQ instruction / wave-state counters of the C4 piece kernel (one counter
# group per run, as tools/pmc_sq_workloads.sh does for the leaf kernel).
set -u
OUT=${1:-gpurun_out/pmc_sq_piece}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
PROG="python $R/bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline"
(cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
   SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD -d $R/$OUT/s_c4 -o s_c4 --output-format csv \
   -- $PROG > $R/$OUT/s_c4.log 2>&1) || exit 1
(cd /tmp && timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS \
   SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS -d $R/$OUT/g_c4 -o g_c4 --output-format csv \
   -- $PROG > $R/$OUT/g_c4.log 2>&1) || exit 2
echo done
