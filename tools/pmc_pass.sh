#!/bin/bash
# PMC counter passes over the C2 leaf kernel (one counter group per run, as
# MI355X_MICROARCH.md prescribes). Usage: tools/pmc_pass.sh <outdir> [variant]
# Each pass: timeout -s KILL; stops at the first failure.
set -u
OUT=${1:-gpurun_out/pmc}
VAR=${2:-1}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
PROG="python $R/tools/ab_leaf.py --rounds 1 --reps 2 --variants $VAR"
pass() {
  local name=$1; shift
  echo "== pass $name: $*"
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" -d $R/$OUT/$name -o $name --output-format csv -- $PROG \
     > $R/$OUT/$name.log 2>&1)
  local rc=$?
  echo "rc=$rc"
  return $rc
}
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD &&
pass grbm GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS &&
pass ta TA_BUSY_avr TA_BUSY_max TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum &&
pass fetch FETCH_SIZE &&
pass tcc TCC_HIT_sum TCC_MISS_sum
