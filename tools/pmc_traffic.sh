#!/bin/bash
# HBM traffic of the C2 leaf kernel from PMC counters (separate passes, as
# MI355X_MICROARCH.md prescribes). Usage: tools/pmc_traffic.sh <outdir> [variant]
set -u
OUT=${1:-gpurun_out/pmc_traffic}
VAR=${2:-43}  # the default leaf variant (kDefaultLeafVariant)
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
pass fetch FETCH_SIZE &&
pass write WRITE_SIZE &&
pass dram TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum &&
pass req TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum &&
pass tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT
