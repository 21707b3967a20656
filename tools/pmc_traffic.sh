#!/bin/bash
# HBM traffic of one kernel from PMC counters, each counter group in a run of
# its own (MI355X_MICROARCH.md, HBM / rocprofv3 section).
# Usage: tools/pmc_traffic.sh <outdir> [-- program args...]
# (default program: the C2 leaf kernel through tools/ab_leaf.py, the default variant 67)
set -u
OUT=${1:-gpurun_out/pmc_traffic}
shift || true
R=$(pwd)
if [ "${1:-}" = "--" ]; then shift; PROG="$*"; else PROG="python $R/tools/ab_leaf.py --product --rounds 1 --reps 2 --variants 67"; fi
mkdir -p $OUT
export TMPDIR=/tmp
pass() {
  local name=$1; shift
  echo "== pass $name: $*"
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc "$@" -d $R/$OUT/$name -o $name --output-format csv -- $PROG \
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
