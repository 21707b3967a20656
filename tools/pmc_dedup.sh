#!/bin/bash
# HBM traffic of the identifier dedup (tools/dedup_probe.py), one counter
# group per rocprofv3 run (MI355X_MICROARCH.md, HBM / rocprofv3 section),
# plus a kernel trace; summarised by tools/pmc_dedup_summary.py.
# usage: tools/pmc_dedup.sh <outdir> <workload c3|c5> [reps] [full | probe flags...]
#   full: the whole corpus (tools/dedup_full.py --no-parity: C3 10 M, C5 50 M files)
set -u
OUT=${1:-gpurun_out/pmc_dedup}
W=${2:-c5}
REPS=${3:-10}
shift 3 2>/dev/null || shift $#
PROG=(tools/dedup_probe.py --workload $W --reps $REPS "$@")
if [ "${1:-}" = full ]; then
  shift
  PROG=(tools/dedup_full.py --workload $W --reps $REPS --no-parity "$@")
fi
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
pass() {
  local name=$1; shift
  echo "== pass $name: $*"
  (cd /tmp && timeout -s KILL 240 rocprofv3 "$@" -d $R/$OUT/$name -o $name --output-format csv -- \
     python3 $R/"${PROG[@]}" > $R/$OUT/$name.log 2>&1)
  local rc=$?
  echo "rc=$rc"
  return $rc
}
pass trace --kernel-trace --stats &&
pass fetch --pmc FETCH_SIZE &&
pass write --pmc WRITE_SIZE &&
pass req --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum &&
pass tcc --pmc TCC_HIT_sum TCC_MISS_sum
