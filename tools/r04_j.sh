#!/bin/bash
# round 4: C5's leaf in the shape-sorted order against the caller's order —
# time (interleaved, one process) and, one pass each, the clock the kernel
# holds (GRBM_GUI_ACTIVE / time) and its HBM read bytes: does gathering
# messages from all over the blob cost clock?
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04j}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
W=${W:-c5}; N=${N:-6250000}
timeout -k 10 300 python3 -u tools/ab_leaf.py --product --workload $W --files $N --variants 67 --sorts 1,0 \
  --rounds 3 --reps 3 > $OUT/ab_sort_$W.txt 2>&1 || exit 1
for so in 1 0; do
  PROG="python3 $R/tools/ab_leaf.py --product --rounds 1 --reps 2 --variants 67 --sorts $so --workload $W --files $N"
  (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU \
     -d $R/$OUT/g_$so -o g_$so --output-format csv -- $PROG > $R/$OUT/g_$so.log 2>&1) || exit 2
  (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $R/$OUT/f_$so -o f_$so --output-format csv \
     -- $PROG > $R/$OUT/f_$so.log 2>&1) || exit 3
done
echo done
