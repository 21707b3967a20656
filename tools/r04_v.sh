#!/bin/bash
# round 4: leaf variant 74 (67 with the split line-pair loop) against 67 in
# the ablation library: interleaved A/B (bit-exact check between them) on C2
# and C5, then one SQ / GRBM pass each on C2 (VALU per compression, clock)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04v}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
for wn in c2:1000000 c5:6250000; do
  w=${wn%%:*}; n=${wn##*:}
  timeout -k 10 400 python3 -u tools/ab_leaf.py --workload $w --files $n --variants 67,74 --rounds 7 --reps 3 \
    > $OUT/ab_split_$w.txt 2>&1 || exit 1
done
for v in 67 74; do
  PROG="python3 $R/tools/ab_leaf.py --rounds 1 --reps 2 --variants $v --workload c2 --files 1000000"
  (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES \
     -d $R/$OUT/g_$v -o g_$v --output-format csv -- $PROG > $R/$OUT/g_$v.log 2>&1) || exit 2
done
echo done
