#!/bin/bash
# round 4: is the shape sort worth its kernels? The whole batch (sort + scan +
# leaf + finish, "seq") with and without it, interleaved in one process per
# workload (tools/ab_leaf.py --sorts 1,0)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04l}
mkdir -p $OUT
export TMPDIR=/tmp
for wn in c5:6250000 c3:1250000 c2:1000000; do
  w=${wn%%:*}; n=${wn##*:}
  timeout -k 10 400 python3 -u tools/ab_leaf.py --product --workload $w --files $n --variants 67 --sorts 1,0 \
    --rounds 7 --reps 3 > $OUT/ab_sort_$w.txt 2>&1 || exit 1
done
echo done
