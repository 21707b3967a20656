#!/bin/bash
# round 5 (g): leaf variants 67 / 75 / 77 / 78 interleaved in one process on
# C2 and C5, then SQ counter passes of 67 and 78
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05g}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_leaf.py --variants 67,75,77,78 --rounds 9 --reps 4 \
  > $OUT/ab_leaf_c2.txt 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab_leaf.py --workload c5 --files 6250000 --variants 67,75,77,78 --rounds 9 --reps 4 \
  > $OUT/ab_leaf_c5.txt 2>&1 || exit 2
echo "ab ok"
bash tools/pmc_sq_ab.sh $OUT/sq "67 78" "c2:1000000 c5:6250000" || exit 3
echo done
