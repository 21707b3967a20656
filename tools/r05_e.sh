#!/bin/bash
# round 5 (e): leaf variants 75-77 (quad tree levels / phase-4 bits) against
# 67, same process, interleaved (ablation library), C2 and C5; then (d)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05e}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_leaf.py --variants 67,75,76,77 --rounds 7 --reps 4 \
  > $OUT/ab_leaf_c2.txt 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab_leaf.py --workload c5 --files 6250000 --variants 67,75,76,77 --rounds 7 --reps 4 \
  > $OUT/ab_leaf_c5.txt 2>&1 || exit 2
echo "ab ok"
bash tools/r05_d.sh $OUT/d || exit 3
echo done
