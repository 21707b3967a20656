#!/bin/bash
# round 5 (z): code placement of the leaf kernel — variant 67 against the
# same kernel shifted by 4, 8, 12 and 16 bytes (ablation variants 79-82,
# s_nop at the entry), same-process interleaved A/B on C2 and C5
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05z}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab_leaf.py --variants 67,79,80,81,82 --rounds 7 --reps 4 \
  > $OUT/ab_place_c2.txt 2>&1 || exit 1
timeout -k 10 500 python -u tools/ab_leaf.py --workload c5 --files 6250000 --variants 67,79,80,81,82 --rounds 7 --reps 4 \
  > $OUT/ab_place_c5.txt 2>&1 || exit 2
echo done
