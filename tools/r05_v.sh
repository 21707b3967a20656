#!/bin/bash
# round 5 (v): the leaf kernel's HBM traffic per launch from PMC passes at the
# final HEAD (tools/pmc_traffic.sh over tools/ab_leaf.py, the product variant
# 67), C2, C3 and C5 — summarised by tools/pmc_summarize.py
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05v}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
for wf in ${WL:-c2:1000000 c3:1250000 c5:6250000}; do
  w=${wf%:*}; f=${wf#*:}
  bash tools/pmc_traffic.sh $OUT/$w -- python3 $R/tools/ab_leaf.py --product --rounds 1 --reps 2 --variants 67 \
    --workload $w --files $f > $OUT/$w.log 2>&1 || exit 1
  find $OUT/$w -name '*.db' -delete
  echo "$w ok"
done
echo done
