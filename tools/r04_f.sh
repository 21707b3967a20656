#!/bin/bash
# round 4: PMC passes at HEAD — HBM traffic of the C2 leaf and C4 piece
# kernels, SQ counters of the leaf kernel on C2 and C5
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04f}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/pmc_traffic.sh $OUT/pmc_c2 > $OUT/pmc_c2.log 2>&1 || exit 1
bash tools/pmc_traffic.sh $OUT/pmc_c4 -- python3 $R/bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e \
  > $OUT/pmc_c4.log 2>&1 || exit 2
VARIANT=67 bash tools/pmc_sq_workloads.sh $OUT/sqw "c2:1000000 c5:6250000" > $OUT/sqw.log 2>&1 || exit 3
echo done
