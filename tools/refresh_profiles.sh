#!/bin/bash
# Round profiles: all bench lines (with CPU baselines), rocprofv3 kernel stats
# of the C2 headline and C5, and the C2 PMC traffic passes.
# usage: tools/refresh_profiles.sh OUTDIR
set -e
OUT=${1:-gpurun_out/refresh}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
tools/bench_all.sh $OUT
for w in c2 c5; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_$w -o $w --output-format csv \
     -- python $R/bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > $R/$OUT/prof_$w.log 2>&1)
done
tools/pmc_traffic.sh $OUT/pmc 43 > $OUT/pmc.log 2>&1  # 43 = the default leaf variant
