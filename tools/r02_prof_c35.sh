#!/bin/bash
# rocprofv3 kernel stats of the C3 and C5 bench steps (dedup + leaf + sort)
set -o pipefail
OUT=${1:-gpurun_out/r02_prof_c35}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
for w in c3 c5; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_$w -o $w --output-format csv -- \
     python $R/bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > $R/$OUT/prof_$w.log 2>&1) || exit 1
done
echo done
