#!/bin/bash
# rocprofv3 kernel traces + stats of the four bench lines (the first half of
# tools/r03_refresh.sh b, without the PMC / SQ passes); then
# tools/rocprof_vs_bench.py OUT compares each dominant kernel's traced launch
# times with the same run's HIP-event figure.
set -o pipefail
OUT=${1:-gpurun_out/r03_rocprof_final}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
for w in c2 c3 c5; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_$w -o $w --output-format csv -- \
     python $R/bench.py --workload $w --steps 20 --warmup 2 --no-cpu-baseline --no-e2e > $R/$OUT/prof_$w.log 2>&1) || exit 1
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_c4 -o c4 --output-format csv -- \
   python $R/bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $R/$OUT/prof_c4.log 2>&1) || exit 2
echo done
