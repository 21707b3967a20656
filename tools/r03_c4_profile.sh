#!/bin/bash
# C4 kernel stats and HBM-traffic PMC passes of the default piece kernels
# (through gpurun, from the repo root); the first failure ends the script.
set -o pipefail
OUT=${1:-gpurun_out/r03_c4_profile}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_c4 -o c4 --output-format csv -- \
   python $R/bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $R/$OUT/prof_c4.log 2>&1) || exit 1
echo "rocprof ok"
bash tools/pmc_traffic.sh $OUT/pmc_c4 -- python $R/bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline \
  > $OUT/pmc_c4.log 2>&1 || exit 2
echo done
