#!/bin/bash
# round 5 (u): where the C3/C5 steps' copyBuffer blits come from: a kernel,
# memory-copy and HIP API trace of a short C5 bench run
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05u}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv \
   -d $R/$OUT/trace -o c5 -- python3 $R/bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
   --sustain-s 0 > $R/$OUT/c5.json 2> $R/$OUT/c5.err) || exit 1
echo done
