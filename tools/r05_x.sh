#!/bin/bash
# round 5 (x): the C2 line's e2e legs with the written files synced before
# their timed reads (bench.settle_files), twice, and the C3 line once
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05x}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 500 python -u bench.py --sustain-s 0 > $OUT/bench_c2_$rep.json 2> $OUT/bench_c2_$rep.err || exit 1
  echo "c2 rep $rep ok"
done
timeout -k 10 500 python -u bench.py --workload c3 --steps 5 --warmup 2 --sustain-s 0 > $OUT/bench_c3.json \
  2> $OUT/bench_c3.err || exit 2
echo done
