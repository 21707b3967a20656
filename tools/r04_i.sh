#!/bin/bash
# round 4: the workgroup-aggregated hash combine (dedup tests, one rank's
# bucket stages at world 8 / 2, sort vs hash); the C3/C5 lines with the
# dedup on the step's own stream; then the plain N = 8 launch rehearsed with
# gloo (tools/r04_h.sh)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04i}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dist_dedup.py -m gpu -v --timeout 200 --timeout-method thread > $OUT/pytest_dedup.log 2>&1 || exit 1
for wl in c5:8 c3:8 c5:2; do
  w=${wl%%:*}; W=${wl##*:}
  timeout -k 10 200 python -u tools/dedup_probe.py --workload $w --reps 10 --world $W --combines sort,hash > $OUT/world_${w}_$W.json 2> $OUT/world_${w}_$W.err || exit 2
done
for w in c5 c3; do
  timeout -k 10 300 python3 -u bench.py --workload $w --no-e2e > $OUT/bench_$w.json 2> $OUT/bench_$w.err || exit 3
done
bash tools/r04_h.sh $OUT || exit 4
echo done
