#!/bin/bash
# round 4: the dedup tests with both tables; one rank's device stages of the
# bucket protocol at world 8 (C5, C3) and 2
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04g}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dist_dedup.py -m gpu -v --timeout 200 --timeout-method thread > $OUT/pytest_dedup.log 2>&1 || exit 1
for wl in c5:8 c3:8 c5:2; do
  w=${wl%%:*}; W=${wl##*:}
  timeout -k 10 200 python -u tools/dedup_probe.py --workload $w --reps 10 --world $W --combines sort,hash > $OUT/world_${w}_$W.json 2> $OUT/world_${w}_$W.err || exit 2
done
echo done
