#!/bin/bash
# round 4: the shape sort without global atomics (per-workgroup histograms,
# one workgroup per bin for the offsets): the whole GPU suite, the sort A/B
# (tools/r04_l.sh), rocprofv3 kernel stats of the C5 and C3 lines
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04t}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
echo "gpu tests ok"
bash tools/r04_l.sh $OUT || exit 2
for w in c5 c3; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_$w -o $w --output-format csv -- \
     python3 $R/bench.py --workload $w --steps 20 --warmup 2 --no-cpu-baseline --no-e2e > $R/$OUT/prof_$w.json 2> $R/$OUT/prof_$w.err) || exit 3
done
echo done
