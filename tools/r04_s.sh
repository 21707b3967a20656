#!/bin/bash
# round 4: the stays rows by the library's own ordered compaction
# (select_stays) instead of hipcub's select: the whole GPU suite, the C5 / C3
# lines, rocprofv3 kernel stats of the C5 line
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04s}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
echo "gpu tests ok"
for w in c5 c3; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || exit 2
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_c5 -o c5 --output-format csv -- \
   python3 $R/bench.py --workload c5 --steps 20 --warmup 2 --no-cpu-baseline --no-e2e > $R/$OUT/prof_c5.json 2> $R/$OUT/prof_c5.err) || exit 3
echo done
