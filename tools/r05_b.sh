#!/bin/bash
# round 5 (b): the whole GPU suite and smoke after the hipCUB removal, then
# the C3 / C5 lines (the exact fallback and node tests run in the suite)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05b}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
echo "gpu tests ok"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 2
for w in c3 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || exit 3
done
echo done
