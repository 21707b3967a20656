#!/bin/bash
# round 5, final refresh at HEAD (a): the whole GPU suite and smoke, then the
# C2 (default), C3, C5 and C4 bench lines
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05fa}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
echo "gpu tests ok"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 3
echo "c2 ok"
for w in c3 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || exit 4
  echo "$w ok"
done
timeout -k 10 600 python3 -u bench.py --workload c4 --steps 3 --warmup 1 --c4-full-parity > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit 5
echo done
