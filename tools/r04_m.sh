#!/bin/bash
# round 4: the slot plan's own kernels (k_plan_sums / k_plan_scan /
# k_plan_write instead of rocPRIM's scan + k_tile_first): the whole GPU suite
# and smoke, then the shape-sort A/B again (tools/r04_l.sh) and the C5 / C3 / C2
# lines
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04m}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
echo "gpu tests ok"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 2
bash tools/r04_l.sh $OUT || exit 3
for w in c5 c3; do
  timeout -k 10 300 python3 -u bench.py --workload $w --no-e2e > $OUT/bench_$w.json 2> $OUT/bench_$w.err || exit 4
done
timeout -k 10 400 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 5
echo done
