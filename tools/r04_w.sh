#!/bin/bash
# round 4: the GPU suite and smoke on the tree as it stands (last check)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04w}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 3
echo done
