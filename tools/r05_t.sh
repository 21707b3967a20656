#!/bin/bash
# round 5 (t): the GPU suite, smoke and the C2 line at HEAD (huge-page
# staging by default), then the job end to end
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05t}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
echo "gpu tests ok"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 3
echo "c2 ok"
timeout -k 10 300 tests/cpp/build/job_bench 100000 > $OUT/job_bench.json 2> $OUT/job_bench.err || exit 4
echo done
