#!/bin/bash
# round 4, second GPU call: the whole GPU suite and smoke, the job end to end
# (job_bench: with and without bulk identify), and the C2 / C3 / C5 / C4 lines
# (C2 with the driver's defaults). Each GPU step has its own limit; the first
# failure ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04b}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
echo "gpu tests ok"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 2
timeout -k 10 300 tests/cpp/build/job_bench 100000 > $OUT/job_bench.json 2> $OUT/job_bench.err || exit 3
echo "job bench ok"
timeout -k 10 400 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 4
for w in c3 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || exit 5
done
timeout -k 10 600 python -u bench.py --workload c4 --steps 3 --warmup 1 --c4-full-parity > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit 6
echo done
