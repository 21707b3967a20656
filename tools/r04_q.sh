#!/bin/bash
# round 4, final refresh at HEAD: the whole GPU suite and smoke, the C2 / C3 /
# C5 lines, then tools/r04_n.sh (the job, the C4 line, rocprofv3 kernel stats
# of the four lines)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04q}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
echo "gpu tests ok"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 3
for w in c3 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || exit 4
done
echo "lines ok"
bash tools/r04_n.sh $OUT || exit 5
echo done
