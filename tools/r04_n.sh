#!/bin/bash
# round 4, final refresh at HEAD: the job end to end, the C4 line (every
# file against the oracle), then rocprofv3 kernel stats and traces of the four
# bench lines (each line's own JSON beside its trace)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04n}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 tests/cpp/build/job_bench 100000 > $OUT/job_bench.json 2> $OUT/job_bench.err || exit 1
echo "job ok"
timeout -k 10 600 python3 -u bench.py --workload c4 --steps 3 --warmup 1 --c4-full-parity > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit 2
echo "c4 ok"
for w in c2 c3 c5; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_$w -o $w --output-format csv -- \
     python3 $R/bench.py --workload $w --steps 20 --warmup 2 --no-cpu-baseline --no-e2e > $R/$OUT/prof_$w.json 2> $R/$OUT/prof_$w.err) || exit 3
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_c4 -o c4 --output-format csv -- \
   python3 $R/bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $R/$OUT/prof_c4.json 2> $R/$OUT/prof_c4.err) || exit 4
echo done
