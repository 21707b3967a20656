#!/bin/bash
# round 5, final refresh at HEAD (b): rocprofv3 kernel stats of the four bench
# lines, the dedup's PMC passes (C3, C5), the job end to end
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05fb}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
for w in c2 c3 c5; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_$w -o $w --output-format csv -- \
     python3 $R/bench.py --workload $w --steps 20 --warmup 2 --no-cpu-baseline --no-e2e --sustain-s 0 \
     > $R/$OUT/prof_$w.json 2> $R/$OUT/prof_$w.err) || exit 1
  echo "prof $w ok"
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_c4 -o c4 --output-format csv -- \
   python3 $R/bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --sustain-s 0 \
   > $R/$OUT/prof_c4.json 2> $R/$OUT/prof_c4.err) || exit 2
echo "prof c4 ok"
find $OUT -name '*kernel_trace.csv' -delete
for w in c3 c5; do
  bash tools/pmc_dedup.sh $OUT/pmc_dedup_$w $w 10 > $OUT/pmc_dedup_$w.log 2>&1 || exit 3
  echo "pmc dedup $w ok"
done
timeout -k 10 300 tests/cpp/build/job_bench 100000 > $OUT/job_bench.json 2> $OUT/job_bench.err || exit 4
echo done
