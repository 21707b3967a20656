#!/bin/bash
# round 5 (a): the dedup GPU tests, then same-process A/Bs of the dedup on
# C5 / C3 at world 1 (round 5's five launches against round 4's eight) and
# one rank's bucket stages at world 8 (the owner's resolve sized on the
# device against round 4's), then rocprofv3 kernel stats of the defaults
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05a}
mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_dist_dedup.py tests/test_gpu_corpora.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $OUT/pytest_dedup.log 2>&1 || exit 1
echo "dedup tests ok"
for w in c5 c3; do
  timeout -k 10 300 python -u tools/dedup_probe.py --workload $w --reps 20 --ab "SDCAS_DEDUP_TABLE=idx4,idx" \
    > $OUT/probe_${w}_w1.json 2> $OUT/probe_${w}_w1.err || exit 2
  timeout -k 10 300 python -u tools/dedup_probe.py --workload $w --reps 10 --world 8 --ab "SDCAS_RESOLVE=split,kv" \
    > $OUT/probe_${w}_w8.json 2> $OUT/probe_${w}_w8.err || exit 3
done
for w in c5 c3; do
  for W in 1 8; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_${w}_w$W -o prof --output-format csv -- \
      python3 -u tools/dedup_probe.py --workload $w --reps 10 --world $W > $OUT/prof_${w}_w$W.json \
      2> $OUT/prof_${w}_w$W.err || exit 4
    find $OUT/prof_${w}_w$W -type f ! -name "*kernel_stats.csv" -delete
  done
done
echo done
