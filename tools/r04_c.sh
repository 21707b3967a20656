#!/bin/bash
# round 4, third GPU call: the dedup's compact table (GPU dedup tests, then a
# same-process A/B against the kv table on C5 and C3), the job with the
# read-ahead connection and deferred checkpoints, and an A/B of C5's message
# alignment in HBM (128 vs 16 bytes, alternating processes on one box).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04c}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_dist_dedup.py tests/test_gpu_corpora.py tests/test_gpu_node.py -m gpu -v \
  --timeout 300 --timeout-method thread > $OUT/pytest_dedup.log 2>&1 || exit 1
echo "dedup tests ok"
for w in c5 c3; do
  timeout -k 10 200 python -u tools/dedup_probe.py --workload $w --reps 20 --tables kv,idx > $OUT/ab_dedup_$w.json 2> $OUT/ab_dedup_$w.err || exit 2
done
timeout -k 10 300 tests/cpp/build/job_bench 100000 > $OUT/job_bench.json 2> $OUT/job_bench.err || exit 3
echo "job bench ok"
for rep in 1 2; do
  for al in 128 16; do
    timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline --msg-align $al \
      > $OUT/c5_align${al}_$rep.json 2> $OUT/c5_align${al}_$rep.err || exit 4
  done
done
echo done
