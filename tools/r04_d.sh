#!/bin/bash
# round 4, fourth GPU call: the compact dedup table with existing Objects too
# (GPU dedup tests + same-process A/B against the kv table), its PMC passes
# (C5, C3), the job with batched Object inserts and ordered pub_ids, and the
# C3 / C5 lines.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04d}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_dist_dedup.py tests/test_gpu_corpora.py tests/test_gpu_node.py \
  tests/test_host_cpp.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_dedup.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
echo "dedup tests ok"
timeout -k 10 200 python -u tools/dedup_probe.py --workload c5 --reps 20 --tables kv,idx > $OUT/ab_dedup_c5.json 2> $OUT/ab_dedup_c5.err || exit 2
timeout -k 10 200 python -u tools/dedup_probe.py --workload c5 --reps 20 --tables kv,idx --existing 500000 > $OUT/ab_dedup_c5_ex.json 2> $OUT/ab_dedup_c5_ex.err || exit 2
timeout -k 10 200 python -u tools/dedup_probe.py --workload c3 --reps 20 --tables kv,idx > $OUT/ab_dedup_c3.json 2> $OUT/ab_dedup_c3.err || exit 2
bash tools/pmc_dedup.sh $OUT/pmc_dedup_c5 c5 10 > $OUT/pmc_dedup_c5.log 2>&1 || exit 3
bash tools/pmc_dedup.sh $OUT/pmc_dedup_c3 c3 10 > $OUT/pmc_dedup_c3.log 2>&1 || exit 3
SDCORE_TRACE_JOB=1 timeout -k 10 300 tests/cpp/build/job_bench 100000 > $OUT/job_bench.json 2> $OUT/job_bench.err || exit 4
echo "job bench ok"
for w in c3 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || exit 5
done
echo done
