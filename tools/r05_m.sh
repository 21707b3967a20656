#!/bin/bash
# round 5 (m): staging slot size sweep (SDCAS_STAGING_MB) for the job's
# 10 000-file calls and the C2 bench's 200 000-file e2e call, alternating
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05m}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for mb in 256 128 96 64; do
    SDCAS_STAGING_MB=$mb SDCAS_TRACE_IO=1 SDCORE_TRACE_JOB=1 timeout -k 10 300 tests/cpp/build/job_bench 100000 20000 \
      > $OUT/job_s${mb}_$rep.json 2> $OUT/job_s${mb}_$rep.err || exit 1
    echo "job staging $mb rep $rep ok"
  done
done
for mb in 256 128 96 64; do
  SDCAS_STAGING_MB=$mb timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline \
    > $OUT/bench_c2_s$mb.json 2> $OUT/bench_c2_s$mb.err || exit 2
  echo "bench staging $mb ok"
done
echo done
