#!/bin/bash
# round 5 (l): the job's read side against the staging slot size
# (SDCAS_STAGING_MB: 256 = the default, 64, 32), alternating processes, with
# the library's per-call phase trace; then the C2 bench's e2e legs at 256 / 64
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05l}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for mb in 256 64 32; do
    SDCAS_STAGING_MB=$mb SDCAS_TRACE_IO=1 SDCORE_TRACE_JOB=1 timeout -k 10 300 tests/cpp/build/job_bench 100000 20000 \
      > $OUT/job_s${mb}_$rep.json 2> $OUT/job_s${mb}_$rep.err || exit 1
    echo "job staging $mb rep $rep ok"
  done
done
for mb in 256 64; do
  SDCAS_STAGING_MB=$mb timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline \
    > $OUT/bench_c2_s$mb.json 2> $OUT/bench_c2_s$mb.err || exit 2
done
echo done
