#!/bin/bash
# round 5 (d): the job's read side with files opened / stat'ed relative to a
# cached directory descriptor (SDCAS_DIRFD / SDCORE_DIRFD, default on)
# against full paths, alternating processes; phase traces of one run each
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05d}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for mode in 1 0; do
    SDCAS_DIRFD=$mode SDCORE_DIRFD=$mode SDCORE_TRACE_JOB=1 timeout -k 10 300 tests/cpp/build/job_bench 100000 20000 \
      > $OUT/job_dirfd${mode}_$rep.json 2> $OUT/job_dirfd${mode}_$rep.err || exit 1
    echo "job dirfd=$mode rep $rep ok"
  done
done
for mode in 1 0; do
  SDCAS_DIRFD=$mode timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline \
    > $OUT/bench_c2_dirfd$mode.json 2> $OUT/bench_c2_dirfd$mode.err || exit 2
done
echo done
