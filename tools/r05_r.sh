#!/bin/bash
# round 5 (r): the path call's host side: the last slot of a call uploaded in
# parts while it is read (SDCAS_LAST_PARTS=1) and the staging slots on
# transparent huge pages (SDCAS_STAGING_THP=1), each against the default,
# alternating processes: the job (10 000-file calls) with the library's
# per-call trace, and the C2 bench's e2e legs (one 200 000-file call)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05r}
mkdir -p $OUT
export TMPDIR=/tmp
SDCAS_LAST_PARTS=1 SDCAS_STAGING_THP=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  -m gpu tests/test_gpu_hash.py tests/test_gpu_stream.py > $OUT/pytest_knobs.txt 2>&1 || exit 3
for rep in 1 2; do
  for cfg in 0,0 1,0 0,1 1,1; do
    lp=${cfg%,*}; thp=${cfg#*,}
    SDCAS_LAST_PARTS=$lp SDCAS_STAGING_THP=$thp SDCAS_TRACE_IO=1 SDCORE_TRACE_JOB=1 timeout -k 10 300 \
      tests/cpp/build/job_bench 100000 20000 > $OUT/job_lp${lp}_thp${thp}_$rep.json 2> $OUT/job_lp${lp}_thp${thp}_$rep.err || exit 1
    echo "job lp=$lp thp=$thp rep $rep ok"
  done
done
for cfg in 0,0 1,0 0,1; do
  lp=${cfg%,*}; thp=${cfg#*,}
  SDCAS_LAST_PARTS=$lp SDCAS_STAGING_THP=$thp timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline \
    --sustain-s 0 > $OUT/bench_c2_lp${lp}_thp${thp}.json 2> $OUT/bench_c2_lp${lp}_thp${thp}.err || exit 2
  echo "bench lp=$lp thp=$thp ok"
done
echo done
