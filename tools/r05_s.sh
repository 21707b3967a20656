#!/bin/bash
# round 5 (s): confirmation of (r) — staging on transparent huge pages
# (SDCAS_STAGING_THP=1) and the last slot uploaded in parts
# (SDCAS_LAST_PARTS=1) — the C2 e2e legs three times each, alternating, and
# the job twice per setting; plus big-file checksums from the page cache
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05s}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for cfg in 0,0 0,1 1,1; do
    lp=${cfg%,*}; thp=${cfg#*,}
    SDCAS_LAST_PARTS=$lp SDCAS_STAGING_THP=$thp timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline \
      --sustain-s 0 > $OUT/bench_c2_lp${lp}_thp${thp}_$rep.json 2> $OUT/bench_c2_lp${lp}_thp${thp}_$rep.err || exit 2
    echo "bench lp=$lp thp=$thp rep $rep ok"
  done
done
for rep in 1 2; do
  for cfg in 0,0 0,1 1,1; do
    lp=${cfg%,*}; thp=${cfg#*,}
    SDCAS_LAST_PARTS=$lp SDCAS_STAGING_THP=$thp SDCORE_TRACE_JOB=1 timeout -k 10 300 \
      tests/cpp/build/job_bench 100000 20000 > $OUT/job_lp${lp}_thp${thp}_$rep.json 2> $OUT/job_lp${lp}_thp${thp}_$rep.err || exit 1
    echo "job lp=$lp thp=$thp rep $rep ok"
  done
done
for thp in 0 1; do
  SDCAS_STAGING_THP=$thp timeout -k 10 400 python -u tools/e2e_big.py --gib 4 > $OUT/e2e_big_thp$thp.json \
    2> $OUT/e2e_big_thp$thp.err || exit 3
  echo "e2e_big thp=$thp ok"
done
echo done
