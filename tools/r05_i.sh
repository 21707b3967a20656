#!/bin/bash
# round 5 (i): the world-of-one files insert with R files per thread
# (SDCAS_INSERT_R; the first run of this script A/B'd the apply's
# SDCAS_APPLY_R = 0,1,2,4,8 the same way: profiles/r05_ab_dedup_apply.json):
# parity over the local dedup tests, same-process A/B per call, kernel times
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05i2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dist_dedup.py \
  -k "local" > $OUT/pytest_local.txt 2>&1 || exit 1
for w in c5 c3; do
  timeout -k 10 300 python -u tools/dedup_probe.py --workload $w --reps 20 \
    --ab "SDCAS_INSERT_R=1,SDCAS_INSERT_R=2,SDCAS_INSERT_R=4" \
    > $OUT/probe_${w}_insert.json 2> $OUT/probe_${w}_insert.err || exit 1
done
for r in 1 4; do
  SDCAS_INSERT_R=$r timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5_r$r -o run -- \
    python -u tools/dedup_probe.py --workload c5 --reps 10 > $OUT/prof_c5_r$r.log 2>&1 || exit 1
done
find $OUT -name '*kernel_trace.csv' -delete
echo done
