#!/bin/bash
# round 5 (y): the bucket combine's slot pass with 4 files per thread
# (SDCAS_SLOT_R=4) against one: the bucket tests, one rank's stages at world 8
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05y}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dist_dedup.py \
  -k "bucket" > $OUT/pytest_bucket.txt 2>&1 || exit 1
for w in c5 c3; do
  timeout -k 10 300 python -u tools/dedup_probe.py --workload $w --world 8 --reps 20 \
    --ab "SDCAS_SLOT_R=1,SDCAS_SLOT_R=4" > $OUT/probe_${w}_w8_slot.json 2> $OUT/probe_${w}_w8_slot.err || exit 1
done
echo done
