#!/bin/bash
# round 5 (p): the world-of-one apply taking a key's first ordinal from its
# first file's index when the ordinals are contiguous (default) against
# reading it (SDCAS_CONTIG=0): the dedup tests, same-process A/B, kernel times
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05p}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dist_dedup.py \
  tests/test_gpu_corpora.py > $OUT/pytest_dedup.txt 2>&1 || exit 1
for w in c5 c3; do
  timeout -k 10 300 python -u tools/dedup_probe.py --workload $w --reps 20 --ab "SDCAS_CONTIG=0,SDCAS_CONTIG=1" \
    > $OUT/probe_${w}_contig.json 2> $OUT/probe_${w}_contig.err || exit 1
done
for c in 0 1; do
  SDCAS_CONTIG=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5_c$c -o run -- \
    python -u tools/dedup_probe.py --workload c5 --reps 10 > $OUT/prof_c5_c$c.log 2>&1 || exit 1
done
find $OUT -name '*kernel_trace.csv' -delete
echo done
