#!/bin/bash
# round 5 (k): the owner's resolve in a u32 table of claiming record indices
# (default) against round 5's 16-byte entries (SDCAS_RESOLVE=kv): the dedup,
# node and two-process tests, one rank's stages at world 8 (same process),
# and the kernels of each
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05k}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dist_dedup.py \
  tests/test_gpu_node.py tests/test_gpu_multiproc.py tests/test_gpu_corpora.py > $OUT/pytest_dedup.txt 2>&1 || exit 1
for w in c5 c3; do
  timeout -k 10 300 python -u tools/dedup_probe.py --workload $w --world 8 --reps 20 \
    --ab "SDCAS_RESOLVE=kv,SDCAS_RESOLVE=idx" > $OUT/probe_${w}_w8_resolve.json 2> $OUT/probe_${w}_w8_resolve.err || exit 1
done
for r in kv idx; do
  SDCAS_RESOLVE=$r timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5_w8_$r -o run -- \
    python -u tools/dedup_probe.py --workload c5 --world 8 --reps 10 > $OUT/prof_c5_w8_$r.log 2>&1 || exit 1
done
find $OUT -name '*kernel_trace.csv' -delete
echo done
