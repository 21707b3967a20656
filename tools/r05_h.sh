#!/bin/bash
# round 5 (h): the world-of-one dedup's table density: the compact u32 table
# and the 16-byte kv table at 2 and 1.25 slots per item, same process
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05h}
mkdir -p $OUT
export TMPDIR=/tmp
T=SDCAS_DEDUP_TABLE; L=SDCAS_DEDUP_LOAD
for w in c5 c3; do
  timeout -k 10 300 python -u tools/dedup_probe.py --workload $w --reps 20 \
    --ab "$T=idx+$L=2,$T=idx+$L=1.25,$T=kv+$L=2,$T=kv+$L=1.25" > $OUT/probe_${w}_load.json 2> $OUT/probe_${w}_load.err || exit 1
done
echo done
