#!/bin/bash
# Per-call latency of sdcas_cas_ids at the C ABI (tools/latency_probe.py):
# the in-tree library against tools/ab_libs/*.so side by side if present,
# then a rocprofv3 kernel / copy / HIP-API trace of batch-1 and batch-100
# calls (no counters). Each GPU step has its own time limit.
set -o pipefail
OUT=${1:-gpurun_out/latency}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
shopt -s nullglob
LIBS=(spacedrive_amd/libsdcas.so tools/ab_libs/*.so)
timeout -k 10 300 python -u tools/latency_probe.py --files 20000 --batches 1,10,100,1000,10000 --calls 200 \
  "${LIBS[@]}" > $OUT/probe.jsonl 2> $OUT/probe.err || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv \
   -d $R/$OUT/trace -o t -- python -u $R/tools/latency_probe.py --files 3000 --batches 1,100 --calls 20 \
   > $R/$OUT/trace.log 2>&1) || exit 2
echo done
