#!/bin/bash
# round 4: the quad-slot small-batch kernel (leaf variant 73): the hash GPU
# tests with it forced for every small batch, then per-call latency of
# sdcas_cas_ids with the default small kernel (71) and with 73, contexts of one
# library alternating per call
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04p}
mkdir -p $OUT
export TMPDIR=/tmp
SDCAS_SMALL_VARIANT=73 timeout -k 10 600 python -u -m pytest tests/test_gpu_hash.py tests/test_gpu_corpora.py \
  tests/test_gpu_stream.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_small73.log 2>&1 || exit 1
echo "tests with 73 ok"
L=spacedrive_amd/libsdcas.so
timeout -k 10 400 python3 -u tools/latency_probe.py --batches 1,10,100,300 --calls 200 $L $L,SDCAS_SMALL_VARIANT=73 \
  > $OUT/latency.json 2> $OUT/latency.err || exit 2
echo done
