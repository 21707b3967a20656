#!/bin/bash
# round 4: the hash combine as the default (dedup and multi-process GPU tests),
# then the C5 sort / clock probe (tools/r04_j.sh)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04k}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dist_dedup.py tests/test_gpu_multiproc.py -m gpu -v --timeout 300 \
  --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
bash tools/r04_j.sh $OUT || exit 2
echo done
