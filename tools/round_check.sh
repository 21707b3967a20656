#!/bin/bash
# GPU tests + smoke + bench lines + rocprof stats + PMC traffic, one call.
# usage: tools/round_check.sh OUTDIR
set -e
OUT=${1:-gpurun_out/check}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "gpu tests ok"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
echo "smoke ok"
tools/refresh_profiles.sh $OUT
echo "profiles ok"
