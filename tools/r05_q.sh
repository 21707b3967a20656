#!/bin/bash
# round 5 (q): the job's metadata calls on a timeline — kernels and memory
# copies of tests/cpp/build/job_bench (30 000 files) under rocprofv3, with the
# library's per-call phase trace beside it
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05q}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
(cd /tmp && SDCAS_TRACE_IO=1 SDCORE_TRACE_JOB=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace \
   --output-format csv -d $R/$OUT/trace -o job -- $R/tests/cpp/build/job_bench 30000 5000 \
   > $R/$OUT/job.json 2> $R/$OUT/job.err) || exit 1
echo done
