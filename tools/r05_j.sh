#!/bin/bash
# round 5 (j): the GPU suite and smoke at HEAD, then the job's row writes
# batched (set_cas_ids_and_connect: 64 rows per UPDATE ... FROM (VALUES ...))
# against one statement per row (SDCORE_LINKS=each), alternating processes
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05j}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
  > $OUT/pytest_gpu.txt 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || exit 1
for rep in 1 2 3; do
  for mode in many each; do
    SDCORE_LINKS=$mode SDCORE_TRACE_JOB=1 timeout -k 10 300 tests/cpp/build/job_bench 100000 20000 \
      > $OUT/job_${mode}_$rep.json 2> $OUT/job_${mode}_$rep.err || exit 1
    echo "job $mode rep $rep ok"
  done
done
echo done
