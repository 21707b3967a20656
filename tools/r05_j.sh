#!/bin/bash
# round 5 (j): the GPU suite and smoke at HEAD, then the job's row writes
# batched (set_cas_ids_and_connect: 64 rows per UPDATE ... FROM (VALUES ...))
# against one statement per row (SDCORE_LINKS=each), alternating processes;
# the world-8 stages with the bucket apply at 4 files per thread against
# round 5's grid-stride apply (SDCAS_APPLY_R=0), same process
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
for w in c5 c3; do
  timeout -k 10 300 python -u tools/dedup_probe.py --workload $w --world 8 --reps 20 \
    --ab "SDCAS_APPLY_R=0,SDCAS_APPLY_R=4" > $OUT/probe_${w}_w8_apply.json 2> $OUT/probe_${w}_w8_apply.err || exit 1
done
echo done
