#!/bin/bash
# round 5 (o): the job's metadata and group-by: the stat pass beside the
# reads at the indexer's sizes (SDCORE_SPEC_STAT=1) and the group-by on a
# sibling context (SDCORE_DEDUP_CTX=own) against round 5's stat-first, one
# context (0 / shared), alternating processes; the host mirror's GPU test
# first (the speculative metadata equal to the plain one)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05o}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_host_cpp.py \
  > $OUT/pytest_host.txt 2>&1 || exit 1
for rep in 1 2 3; do
  for cfg in 1,own 0,shared 0,own 1,shared; do
    spec=${cfg%,*}; ctx=${cfg#*,}
    SDCORE_SPEC_STAT=$spec SDCORE_DEDUP_CTX=$ctx SDCORE_TRACE_JOB=1 timeout -k 10 300 tests/cpp/build/job_bench 100000 20000 \
      > $OUT/job_s${spec}_${ctx}_$rep.json 2> $OUT/job_s${spec}_${ctx}_$rep.err || exit 2
    echo "job spec=$spec ctx=$ctx rep $rep ok"
  done
done
echo done
