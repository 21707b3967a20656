#!/bin/bash
# round 4, first GPU call: the new launcher, stream and node tests, the C4
# and C2 lines, the dedup's PMC passes
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_stream.py tests/test_gpu_node.py "tests/test_gpu_multiproc.py::test_bench_two_ranks" \
  -m gpu > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c4 --steps 5 --warmup 2 > $O/c4.json 2> $O/c4.err &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-e2e > $O/c2.json 2> $O/c2.err &&
bash tools/pmc_dedup.sh $O/pmc_dedup_c5 c5 10 > $O/pmc_dedup_c5.log 2>&1 &&
bash tools/pmc_dedup.sh $O/pmc_dedup_c3 c3 10 > $O/pmc_dedup_c3.log 2>&1
