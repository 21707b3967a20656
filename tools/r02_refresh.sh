#!/bin/bash
# Round-2 refresh on one MI355X (through gpurun, from the repo root): the GPU
# tests, the four bench lines, rocprofv3 kernel stats of the C2 / C4 benches,
# and the HBM-traffic PMC passes of the default leaf kernel. Each GPU step has
# its own time limit; the first failure ends the script.
set -o pipefail
OUT=${1:-gpurun_out/r02_refresh}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 2
for w in c3 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || exit 3
done
timeout -k 10 400 python -u bench.py --workload c4 --steps 3 --warmup 1 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit 4
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_c2 -o c2 --output-format csv -- \
   python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $R/$OUT/prof_c2.log 2>&1) || exit 5
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_c4 -o c4 --output-format csv -- \
   python $R/bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $R/$OUT/prof_c4.log 2>&1) || exit 6
bash tools/pmc_traffic.sh $OUT/pmc_c2 > $OUT/pmc_c2.log 2>&1 || exit 7
bash tools/pmc_traffic.sh $OUT/pmc_c4 -- python $R/bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline \
  > $OUT/pmc_c4.log 2>&1 || exit 8
VARIANT=51 bash tools/pmc_sq_workloads.sh $OUT/sqw > $OUT/sqw.log 2>&1 || exit 9
echo done
