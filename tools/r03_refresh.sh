#!/bin/bash
# Round-3 refresh on one MI355X (through gpurun, from the repo root), in two
# parts so each fits one call:
#   part a: the GPU tests, smoke, the four bench lines (C2 with the driver's
#           defaults), an N = 2 rehearsal of the driver's torchrun launch (gloo,
#           two ranks on the one GPU);
#   part b: rocprofv3 kernel stats of the C2 / C3 / C4 / C5 benches, the
#           HBM-traffic PMC passes of the default leaf (C2) and piece (C4)
#           kernels and the SQ passes of the leaf kernel per workload.
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
PART=${1:?part a or b}
OUT=${2:-gpurun_out/r03_refresh}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$PART" = a ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
  echo "gpu tests ok"
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 2
  timeout -k 10 400 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 3
  for w in c3 c5; do
    timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || exit 4
  done
  timeout -k 10 600 python -u bench.py --workload c4 --steps 3 --warmup 1 --c4-full-parity > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit 5
  echo "bench ok"
  SDCAS_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 \
    > $OUT/n2_gloo_c2.json 2> $OUT/n2_gloo_c2.err || exit 6
  echo done
else
  for w in c2 c3 c5; do
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_$w -o $w --output-format csv -- \
       python $R/bench.py --workload $w --steps 20 --warmup 2 --no-cpu-baseline --no-e2e > $R/$OUT/prof_$w.log 2>&1) || exit 7
  done
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_c4 -o c4 --output-format csv -- \
     python $R/bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $R/$OUT/prof_c4.log 2>&1) || exit 8
  echo "rocprof ok"
  bash tools/pmc_traffic.sh $OUT/pmc_c2 > $OUT/pmc_c2.log 2>&1 || exit 9
  bash tools/pmc_traffic.sh $OUT/pmc_c4 -- python $R/bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline \
    > $OUT/pmc_c4.log 2>&1 || exit 10
  VARIANT=67 bash tools/pmc_sq_workloads.sh $OUT/sqw > $OUT/sqw.log 2>&1 || exit 11
  echo done
fi
