#!/bin/bash
# round 5 (n): the N = 8 launch rehearsal (gloo on the one GPU) at the final
# HEAD — the owner's resolve in its compact form and the batched applies — for
# C5, C3 and the driver's default C2; every rank's links against the oracle
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05n}
mkdir -p $OUT
export TMPDIR=/tmp
for w in c5 c3 c2; do
  SDCAS_BENCH_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 400 python3 -u bench.py --gpus 8 --workload $w --files 100000 \
    --steps 3 --warmup 1 --sustain-s 0 > $OUT/n8_gloo_$w.json 2> $OUT/n8_gloo_$w.err || exit 1
  echo "$w ok"
done
echo done
