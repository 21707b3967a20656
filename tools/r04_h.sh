#!/bin/bash
# round 4: the driver's plain N = 8 launch rehearsed on the one GPU (gloo
# standing in for RCCL: RCCL refuses two ranks on one device): C2 and C5 with
# 100 K files per rank, each line's per-rank oracle samples and (C5) every
# rank's links against the chunked oracle over the whole corpus
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04h}
mkdir -p $OUT
export TMPDIR=/tmp
for w in c2 c5; do
  SDCAS_BENCH_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 400 python3 -u bench.py --gpus 8 --workload $w --files 100000 \
    --steps 3 --warmup 1 > $OUT/n8_gloo_$w.json 2> $OUT/n8_gloo_$w.err || exit 1
done
echo done
