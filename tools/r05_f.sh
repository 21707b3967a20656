#!/bin/bash
# round 5 (f): the driver's plain N = 8 launch rehearsed on the one GPU (gloo
# standing in for RCCL) with round 5's C5 shares (bench.c5_share: each rank's
# 100 K files an even sample of the 50 M corpus, so the Zipf head's
# duplicates cross ranks), every rank's links against the chunked oracle;
# then the GPU suite and smoke at HEAD
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05f}
mkdir -p $OUT
export TMPDIR=/tmp
for w in c5 c3; do
  SDCAS_BENCH_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 400 python3 -u bench.py --gpus 8 --workload $w --files 100000 \
    --steps 3 --warmup 1 --sustain-s 0 > $OUT/n8_gloo_$w.json 2> $OUT/n8_gloo_$w.err || exit 1
done
echo "rehearsal ok"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 3
echo done
