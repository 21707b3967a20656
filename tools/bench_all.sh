#!/bin/bash
# All four bench lines (C2 headline, C3/C4/C5) with CPU baselines, one GPU.
# usage: tools/bench_all.sh OUTDIR
set -e
OUT=${1:-gpurun_out/bench}
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $OUT/bench_c2.log 2>&1
timeout -k 10 300 python -u bench.py --workload c3 --steps 5 --warmup 2 > $OUT/bench_c3.log 2>&1
timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 2 > $OUT/bench_c5.log 2>&1
timeout -k 10 400 python -u bench.py --workload c4 --steps 2 --warmup 1 > $OUT/bench_c4.log 2>&1
