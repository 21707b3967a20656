#!/bin/bash
# Round-2 measurement pass on one MI355X (run through gpurun from the repo
# root): headline bench (C2 with e2e + reference-faithful CPU leg), piece
# kernel A/B (C4), C3 / C5 bench lines. Every GPU step has its own time limit;
# the first failure ends the script.
set -o pipefail
OUT=${1:-gpurun_out/r02}
mkdir -p $OUT
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 1
timeout -k 10 300 python -u tools/ab_piece.py --gib 16 --rounds 4 --reps 2 > $OUT/ab_piece.txt 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 3 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit 3
timeout -k 10 300 python -u bench.py --workload c3 --steps 10 --warmup 3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit 4
echo done
