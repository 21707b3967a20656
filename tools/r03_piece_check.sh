#!/bin/bash
# Round 3: the full-chunk piece kernel (17) against the previous default (15):
# the piece tests, a same-process A/B (product library), the C4 bench line.
set -o pipefail
O=${1:-gpurun_out/r03_piece}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_hash.py -x -q --timeout 200 --timeout-method thread -k "piece or diagnostic or big" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab_piece.py --variants 15,17 --rounds 7 --reps 3 > $O/ab_piece_15_17.txt 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || exit 3
echo done
