#!/bin/bash
# A/B of the asm G blocks (leaf 51 vs 50, piece 14 vs 6) + their parity tests.
set -o pipefail
OUT=${1:-gpurun_out/r02_ga}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_hash.py tests/test_gpu_stream.py -m gpu -k "variant" -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
if [ -z "$NO_UBENCH" ]; then timeout -k 10 200 ./tools/ubench_compress 2000 > $OUT/ubench_compress.txt 2>&1 || exit 2; fi
for w in c2 c3 c5; do
  timeout -k 10 300 python -u tools/ab_leaf.py --product --workload $w --variants ${LEAF_VARIANTS:-50,51} --rounds 5 --reps 3 > $OUT/ab_$w.txt 2>&1 || exit 3
done
timeout -k 10 300 python -u tools/ab_piece.py --variants ${PIECE_VARIANTS:-6,14} --rounds 4 > $OUT/ab_piece.txt 2>&1 || exit 4
echo done
