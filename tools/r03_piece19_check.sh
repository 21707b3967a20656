set -o pipefail
O=gpurun_out/p19
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stream.py > $O/pytest_stream.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab_piece.py --variants 17,19 --rounds 5 --reps 3 > $O/ab_17_19.txt 2>&1 || exit 2
SDCAS_PIECE_VARIANT=19 timeout -k 10 600 python -u bench.py --workload c4 --steps 3 --warmup 1 --c4-full-parity > $O/bench_c4_v19.json 2> $O/bench_c4_v19.err || exit 3
echo done
