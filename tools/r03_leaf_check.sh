#!/bin/bash
# Round 3: leaf 67 (table-driven tail masks) against 52, and the piece kernel
# 17 against 15, in the product library: GPU tests, same-process A/Bs, the C2
# bench line at the driver's defaults.
set -o pipefail
O=${1:-gpurun_out/r03_leaf}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 400 python -u tools/ab_leaf.py --product --variants 52,67 --rounds 7 --reps 3 > $O/ab_leaf_52_67_c2.txt 2>&1 || exit 3
timeout -k 10 400 python -u tools/ab_leaf.py --product --workload c5 --files 6250000 --variants 52,67 --rounds 5 --reps 3 > $O/ab_leaf_52_67_c5.txt 2>&1 || exit 4
timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit 5
echo done
