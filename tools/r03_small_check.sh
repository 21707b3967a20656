#!/bin/bash
# Round 3: the small-batch leaf kernel (variant 71, 128-slot tiles) and the
# parts upload of single-slot calls: the GPU tests, per-call latency of
# sdcas_cas_ids with both (default) and without either (one library, contexts
# alternating per call), and the C2 bench line (the 1 MiB-tile path).
set -o pipefail
O=${1:-gpurun_out/r03_small}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
L=spacedrive_amd/libsdcas.so
timeout -k 10 400 python -u tools/latency_probe.py --files 20000 --batches 1,10,100,300,1000,10000 --calls 200 \
  $L "$L,SDCAS_SMALL_SLOTS=0" "$L,SDCAS_SMALL_SLOTS=0,SDCAS_UPLOAD_PARTS=0" > $O/probe.jsonl 2> $O/probe.err || exit 3
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit 4
echo done
