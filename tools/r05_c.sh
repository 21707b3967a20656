#!/bin/bash
# round 5 (c): the bound step stream (sdcas_dev_bind_stream): the two-stream
# tests, C2 / C5 lines bound and unbound, and the C5 step's kernel trace both
# ways (the gap after the hash's last kernel)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05c}
mkdir -p $OUT
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_multiproc.py -k two_streams -v --timeout 120 \
  --timeout-method thread > $OUT/pytest_streams.log 2>&1 || exit 1
echo "stream tests ok"
for w in c5 c2; do
  for b in "" "--no-bind-stream"; do
    tag=${b:+unbound}; tag=${tag:-bound}
    timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-e2e $b \
      > $OUT/bench_${w}_$tag.json 2> $OUT/bench_${w}_$tag.err || exit 2
  done
done
for b in "" "--no-bind-stream"; do
  tag=${b:+unbound}; tag=${tag:-bound}
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/trace_$tag -o c5 --output-format csv \
    -- python3 -u $R/bench.py --workload c5 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e $b \
    > $R/$OUT/trace_$tag.json 2> $R/$OUT/trace_$tag.err) || exit 3
  f=$(find $OUT/trace_$tag -name "*kernel_trace.csv" | head -1)
  python3 tools/kernel_gaps.py $f --after k_finish_q > $OUT/gaps_hash_$tag.json
  python3 tools/kernel_gaps.py $f --after k_solo_apply_idx > $OUT/gaps_dedup_$tag.json
  find $OUT/trace_$tag -type f ! -name "*kernel_trace.csv" -delete
done
echo done
