#!/bin/bash
# round 4: the quad-lane finish kernel (k_finish_q): the whole GPU suite, then
# rocprofv3 kernel stats of the C2 and C5 lines with it and with the lane
# kernel (SDCAS_FINISH=lane); then the quad-slot small kernel (tools/r04_p.sh)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r04o}
R=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
echo "gpu tests ok"
for fin in quad lane; do
  for w in c2 c5; do
    (cd /tmp && SDCAS_FINISH=$fin timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_${w}_$fin -o $w \
       --output-format csv -- python3 $R/bench.py --workload $w --steps 20 --warmup 2 --no-cpu-baseline --no-e2e \
       > $R/$OUT/prof_${w}_$fin.json 2> $R/$OUT/prof_${w}_$fin.err) || exit 2
  done
done
bash tools/r04_p.sh $OUT/p || exit 3
echo done
