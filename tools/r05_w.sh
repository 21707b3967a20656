#!/bin/bash
# round 5 (w): the bulk-identify leg's end-of-job work: SQLite's own WAL
# checkpoints during the job (SDCORE_BULK_CKPT=auto) and the cas_id index
# kept current instead of dropped and rebuilt (SDCORE_BULK_KEEP_INDEX=1),
# against the default, alternating processes
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/r05w}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for cfg in drop,0 drop,auto keep,0 keep,auto; do
    ix=${cfg%,*}; ck=${cfg#*,}
    ki=0; [ "$ix" = keep ] && ki=1
    SDCORE_BULK_KEEP_INDEX=$ki SDCORE_BULK_CKPT=$ck SDCORE_TRACE_JOB=1 timeout -k 10 300 \
      tests/cpp/build/job_bench 100000 20000 > $OUT/job_${ix}_${ck}_$rep.json 2> $OUT/job_${ix}_${ck}_$rep.err || exit 1
    echo "job $cfg rep $rep ok"
  done
done
echo done
