set -e
mkdir -p gpurun_out/r01
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r01/bench_c2.log 2>&1
for w in c3 c5; do timeout -k 10 300 python -u bench.py --workload $w --steps 5 --warmup 2 > gpurun_out/r01/bench_$w.log 2>&1; done
timeout -k 10 400 python -u bench.py --workload c4 --steps 2 --warmup 1 > gpurun_out/r01/bench_c4.log 2>&1
for w in c2 c3 c5; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r01/prof_$w -o $w --output-format csv -- python $R/bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/r01/prof_$w.log 2>&1)
done
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r01/prof_c4 -o c4 --output-format csv -- python $R/bench.py --workload c4 --steps 1 --warmup 1 > $R/gpurun_out/r01/prof_c4.log 2>&1)
