set -o pipefail
mkdir -p gpurun_out/s16
true
for w in c5; do
SDCAS_BENCH_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 8 --workload $w --files $([ $w = c5 ] && echo 3000000 || echo 500000) --steps 2 --warmup 1 \
  > gpurun_out/s16/n8_gloo_$w.json 2> gpurun_out/s16/n8_gloo_$w.err || exit 2
done
echo done
