set -o pipefail
O=gpurun_out/plan; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_hash.py > $O/pytest_hash.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/latency_probe.py --files 20000 --batches 1,10,100,300 --calls 200 spacedrive_amd/libsdcas.so "spacedrive_amd/libsdcas.so,SDCAS_PLAN_SMALL=0" > $O/probe.jsonl 2> $O/probe.err || exit 2
echo done
