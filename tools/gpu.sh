#!/bin/bash
# One parameterised GPU session (replaces the rounds' one-off r0x_*.sh
# scripts): each step runs under its own time limit, output under OUT, and the
# session stops at the first failing step (no GPU work after a fault, abort or
# time limit).
#
# usage: tools/gpu.sh OUT STEP [STEP ...]
#   tests[=EXPR]          pytest -m gpu (EXPR: a -k expression, '~' for ' '), OUT/pytest_gpu[_EXPR].log
#   smoke                 __graft_entry__.smoke()
#   bench=W[:STEPS:WARM]  bench.py --workload W (c2 c3 c4 c5), OUT/bench_W.json
#   stats=W               rocprofv3 --kernel-trace --stats of a bench.py W run (20 steps, no baselines), OUT/stats_W/
#   n8=W                  bench.py --gpus 8 --workload W at 100 000 files per rank, gloo on the one GPU (the driver's
#                         N = 8 launch rehearsed; every rank's links against the oracle), OUT/n8_gloo_W.json
#   dedupfull=W[:ARGS]    tools/dedup_full.py --workload W (ARGS: extra flags, '~' for ' '), OUT/dedup_full_W_N.json
#   pmcdedup=W[:ARGS]     tools/pmc_dedup.sh over tools/dedup_full.py or dedup_probe.py (ARGS: 'full' or probe flags)
#   probe=ARGS            tools/dedup_probe.py ARGS ('~' for ' '), OUT/probe_N.json
#   jobbench[=ARGS]       tests/cpp/build/job_bench ARGS ('~' for ' '; default 100000 files), OUT/job_bench.json
#   trace=PY[~ARGS]       rocprofv3 --kernel-trace --stats -- python3 PY ARGS ('~' for ' '), OUT/trace_N/
#   cmd=TEXT              any command ('~' for ' '), OUT/cmd_N.log, 600 s
set -o pipefail
cd "$(dirname "$0")/.."
OUT=$1
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$(pwd)
n=0
step() {
  local s=$1 name=${1%%=*} arg=${1#*=}
  [ "$arg" = "$1" ] && arg=""
  n=$((n + 1))
  echo "== step $n: $s ($(date +%T))"
  case $name in
    tests)
      local k=() tag=""
      [ -n "$arg" ] && k=(-k "${arg//\~/ }") && tag=_$(echo "$arg" | tr -c 'a-zA-Z0-9' '_' | cut -c1-40)
      timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "${k[@]}" \
        > "$OUT/pytest_gpu$tag.log" 2>&1
      local rc=$?; tail -2 "$OUT/pytest_gpu$tag.log"; return $rc ;;
    smoke)
      timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 ;;
    bench)
      IFS=: read -r w st wu <<< "$arg"
      local extra=()
      [ -n "$st" ] && extra=(--steps "$st" --warmup "${wu:-3}")
      timeout -k 10 700 python -u bench.py --workload "$w" "${extra[@]}" > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
      local rc=$?; cut -c1-300 "$OUT/bench_$w.json"; return $rc ;;
    stats)
      local st=20
      [ "$arg" = c4 ] && st=3
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/$OUT/stats_$arg" -o "$arg" \
        --output-format csv -- python3 "$R/bench.py" --workload "$arg" --steps $st --warmup 1 --no-cpu-baseline \
        --no-e2e --sustain-s 0 > "$R/$OUT/stats_$arg.json" 2> "$R/$OUT/stats_$arg.err")
      local rc=$?; find "$OUT/stats_$arg" -name '*kernel_trace.csv' -delete; return $rc ;;
    n8)
      SDCAS_BENCH_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 500 python3 -u bench.py --gpus 8 --workload "$arg" \
        --files 100000 --steps 3 --warmup 1 --sustain-s 0 > "$OUT/n8_gloo_$arg.json" 2> "$OUT/n8_gloo_$arg.err"
      local rc=$?; cut -c1-300 "$OUT/n8_gloo_$arg.json"; return $rc ;;
    dedupfull)
      IFS=: read -r w rest <<< "$arg"
      timeout -k 10 900 python -u tools/dedup_full.py --workload "$w" ${rest//\~/ } --out "$OUT/dedup_full_${w}_$n.json" \
        > "$OUT/dedup_full_${w}_$n.log" 2>&1
      local rc=$?; tail -3 "$OUT/dedup_full_${w}_$n.log" | cut -c1-400; return $rc ;;
    pmcdedup)
      IFS=: read -r w rest <<< "$arg"
      bash tools/pmc_dedup.sh "$OUT/pmc_dedup_$w" "$w" 3 ${rest//\~/ } ;;
    probe)
      timeout -k 10 600 python -u tools/dedup_probe.py ${arg//\~/ } > "$OUT/probe_$n.json" 2> "$OUT/probe_$n.err"
      local rc=$?; cut -c1-600 "$OUT/probe_$n.json"; return $rc ;;
    jobbench)
      local a=${arg//\~/ }
      timeout -k 10 600 tests/cpp/build/job_bench ${a:-100000} > "$OUT/job_bench_$n.json" 2> "$OUT/job_bench_$n.err"
      local rc=$?; tail -c 800 "$OUT/job_bench_$n.json"; return $rc ;;
    trace)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/$OUT/trace_$n" -o trace \
        --output-format csv -- python3 "$R"/${arg//\~/ } > "$R/$OUT/trace_$n.log" 2>&1)
      local rc=$?; tail -2 "$OUT/trace_$n.log" | cut -c1-300; return $rc ;;
    cmd)
      timeout -k 10 600 bash -c "${arg//\~/ }" > "$OUT/cmd_$n.log" 2>&1
      local rc=$?; tail -5 "$OUT/cmd_$n.log"; return $rc ;;
    *) echo "unknown step $s"; return 2 ;;
  esac
}
for s in "$@"; do
  step "$s" || { echo "step '$s' failed (rc=$?): stopping"; exit 1; }
done
echo "all steps ok"
