#!/usr/bin/env python3
"""Per-launch durations of each bench line's dominant kernel from a
rocprofv3 kernel trace (tools/r03_rocprof_final.sh OUT) against the HIP-event
figure the same run's bench line reports.
usage: rocprof_vs_bench.py OUT DST"""
import csv
import glob
import json
import os
import sys


def bench_line(log):
    for line in reversed(open(log).read().splitlines()):
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    return None


def main():
    src, dst = sys.argv[1], sys.argv[2]
    out = {"what": "rocprofv3 --kernel-trace --stats around bench.py (tools/r03_rocprof_final.sh, the final "
                   "HEAD's default kernels: leaf 67, piece 19 = k_piece_l4 + k_piece_top): the dominant "
                   "kernel's per-launch durations from the kernel trace against the HIP-event time the same "
                   "run's bench line reports; the *_kernel_stats.csv Average includes the warmup launches",
           "command": "rocprofv3 --kernel-trace --stats -- python bench.py --workload W --steps 20 --warmup 2 "
                      "--no-cpu-baseline --no-e2e (C4: --steps 2 --warmup 1)"}
    for w, steps in (("c2", 20), ("c3", 20), ("c5", 20), ("c4", 2)):
        tr = glob.glob(os.path.join(src, f"prof_{w}", "**", f"{w}_kernel_trace.csv"), recursive=True)
        logs = [os.path.join(src, f"prof_{w}.{x}") for x in ("log", "json")]
        b = next((bench_line(x) for x in logs if os.path.exists(x)), None)
        if not tr or not b:
            continue
        steps = int(b.get("steps", steps))
        rows = list(csv.DictReader(open(tr[0])))
        def launches(sub):
            return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in
                    sorted(rows, key=lambda r: int(r["Start_Timestamp"])) if sub in r["Kernel_Name"]]
        r = b["roofline"]
        if w == "c4":
            l4, top = launches("k_piece_l4"), launches("k_piece_top")
            timed = [a + t for a, t in zip(l4[-steps:], top[-steps:])]
            comp_s = r["valu"]["compressions_per_s_node"]
            out[w] = {"kernel": "k_piece_l4 + k_piece_top", "l4_launch_ms": l4, "top_launch_ms": top,
                      "timed_launches_mean_ms": sum(timed) / len(timed),
                      "bench_value": b["value"], "bench_unit": b["unit"], "bench_roofline_frac": r["frac"],
                      "bench_hip_event_piece_ms": r["compressions_per_launch"] / comp_s * 1e3}
        else:
            ls = launches("k_leaf_tree")
            timed = ls[-steps:]
            out[w] = {"kernel": "k_leaf_tree", "launch_ms": ls, "timed_launches_mean_ms": sum(timed) / len(timed),
                      "bench_value": b["value"], "bench_unit": b["unit"], "bench_roofline_frac": r["frac"],
                      "bench_ms_per_step": b["ms_per_step"], "bench_hip_event_leaf_ms": r.get("leaf_ms")}
        o = out[w]
        ref = o.get("bench_hip_event_leaf_ms") or o.get("bench_hip_event_piece_ms")
        o["trace_over_hip_events"] = o["timed_launches_mean_ms"] / ref if ref else None
    json.dump(out, open(dst, "w"), indent=1)
    for w in ("c2", "c3", "c5", "c4"):
        if w in out:
            print(w, round(out[w]["timed_launches_mean_ms"], 3), out[w].get("trace_over_hip_events"))


if __name__ == "__main__":
    main()
