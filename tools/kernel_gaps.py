#!/usr/bin/env python3
"""Idle gaps between consecutive kernels of a rocprofv3 kernel trace (CSV):
for every kernel whose name matches --after, the gap from its end to the next
kernel's start on the same queue. Used to check that a bound stream
(sdcas_dev_bind_stream) removes the scratch fence's wait between the hash and
the dedup of a bench step.

usage: kernel_gaps.py TRACE.csv [--after k_finish_q] [--json]"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--after", default="k_finish_q")
    ap.add_argument("--skip", type=int, default=1, help="leading matches to ignore (warm-up)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    gaps, nxt = [], {}
    for i, r in enumerate(rows[:-1]):
        if a.after not in r["Kernel_Name"]:
            continue
        q = r.get("Queue_Id") or r.get("Stream_Id") or "0"
        j = i + 1
        while j < len(rows) and (rows[j].get("Queue_Id") or rows[j].get("Stream_Id") or "0") != q:
            j += 1
        if j == len(rows):
            continue
        g = (int(rows[j]["Start_Timestamp"]) - int(r["End_Timestamp"])) / 1e3
        gaps.append(g)
        name = rows[j]["Kernel_Name"].split("(")[0][:40]
        nxt[name] = nxt.get(name, 0) + 1
    gaps = gaps[a.skip:]
    print(json.dumps({"after": a.after, "count": len(gaps), "gap_us_median": statistics.median(gaps) if gaps else None,
                      "gap_us_max": max(gaps) if gaps else None, "gap_us_min": min(gaps) if gaps else None,
                      "next_kernels": nxt}))


if __name__ == "__main__":
    main()
