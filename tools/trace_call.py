#!/usr/bin/env python3
"""Timeline of single path calls from a rocprofv3 trace (kernel, memory-copy
and HIP-API CSVs of tools/latency_trace.sh): every event between two
consecutive hipEventSynchronize returns, relative to the first (µs)."""
import csv
import os
import sys

SKIP = {"hipGetDevice", "hipGetLastError", "hipGetStreamDeviceId"}


def load(d):
    ev = []
    for r in csv.DictReader(open(os.path.join(d, "t_hip_api_trace.csv"))):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "API", r["Function"], r["Thread_Id"]))
    for r in csv.DictReader(open(os.path.join(d, "t_kernel_trace.csv"))):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K",
                   r["Kernel_Name"][:50] + " g%s" % r["Grid_Size_X"], r["Stream_Id"]))
    p = os.path.join(d, "t_memory_copy_trace.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "MC", r["Direction"], r["Stream_Id"]))
    ev.sort()
    return ev


def main():
    d = sys.argv[1]
    ev = load(d)
    syncs = [e for e in ev if e[3] == "hipEventSynchronize"]
    for k in [int(x) for x in sys.argv[2:]]:
        a, b = syncs[k][1], syncs[k + 1][1]
        print(f"--- call ending at sync {k + 1}: {(b - a) / 1e3:.1f} us")
        for e in ev:
            if a <= e[0] <= b and e[3] not in SKIP:
                print("%8.1f %7.1f %-3s %s %s" % ((e[0] - a) / 1e3, (e[1] - e[0]) / 1e3, e[2], e[3], e[4]))


if __name__ == "__main__":
    main()
