#!/usr/bin/env python3
"""Summarise tools/pmc_traffic.sh output into profiles/<name>.json: HBM bytes
per launch of one kernel, corrected as MI355X_MICROARCH.md prescribes
(FETCH_SIZE counts half the bytes of wide coalesced reads on gfx950 -> x2;
cross-checked against TCC_EA0_RDREQ x request size).
usage: pmc_summarize.py SRC DST [WORKLOAD KERNEL_SUBSTR ALGORITHMIC_BYTES_PER_LAUNCH SOURCE_TEXT]"""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_traffic"
    dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/r01_pmc_c2.json"
    workload = sys.argv[3] if len(sys.argv) > 3 else "C2"
    ksub = sys.argv[4] if len(sys.argv) > 4 else "k_leaf_tree"
    algo = float(sys.argv[5]) if len(sys.argv) > 5 else None
    source = sys.argv[6] if len(sys.argv) > 6 else (
        "rocprofv3 --pmc passes (tools/pmc_traffic.sh) over tools/ab_leaf.py C2, 1M files, "
        "128-B aligned messages; FETCH_SIZE x2 per MI355X_MICROARCH.md HBM section")
    vals = collections.defaultdict(list)
    kname = None
    for f in glob.glob(os.path.join(src, "*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if ksub not in r["Kernel_Name"]:
                continue
            kname = r["Kernel_Name"]
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    med = {k: statistics.median(v) for k, v in vals.items()}
    fetch = med.get("FETCH_SIZE", 0) * 1024 * 2      # KB, x2 gfx950 correction
    write = med.get("WRITE_SIZE", 0) * 1024
    rdreq = med.get("TCC_EA0_RDREQ_128B_sum", 0) * 128 + med.get("TCC_EA0_RDREQ_64B_sum", 0) * 64 + \
        med.get("TCC_EA0_RDREQ_32B_sum", 0) * 32
    out = {
        "workload": workload, "kernel": ksub + (kname.split(ksub, 1)[1][:40] if kname else ""),
        "hbm_bytes_per_launch": fetch + write,
        "read_bytes_fetch_size_x2": fetch, "read_bytes_ea_rdreq": rdreq, "write_bytes": write,
        "counters_median": med, "launches_counted": len(vals.get("FETCH_SIZE", [])),
        "source": source,
    }
    if algo:
        out["algorithmic_bytes_per_launch"] = algo
        out["traffic_over_algorithmic"] = (fetch + write) / algo
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("hbm_bytes_per_launch", "read_bytes_ea_rdreq", "write_bytes")}))


if __name__ == "__main__":
    main()
