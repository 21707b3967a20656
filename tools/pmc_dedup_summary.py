#!/usr/bin/env python3
"""Summarise tools/pmc_dedup.sh into profiles/<name>.json: per dedup call,
the kernel time (kernel trace) and the HBM bytes (FETCH_SIZE x2 per
MI355X_MICROARCH.md, WRITE_SIZE), summed over every dispatch after the hash's
last kernel (tools/dedup_probe.py creates all the dedup's inputs before the
hash), divided by the probe's dedup calls; with a per-kernel breakdown.

usage: pmc_dedup_summary.py SRC DST CALLS"""
import collections
import csv
import glob
import json
import os
import re
import sys

HASH = ("k_leaf_tree", "k_finish_t", "k_finish_q", "k_tile_first", "k_plan_", "k_shape_", "k_synth_cas_messages")


def short(name):
    n = name.split("(")[0]
    n = re.sub(r"^void ", "", n)
    if "rocprim" in n:
        m = re.search(r"detail::(\w+)", n)
        return "rocprim::" + (m.group(1) if m else "kernel")
    return n[:60]


def rows(src, pass_name, kind):
    for f in glob.glob(os.path.join(src, pass_name, f"*_{kind}.csv")):
        yield from csv.DictReader(open(f))


def after_hash(rs):
    """the dispatches after the hash's last kernel, up to the last dedup
    apply (the probe's read-back copies after it are not the dedup's)"""
    rs = sorted(rs, key=lambda r: int(r["Dispatch_Id"]))
    # the hash's kernels before the first dedup insert (a later hash, e.g. a
    # parity check after the calls, is not the boundary)
    first = min((int(r["Dispatch_Id"]) for r in rs if "insert" in r["Kernel_Name"]), default=1 << 62)
    last = max((int(r["Dispatch_Id"]) for r in rs
                if any(h in r["Kernel_Name"] for h in HASH) and int(r["Dispatch_Id"]) < first), default=-1)
    end = max((int(r["Dispatch_Id"]) for r in rs if "apply" in r["Kernel_Name"]), default=1 << 62)
    return [r for r in rs if last < int(r["Dispatch_Id"]) <= end]


def main():
    src, dst, calls = sys.argv[1], sys.argv[2], int(sys.argv[3])
    # kernel time per call from the trace pass
    tr = after_hash(list(rows(src, "trace", "kernel_trace")))
    per_k = collections.defaultdict(lambda: [0, 0.0])
    for r in tr:
        k = short(r["Kernel_Name"])
        per_k[k][0] += 1
        per_k[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    kernel_us = sum(v[1] for v in per_k.values()) / calls
    # counters per call: sum over the dedup's dispatches
    byk = collections.defaultdict(lambda: collections.defaultdict(float))
    tot = collections.defaultdict(float)
    for p in ("fetch", "write", "req", "tcc"):
        for r in after_hash(list(rows(src, p, "counter_collection"))):
            v = float(r["Counter_Value"])
            tot[r["Counter_Name"]] += v
            byk[short(r["Kernel_Name"])][r["Counter_Name"]] += v
    fetch = tot["FETCH_SIZE"] * 1024 * 2 / calls
    write = tot["WRITE_SIZE"] * 1024 / calls
    rdreq = (tot["TCC_EA0_RDREQ_128B_sum"] * 128 + tot["TCC_EA0_RDREQ_64B_sum"] * 64 +
             tot["TCC_EA0_RDREQ_32B_sum"] * 32) / calls
    probe = None
    for lg in glob.glob(os.path.join(src, "trace.log")):
        for ln in open(lg):
            if ln.startswith("{"):
                probe = json.loads(ln)
    out = {
        "workload": probe["workload"] if probe else None, "kernel": "dedup (world of one: sdcas_dev_dedup_local)",
        "files": probe["files"] if probe else None, "calls": calls,
        "kernel_us_per_call": kernel_us,
        "hbm_bytes_per_call": fetch + write, "read_bytes_fetch_size_x2": fetch, "read_bytes_ea_rdreq": rdreq,
        "write_bytes": write,
        "tcc_hit_rate": tot["TCC_HIT_sum"] / max(1.0, tot["TCC_HIT_sum"] + tot["TCC_MISS_sum"]),
        "per_kernel": {k: {"launches_per_call": v[0] / calls, "us_per_call": v[1] / calls,
                           "fetch_bytes_x2": byk[k]["FETCH_SIZE"] * 2048 / calls,
                           "write_bytes": byk[k]["WRITE_SIZE"] * 1024 / calls}
                       for k, v in sorted(per_k.items(), key=lambda kv: -kv[1][1])},
        "probe": probe,
        "source": f"rocprofv3 --kernel-trace and --pmc passes (tools/pmc_dedup.sh) over tools/dedup_probe.py; "
                  f"every dispatch after the hash's last kernel, / {calls} dedup calls; FETCH_SIZE x2 per "
                  f"MI355X_MICROARCH.md (random 16-B accesses: uncalibrated, EA RDREQ x request size beside it)",
    }
    if probe:
        out["algorithmic_bytes_per_call"] = probe["algorithmic_bytes"]
        out["traffic_over_algorithmic"] = (fetch + write) / probe["algorithmic_bytes"]
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("kernel_us_per_call", "hbm_bytes_per_call", "read_bytes_ea_rdreq",
                                          "write_bytes")}))


if __name__ == "__main__":
    main()
