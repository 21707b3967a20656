#!/usr/bin/env python3
"""Summarise tools/pmc_sq_workloads.sh: per leaf workload, the default leaf
kernel's VALU / SALU / LDS / VMEM instructions per compression, VALU issue per
SIMD per cycle, HBM read bytes over the algorithmic message bytes, and the
clock the kernel ran at (GRBM_GUI_ACTIVE per XCD over the kernel time the same
run printed).
Also writes profiles/<PREFIX>_pmc_<w>.json for C3 and C5 (the HBM traffic per
launch in tools/pmc_summarize.py's format, which bench.py reads); C2's comes
from tools/pmc_traffic.sh's dedicated passes.
usage: pmc_sq_workloads_summary.py SRC DST [VARIANT [PREFIX]]   (VARIANT: the leaf
variant the passes ran, tools/pmc_sq_workloads.sh's $VARIANT, default 67;
PREFIX: the round prefix of the per-workload traffic files, default r03)"""
import collections
import csv
import glob
import json
import os
import re
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

WORKLOADS = (("c2", 1_000_000), ("c3", 1_250_000), ("c5", 6_250_000))
SIMDS = 1024
XCDS = 8


def main():
    src, dst = sys.argv[1], sys.argv[2]
    variant = int(sys.argv[3]) if len(sys.argv) > 3 else 67
    prefix = sys.argv[4] if len(sys.argv) > 4 else "r03"
    out = {"source": "rocprofv3 --pmc passes (tools/pmc_sq_workloads.sh) over tools/ab_leaf.py --product "
                     f"--variants {variant}, one counter group per run; FETCH_SIZE x2 per MI355X_MICROARCH.md",
           "workloads": {}}
    for w, n in WORKLOADS:
        sizes, _, _ = bench.files_of(w, 0, n)
        lens = bench.S.cas_msg_len(sizes)
        comp = int(bench.compressions(lens).sum())
        msg = int(lens.sum())
        slots = int(np.maximum(1, (lens + 1023) // 1024).sum())
        acc = collections.defaultdict(float)
        ms = []
        for p in ("s", "g", "f", "w"):
            for f in glob.glob(os.path.join(src, f"{p}_{w}", "*counter_collection.csv")):
                for r in csv.DictReader(open(f)):
                    if "k_leaf_tree" in r["Kernel_Name"]:
                        acc[(p, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            log = os.path.join(src, f"{p}_{w}.log")
            if os.path.exists(log):
                ms += [float(x) for x in re.findall(r"leaf med ([0-9.]+)", open(log).read())]
        if not acc:
            continue
        per = collections.defaultdict(list)
        for (_, _, c), x in acc.items():
            per[c].append(x)
        m = {c: statistics.median(x) for c, x in per.items()}
        kms = statistics.median(ms) if ms else None
        cyc = m["GRBM_GUI_ACTIVE"] / XCDS
        out["workloads"][w] = {
            "files": n, "compressions": comp, "message_bytes": msg, "chunk_slots": slots,
            "leaf_kernel_ms_under_pmc": kms,
            "valu_per_compression": m["SQ_INSTS_VALU"] * 64 / comp,
            "salu_per_compression": m["SQ_INSTS_SALU"] * 64 / comp,
            "lds_per_compression": m["SQ_INSTS_LDS"] * 64 / comp,
            "vmem_rd_per_compression": m["SQ_INSTS_VMEM_RD"] * 64 / comp,
            "valu_instr_per_simd_per_cycle": m["SQ_INSTS_VALU"] / SIMDS / cyc,
            "cycles_per_xcd": cyc,
            "clock_ghz": cyc / (kms * 1e6) if kms else None,
            "wait_any_over_wave_cycles": m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"],
            "hbm_read_over_algorithmic": m["FETCH_SIZE"] * 1024 * 2 / msg,
            "hbm_write_bytes": m["WRITE_SIZE"] * 1024,
            "counters_median": m,
        }
    json.dump(out, open(dst, "w"), indent=1)
    # the kernel name bench.load_traffic matches against its default kernel
    kernel = {51: "k_leaf_tree<512, 109, 1, 1, 2, 2, 0>", 52: "k_leaf_tree<512, 209, 1, 1, 2, 2, 0, 1024u>",
              67: "k_leaf_tree<512, 279, 1, 1, 2, 2, 0, 1024u>"}[variant]
    for w in ("c3", "c5"):
        d = out["workloads"].get(w)
        if not d:
            continue
        m = d["counters_median"]
        rd = m["FETCH_SIZE"] * 1024 * 2
        tr = {"workload": w.upper(), "kernel": kernel, "hbm_bytes_per_launch": rd + m["WRITE_SIZE"] * 1024,
              "read_bytes_fetch_size_x2": rd, "write_bytes": m["WRITE_SIZE"] * 1024,
              "algorithmic_bytes_per_launch": d["message_bytes"],
              "traffic_over_algorithmic": (rd + m["WRITE_SIZE"] * 1024) / d["message_bytes"],
              "source": out["source"] + f"; {w.upper()} {d['files']} files"}
        json.dump(tr, open(os.path.join(os.path.dirname(dst), f"{prefix}_pmc_{w}.json"), "w"), indent=1)
    for w, d in out["workloads"].items():
        print(w, {k: round(v, 4) if isinstance(v, float) else v for k, v in d.items() if k != "counters_median"})


if __name__ == "__main__":
    main()
