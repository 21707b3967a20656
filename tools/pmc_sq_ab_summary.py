#!/usr/bin/env python3
"""Summarise tools/pmc_sq_ab.sh: per (leaf variant, workload), VALU / SALU /
LDS instructions per compression, VALU issue per SIMD per cycle, cycles per
XCD and the clock (GRBM_GUI_ACTIVE per XCD over the leaf time the same run
printed). usage: pmc_sq_ab_summary.py SRC [DST.json]"""
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

SIMDS, XCDS = 1024, 8
N = {"c2": 1_000_000, "c3": 1_250_000, "c5": 6_250_000}


def main():
    src = sys.argv[1]
    out = {"source": f"rocprofv3 --pmc passes (tools/pmc_sq_ab.sh) over tools/ab_leaf.py (ablation library), {src}",
           "runs": {}}
    keys = sorted({tuple(os.path.basename(d).split("_")[1:]) for d in glob.glob(os.path.join(src, "s_*"))})
    for w, v in keys:
        sizes, _, _ = bench.files_of(w, 0, N[w])
        comp = int(bench.compressions(bench.S.cas_msg_len(sizes)).sum())
        acc = collections.defaultdict(float)
        ms = []
        for p in ("s", "g"):
            for f in glob.glob(os.path.join(src, f"{p}_{w}_{v}", "**", "*counter_collection.csv"), recursive=True):
                for r in csv.DictReader(open(f)):
                    if "k_leaf_tree" in r["Kernel_Name"]:
                        acc[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            log = os.path.join(src, f"{p}_{w}_{v}.log")
            if os.path.exists(log):
                ms += [float(x) for x in re.findall(r"leaf med ([0-9.]+)", open(log).read())]
        per = collections.defaultdict(list)
        for (_, c), x in acc.items():
            per[c].append(x)
        m = {c: statistics.median(x) for c, x in per.items()}
        if "SQ_INSTS_VALU" not in m or "GRBM_GUI_ACTIVE" not in m:
            continue
        kms = statistics.median(ms) if ms else None
        cyc = m["GRBM_GUI_ACTIVE"] / XCDS
        out["runs"][f"{w}_v{v}"] = {
            "workload": w, "variant": int(v), "compressions": comp, "leaf_ms_under_pmc": kms,
            "valu_per_compression": m["SQ_INSTS_VALU"] * 64 / comp,
            "salu_per_compression": m["SQ_INSTS_SALU"] * 64 / comp,
            "lds_per_compression": m["SQ_INSTS_LDS"] * 64 / comp,
            "valu_instr_per_simd_per_cycle": m["SQ_INSTS_VALU"] / SIMDS / cyc,
            "cycles_per_xcd": cyc, "clock_ghz": cyc / (kms * 1e6) if kms else None,
            "counters_median": m}
    for k, d in out["runs"].items():
        print(k, {a: round(b, 4) if isinstance(b, float) else b for a, b in d.items() if a != "counters_median"})
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
