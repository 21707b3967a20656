#!/usr/bin/env python3
"""Summarise tools/pmc_sq_variants.sh output (C2, 1 M files) into a profile:
per variant the SQ wave-state fractions, VALU instructions per SIMD-cycle,
VALU instructions per compression and the effective clock.
usage: pmc_sq_summary.py OUTDIR "36 39 40 41" DEST.json [leaf_ms per variant, comma list]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_table import medians  # noqa: E402

WHAT = {"36": "default k_leaf_tree<512,4,1,0,0,1,1> (ping-pong blocks, leaf order, dynamic tiles)",
        "39": "diagnostic: 36 without the in-tile tree",
        "40": "diagnostic: 36 without message loads (register-made blocks)",
        "41": "diagnostic: 36 with neither"}
COMP = 859165969          # C2 compressions per launch (bench.py compressions())
COMP_NO_TREE = COMP - 50039370  # minus the parent compressions (chunks - messages)


def main():
    src, vs, dst = sys.argv[1], sys.argv[2].split(), sys.argv[3]
    ms = dict(zip(vs, (float(x) for x in sys.argv[4].split(",")))) if len(sys.argv) > 4 else {}
    out = {"workload": "C2 (1 M files, tools/ab_leaf.py)", "source": "rocprofv3 --pmc, tools/pmc_sq_variants.sh; "
           "SQ_* are wave-cycle counts summed over the chip, GRBM over 8 XCDs", "variants": {}}
    for v in vs:
        c = medians(os.path.join(src, "v" + v), "leaf")
        c.update(medians(os.path.join(src, "g" + v), "leaf"))
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        comp = COMP_NO_TREE if v in ("39", "41") else COMP
        e = {"what": WHAT.get(v, ""), "counters": c,
             "wait_any_frac": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
             "wait_inst_frac": c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"],
             "valu_insts_per_simd_cycle": c["SQ_INSTS_VALU"] / (cyc * 1024),
             "valu_insts_per_compression": c["SQ_INSTS_VALU"] / (comp / 64),
             "cycles_per_xcd": cyc}
        if v in ms:
            e["leaf_ms"] = ms[v]
            e["clock_ghz"] = cyc / (ms[v] * 1e-3) / 1e9
        out["variants"][v] = e
    json.dump(out, open(dst, "w"), indent=1)
    for v, e in out["variants"].items():
        print(v, {k: round(x, 3) for k, x in e.items() if isinstance(x, float)})


if __name__ == "__main__":
    main()
