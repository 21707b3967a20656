#!/usr/bin/env python3
"""profiles/r06_dedup_full_<w>.json from one tools/gpu.sh session: the plain
full-corpus run (tools/dedup_full.py, every link against the oracle), the
run with existing Objects and I/O errors (stays rows: the job's plan), and
the PMC passes over the plain run (tools/pmc_dedup.sh W 3 full, summarised by
tools/pmc_dedup_summary.py with 4 calls: 3 reps + the sizing call).

usage: dedup_full_summary.py OUTDIR WORKLOAD PLAIN.json STAYS.json PMCDIR DST"""
import json
import os
import subprocess
import sys


def last_json(path):
    line = None
    for ln in open(path):
        if ln.startswith("{"):
            line = ln
    return json.loads(line)


def main():
    outdir, w, plain, stays, pmcdir, dst = sys.argv[1:7]
    a, b = last_json(plain), last_json(stays)
    tmp = os.path.join(outdir, f"pmc_summary_{w}.json")
    here = os.path.dirname(os.path.abspath(__file__))
    subprocess.run([sys.executable, os.path.join(here, "pmc_dedup_summary.py"), pmcdir, tmp, "4"], check=True)
    pmc = json.load(open(tmp))
    keep = lambda d: {k: v for k, v in d.items() if k != "ms_all"}
    out = {
        "what": "the identifier dedup (file_identifier/mod.rs:149-254 in the job's steps) over the WHOLE "
                f"BASELINE {w.upper()} corpus in one world-of-one call (sdcas_dev_dedup_local) on one MI355X",
        "plain": keep(a),
        "with_existing_and_errors": keep(b),
        "pmc_plain": {k: pmc[k] for k in ("kernel_us_per_call", "hbm_bytes_per_call", "read_bytes_fetch_size_x2",
                                          "write_bytes", "tcc_hit_rate", "per_kernel") if k in pmc},
        "traffic_over_algorithmic": pmc["hbm_bytes_per_call"] / a["algorithmic_bytes"],
        "links_equal_oracle": a["device"]["links_equal"] and b["device"]["links_equal"]
        and a["host_abi"]["links_equal"] and b["host_abi"]["links_equal"],
    }
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(json.dumps({k: out[k] for k in ("traffic_over_algorithmic", "links_equal_oracle")}),
          a["ms_median"], b["ms_median"])


if __name__ == "__main__":
    main()
