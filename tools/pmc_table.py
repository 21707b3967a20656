#!/usr/bin/env python3
"""Per-kernel medians of rocprofv3 --pmc counter CSVs (counter_collection.csv,
summed over dimensions per dispatch). usage: pmc_table.py DIR [kernel-substring]"""
import collections
import csv
import glob
import sys


def medians(d, ksub):
    per = collections.defaultdict(float)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if ksub in r["Kernel_Name"]:
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    agg = collections.defaultdict(list)
    for (_, c), v in per.items():
        agg[c].append(v)
    return {c: sorted(v)[len(v) // 2] for c, v in agg.items()}


if __name__ == "__main__":
    print(medians(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "leaf"))
