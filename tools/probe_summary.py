"""one line per A/B setting of tools/dedup_probe.py outputs"""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["workload"], "world", d.get("world", 1))
    if "ab" in d:
        for k, v in d["ab"].items():
            print(f"   {k:60s} {v['ms_median']:.4f} ms")
        print("   equal", d.get("ab_equal"))
    else:
        for k, v in d["ms_median"].items():
            print(f"   {k:60s} " + " ".join(f"{s} {t:.4f}" for s, t in v.items()) + f"  total {d['ms_total'][k]:.4f}")
        print("   equal", d["equal"])
