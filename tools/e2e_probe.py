#!/usr/bin/env python3
"""Where the page-cache cas_id path's time goes (measurement tool): writes C2
files once, then times sdcas_cas_ids over them with several I/O-thread counts
and staging sizes, and a hashing-free read of the same files by the library's
own reader (sdcas_io through tools/ubench_read, open + pread + close per file).
Prints one JSON line per configuration."""
import argparse
import json
import os
import shutil
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=200_000)
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "sdcas_probe"))
    ap.add_argument("--threads", default="8,16,24,32")
    ap.add_argument("--staging-mib", default="64,256")
    ap.add_argument("--direct", action="store_true", help="also time SDCAS_OPT_DIRECT_IO (O_DIRECT reads)")
    a = ap.parse_args()
    from spacedrive_amd import Engine
    import bench
    n = a.files
    sizes, keys, _ = bench.files_of("c2", 0, n)
    shutil.rmtree(a.dir, ignore_errors=True)
    os.makedirs(a.dir)
    rng = np.random.default_rng(1)
    buf = rng.integers(0, 256, 1 << 17, dtype=np.uint8).tobytes()
    paths = []
    t0 = time.perf_counter()
    for i in range(n):
        p = os.path.join(a.dir, f"{i:07d}")
        with open(p, "wb") as f:
            f.write(buf[: int(sizes[i])])
        paths.append(p)
    print(json.dumps({"written_s": time.perf_counter() - t0, "files": n}), flush=True)
    ub = os.path.join(ROOT, "tools", "ubench_read")
    if os.path.exists(ub):
        for t in (8, 16, 32):
            r = subprocess.run([ub, a.dir, str(n), str(t), "32", "2"], capture_output=True, text=True, timeout=300)
            print(json.dumps({"ubench_read_threads": t, "out": r.stdout.strip().splitlines()[-4:]}), flush=True)
    ref = None
    configs = [(d, mib, t) for d in ([False, True] if a.direct else [False])
               for mib in [int(x) for x in a.staging_mib.split(",")] for t in [int(x) for x in a.threads.split(",")]]
    for direct, mib, t in configs:
        with Engine(io_threads=t, staging_bytes=mib << 20, direct_io=direct) as e:
            best = None
            for _ in range(3):
                t0 = time.perf_counter()
                got, st = e.generate_cas_ids(paths, sizes)
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            if ref is None:
                ref = got
            print(json.dumps({"io_threads": t, "staging_mib": mib, "direct": direct, "files_per_s": n / best,
                              "same_as_first": bool(np.array_equal(got, ref)), "errors": int((st != 0).sum())}),
                  flush=True)
    shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
