#!/usr/bin/env python3
"""Per-call latency of sdcas_cas_ids at the C ABI (measurement tool).

Writes C2-shaped files (bench.files_of("c2")) to the page cache, a manifest of
"size path" lines, and runs tools/ubench_latency (built beforehand:
g++ -O2 -std=c++17 tools/ubench_latency.cpp -ldl -o tools/ubench_latency) on
one library or two side by side, as a child process: no Python in the timed
region, so the numbers are what a Rust or C caller of the library sees.
"""
import argparse
import os
import shutil
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=20_000)
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "sdcas_latency_probe"))
    ap.add_argument("--batches", default="1,10,100,1000")
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("libs", nargs="*", default=[os.path.join(ROOT, "spacedrive_amd", "libsdcas.so")])
    a = ap.parse_args()
    import bench
    sizes, _, _ = bench.files_of("c2", 0, a.files)
    shutil.rmtree(a.dir, ignore_errors=True)
    os.makedirs(a.dir)
    rng = np.random.default_rng(1)
    buf = rng.integers(0, 256, 1 << 17, dtype=np.uint8).tobytes()
    man = os.path.join(a.dir, "manifest.txt")
    try:
        with open(man, "w") as m:
            for i in range(a.files):
                p = os.path.join(a.dir, f"{i:07d}")
                with open(p, "wb") as f:
                    f.write(buf[(i * 7919) % 4096: (i * 7919) % 4096 + int(sizes[i])])
                m.write(f"{int(sizes[i])} {p}\n")
        exe = os.path.join(ROOT, "tools", "ubench_latency")
        r = subprocess.run([exe, man, a.batches, str(a.calls)] + a.libs)
        return r.returncode
    finally:
        shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    sys.exit(main())
