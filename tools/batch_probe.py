#!/usr/bin/env python3
"""Per-call latency and throughput of the host-facing cas_id call
(`sdcas_cas_ids`, files in the page cache) against its batch size, next to
the reference-faithful CPU shape at the same step sizes (measurement tool).

sd-core calls `generate_cas_id` for ONE file from the watcher
(location/manager/watcher/utils.rs:236-240) and the ephemeral browse
(location/non_indexed.rs:181), and the identifier job in steps of 100 files
(file_identifier/mod.rs:34, job/mod.rs:559-673). This prints, per batch size
B, the median wall time of one call and the files/s it implies, for the
library and for the CPU restatement of the reference's step (one hashing
thread after the step's reads on an I/O pool; oracle/cpu_bench.c), so an
integrator can pick the batch size below which the CPU crate is the
lower-latency choice. One JSON line per configuration."""
import argparse
import json
import os
import shutil
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=100_000)
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "sdcas_batch_probe"))
    ap.add_argument("--batches", default="1,10,100,1000,10000,100000")
    ap.add_argument("--max-calls", type=int, default=200)
    a = ap.parse_args()
    from spacedrive_amd import Engine
    from tests._oracle import load_oracle
    import bench
    n = a.files
    sizes, _, _ = bench.files_of("c2", 0, n)
    shutil.rmtree(a.dir, ignore_errors=True)
    os.makedirs(a.dir)
    rng = np.random.default_rng(1)
    buf = rng.integers(0, 256, 1 << 17, dtype=np.uint8).tobytes()
    paths = []
    for i in range(n):
        p = os.path.join(a.dir, f"{i:07d}")
        with open(p, "wb") as f:
            f.write(buf[(i * 7919) % 4096: (i * 7919) % 4096 + int(sizes[i])])
        paths.append(p)
    o = load_oracle()
    try:
        with Engine() as e:
            ref, _ = e.generate_cas_ids(paths, sizes)  # warm: context, pool, page cache
            for B in [int(x) for x in a.batches.split(",")]:
                if B > n:
                    continue
                calls = min(n // B, a.max_calls)
                lat, bad = [], 0
                for c in range(calls):
                    lo = c * B
                    t0 = time.perf_counter()
                    got, st = e.generate_cas_ids(paths[lo:lo + B], sizes[lo:lo + B])
                    lat.append(time.perf_counter() - t0)
                    bad += int((got != ref[lo:lo + B]).sum()) + int((st != 0).sum())
                med = float(np.median(lat))
                print(json.dumps({"path": "gpu sdcas_cas_ids", "batch": B, "calls": calls, "median_ms": med * 1e3,
                                  "p90_ms": float(np.percentile(lat, 90)) * 1e3, "files_per_s": B / med,
                                  "mismatches_or_errors": bad}), flush=True)
        # the reference's step shape on the CPU: `chunk` files per step in
        # series, the step's reads on 16 I/O threads, one hashing thread
        for chunk, m in ((1, 2000), (100, 20000), (1000, 20000)):
            keys, st, secs, hasher = o.cpu_faithful(paths[:m], sizes[:m], chunk=chunk)
            bad = int((keys != ref[:m]).sum()) + int((st != 0).sum())
            print(json.dumps({"path": "cpu reference-faithful step", "batch": chunk, "steps": m // chunk,
                              "mean_step_ms": secs / (m // chunk) * 1e3, "files_per_s": m / secs,
                              "hasher": hasher, "mismatches_or_errors": bad}), flush=True)
    finally:
        shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
