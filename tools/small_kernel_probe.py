#!/usr/bin/env python3
"""The small-batch leaf kernel on ONE message from device memory, launched
back to back (a busy GPU) and with host pauses between launches (a lone call
of the watcher or browse: an idle GPU between calls) — run under
`rocprofv3 --kernel-trace` to compare the kernel's duration in the two
regimes (measurement tool; round 6)."""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--len", type=int, default=51200)
    ap.add_argument("--calls", type=int, default=300)
    ap.add_argument("--pause-us", type=float, default=50.0)
    a = ap.parse_args()
    import torch
    from spacedrive_amd import Engine
    rng = np.random.default_rng(1)
    msg = rng.integers(0, 256, a.len + 256, dtype=np.uint8)
    with Engine() as e:
        blob = torch.from_numpy(msg).cuda()
        offs = torch.zeros(1, dtype=torch.int64, device="cuda")
        lens = torch.full((1,), a.len, dtype=torch.int64, device="cuda")
        keys = torch.zeros(1, dtype=torch.int64, device="cuda")
        e.dev_reserve(1, a.len // 1024 + 2)
        args = (blob.data_ptr(), offs.data_ptr(), lens.data_ptr(), 1)
        for _ in range(20):
            e.dev_hash_messages(*args, keys=keys.data_ptr())
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.calls):  # back to back
            e.dev_hash_messages(*args, keys=keys.data_ptr())
        torch.cuda.synchronize()
        busy = (time.perf_counter() - t0) / a.calls
        t0 = time.perf_counter()
        for _ in range(a.calls):  # one at a time, the GPU idle between
            e.dev_hash_messages(*args, keys=keys.data_ptr())
            torch.cuda.synchronize()
            t = time.perf_counter() + a.pause_us * 1e-6
            while time.perf_counter() < t:
                pass
        idle = (time.perf_counter() - t0) / a.calls
        print({"len": a.len, "calls": a.calls, "back_to_back_us_per_call": round(busy * 1e6, 1),
               "paused_us_per_call": round(idle * 1e6, 1), "key": hex(int(keys[0]) & (2**64 - 1))})


if __name__ == "__main__":
    main()
