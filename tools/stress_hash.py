#!/usr/bin/env python3
"""Randomised parity sweep of the hash path (TEST INFRASTRUCTURE: the oracle
is the checker). For --batches random batches — message counts from 1 to a
few thousand, lengths drawn from a mixture of tiny messages, lengths at and
around chunk (1 KiB) and tile (1 MiB) multiples, cas-message sizes and a few
multi-MiB messages, random bytes — every BLAKE3 digest of sdcas_hash_messages
(hash_messages: pinned staging, the small-batch and leaf kernels, the
tile-crossing finish, the 1 MiB-piece path above 1 MiB) against the oracle's
BLAKE3. Prints one JSON line: batches, messages, bytes, mismatches.

usage: stress_hash.py [--batches 200] [--seed 0]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def lengths(rng, n):
    kind = rng.integers(0, 6, n)
    out = np.empty(n, np.int64)
    for i, k in enumerate(kind):
        if k == 0:
            out[i] = rng.integers(0, 256)
        elif k == 1:
            out[i] = rng.integers(1, 64) * 1024 + rng.integers(-2, 3)
        elif k == 2:
            out[i] = rng.integers(0, 102_400 + 9)  # whole-file cas messages
        elif k == 3:
            out[i] = 57_352  # a sampled cas message (8 + 8 KiB + 4 x 10 KiB + 8 KiB)
        elif k == 4:
            out[i] = rng.integers(1, 4) * 1_048_576 + rng.integers(-1025, 1026)
        else:
            out[i] = rng.integers(0, 8192)
    return np.maximum(out, 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=200)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    from spacedrive_amd import Engine
    from tests._oracle import load_oracle

    oracle = load_oracle()
    eng = Engine()
    rng = np.random.default_rng(a.seed)
    msgs_total = bytes_total = 0
    bad = []
    t0 = time.perf_counter()
    for b in range(a.batches):
        n = int(rng.choice([1, 2, 3, 17, 100, 1000, 4000]))
        lens = lengths(rng, n)
        if lens.sum() > (96 << 20):  # keep a batch's bytes bounded
            lens = lens[np.cumsum(lens) <= (96 << 20)]
            if lens.size == 0:
                lens = np.array([1], np.int64)
        msgs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in lens]
        out = eng.hash_messages(*eng.pack(msgs))
        for i, (m, d) in enumerate(zip(msgs, out)):
            if bytes(d).hex() != oracle.hash(m):
                bad.append({"batch": b, "index": i, "len": len(m)})
        msgs_total += len(msgs)
        bytes_total += int(lens.sum())
        if b % 20 == 19:
            print(f"batch {b}: {msgs_total} messages, {len(bad)} mismatching", file=sys.stderr, flush=True)
    print(json.dumps({"batches": a.batches, "messages": msgs_total, "bytes": bytes_total, "mismatching": bad[:20],
                      "n_mismatching": len(bad), "seconds": time.perf_counter() - t0}))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
