#!/usr/bin/env python3
"""Randomised parity sweep of the device dedup (TEST INFRASTRUCTURE: the
oracle is the checker). For --seeds random corpora — sizes, key pools, Zipf
skew, rows without a key, I/O errors, existing Objects, chunk sizes and
virtual world sizes drawn per seed — every link and both counts of

  * the world-of-one fused path (sdcas_dev_dedup_local), and
  * the bucket protocol over R virtual ranks (combine_buckets -> exchange ->
    resolve_buckets -> apply), buckets sized to fit

against tests/_oracle.py's identifier_dedup. Prints one JSON line: cases
run, mismatching cases (seed and path), wall time.

usage: stress_dedup.py [--seeds 60] [--first-seed 0] [--max-files 200000]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=60)
    ap.add_argument("--first-seed", type=int, default=0, help="seeds first-seed .. first-seed + seeds - 1")
    ap.add_argument("--max-files", type=int, default=200_000)
    a = ap.parse_args()
    import torch

    from spacedrive_amd import Engine
    from spacedrive_amd.dist_dedup import DeviceStages
    from tests._dist_stages import dedup_virtual_buckets, make_corpus, shard
    from tests._oracle import load_oracle

    oracle = load_oracle()
    eng = Engine()
    st = DeviceStages(eng)
    bad, cases = [], 0
    t0 = time.perf_counter()
    for seed in range(a.first_seed, a.first_seed + a.seeds):
        rng = np.random.default_rng(1000 + seed)
        n = int(rng.integers(1, a.max_files))
        pool = int(rng.integers(1, max(2, n)))
        zipf = float(rng.uniform(1.05, 2.0))
        p_none, p_err = float(rng.uniform(0, 0.2)), float(rng.uniform(0, 0.1))
        n_ex = int(rng.integers(0, 2000))
        keys, has, status, existing = make_corpus(seed, n, pool=pool, zipf=zipf, p_none=p_none, p_err=p_err,
                                                  n_existing=n_ex)
        if rng.random() < 0.3:  # the tables' empty marker is a legal key
            keys[rng.integers(0, n, 3)] = np.uint64(2**64 - 1)
        cs = int(rng.choice([1, 7, 100, 1000]))
        want, wc, wl = oracle.identifier_dedup(keys, has, status, cs, existing)
        # world of one, with the existing Objects
        (k, h, s, ids), = shard(keys, has, status, existing, 1, device="cuda")[0]
        ek = torch.from_numpy(existing.view(np.int64)).cuda()
        eids = torch.arange(existing.size, dtype=torch.int64, device="cuda")
        link, cnt = st.local(k, h, s, ids, cs, ek if existing.size else None, eids if existing.size else None)
        cases += 1
        if not (np.array_equal(link.cpu().numpy(), want) and tuple(cnt.tolist()) == (wc, wl)):
            bad.append({"seed": seed, "path": "local", "n": n, "chunk": cs})
        # the bucket protocol over R virtual ranks
        R = int(rng.choice([2, 3, 5, 8]))
        shards, ex = shard(keys, has, status, existing, R, device="cuda")
        caps = (max(int(x[3].numel()) for x in shards) + 1, max(int(e[0].numel()) for e in ex) + 1)
        links, c, l, over = dedup_virtual_buckets(lambda r: st, shards, cs, ex, caps)
        cases += 1
        got = np.concatenate([x.cpu().numpy() for x in links])
        if over or not (np.array_equal(got, want) and (c, l) == (wc, wl)):
            bad.append({"seed": seed, "path": f"buckets R={R}", "n": n, "chunk": cs, "overflow": bool(over)})
        if seed % 10 == 9:
            print(f"seed {seed}: {cases} cases, {len(bad)} mismatching", file=sys.stderr, flush=True)
    print(json.dumps({"cases": cases, "mismatching": bad, "seconds": time.perf_counter() - t0}))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
