#!/usr/bin/env python3
"""Randomised parity sweep of the path calls (TEST INFRASTRUCTURE: the oracle
is the checker). For --rounds rounds: a fresh directory of random files —
sizes from empty to several MiB, around the 100 KiB whole-file / sampled
cut and the 1 MiB piece, random bytes — then sdcas_cas_ids with each file's
size (and, for a few, a size recorded larger or smaller than the file: the
reference's UnexpectedEof and grown-file cases), sdcas_file_metadata with
those recorded sizes as its staging hints (FileMetadata::new: the size from
the read's own descriptor, a cas_id for every non-empty file; round 6) and
sdcas_checksums, every key, size, flag, digest and status against the
oracle's cas.rs / hash.rs restatements.
Prints one JSON line.

usage: stress_files.py [--rounds 4] [--files 3000] [--dir $TMPDIR/sdcas_stress]"""
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
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--files", type=int, default=3000)
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "sdcas_stress"))
    a = ap.parse_args()
    from spacedrive_amd import Engine
    from spacedrive_amd.engine import key_to_hex
    from tests._oracle import load_oracle

    oracle = load_oracle()
    eng = Engine()
    bad = []
    files = bytes_total = 0
    t0 = time.perf_counter()
    for rnd in range(a.rounds):
        rng = np.random.default_rng(500 + rnd)
        shutil.rmtree(a.dir, ignore_errors=True)
        os.makedirs(a.dir)
        paths, sizes = [], []
        for i in range(a.files):
            k = rng.integers(0, 5)
            L = [rng.integers(0, 4096), 102_400 + rng.integers(-3, 4), rng.integers(0, 300_000),
                 1_048_576 + rng.integers(-2, 3), rng.integers(0, 5_000_000)][k]
            L = max(int(L), 0)
            p = os.path.join(a.dir, f"f{i:05d}")
            with open(p, "wb") as f:
                f.write(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
            paths.append(p)
            sizes.append(L)
        rec = list(sizes)
        for i in rng.choice(a.files, size=min(20, a.files), replace=False):
            rec[i] = max(0, sizes[i] + int(rng.choice([-5000, -1, 1, 5000, 200_000])))
        sel = [i for i in range(a.files) if rec[i] > 0]  # the identifier hashes non-empty files only
        keys, st = eng.generate_cas_ids([paths[i] for i in sel], [rec[i] for i in sel])
        for j, i in enumerate(sel):
            try:
                want, wst = oracle.generate_cas_id(paths[i], rec[i]), 0
            except OSError as e:
                want, wst = None, e.errno
            got_ok = int(st[j]) == 0
            if (wst == 0) != got_ok or (got_ok and key_to_hex(keys[j]) != want):
                bad.append({"round": rnd, "file": i, "size": sizes[i], "recorded": rec[i], "call": "cas_ids",
                            "status": int(st[j]), "oracle_status": wst})
        # FileMetadata::new (mod.rs:48-96) over every file, planned from the
        # recorded sizes: actual sizes, keys of the non-empty files
        ms, mk, mst, mfl = eng.file_metadata(paths, rec)
        for i in range(a.files):
            ok = int(mst[i]) == 0 and int(ms[i]) == sizes[i] and int(mfl[i]) == (1 if sizes[i] else 0)
            if ok and sizes[i]:
                ok = key_to_hex(mk[i]) == oracle.generate_cas_id(paths[i], sizes[i])
            if not ok:
                bad.append({"round": rnd, "file": i, "size": sizes[i], "recorded": rec[i], "call": "file_metadata",
                            "status": int(mst[i]), "got_size": int(ms[i]), "flags": int(mfl[i])})
        dig, st2 = eng.file_checksums(paths)
        for i in range(a.files):
            if int(st2[i]) != 0 or bytes(dig[i]).hex() != oracle.file_checksum(paths[i]):
                bad.append({"round": rnd, "file": i, "size": sizes[i], "call": "checksums", "status": int(st2[i])})
        files += a.files
        bytes_total += int(sum(sizes))
        print(f"round {rnd}: {files} files, {len(bad)} mismatching", file=sys.stderr, flush=True)
    shutil.rmtree(a.dir, ignore_errors=True)
    print(json.dumps({"rounds": a.rounds, "files": files, "bytes": bytes_total, "n_mismatching": len(bad),
                      "mismatching": bad[:20], "seconds": time.perf_counter() - t0}))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
