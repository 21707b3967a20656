#!/usr/bin/env python3
"""End-to-end (PCIe- and I/O-inclusive) throughput of the host-facing C ABI,
reported separately from bench.py's on-device headline.

  messages  sdcas_cas_ids_from_messages: C2 cas messages already in host RAM
            -> double-buffered pinned staging -> H2D -> kernels -> keys
  files     sdcas_cas_ids: C2 files in the page cache (tmpfs/local disk) read
            with cas.rs's pattern by the library's I/O threads into pinned
            staging, overlapped with H2D + hashing of the previous batch
  checksum  sdcas_checksums over the same files (hash.rs: whole content)

Every GPU key is checked against the device-resident path
(sdcas_dev_hash_messages) on the same messages. Prints one JSON line.
"""
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
    ap.add_argument("--dir", default="/tmp/sdcas_e2e")
    ap.add_argument("--io-threads", type=int, default=16)
    ap.add_argument("--staging-mib", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    from spacedrive_amd import Engine
    from spacedrive_amd import synth as S

    n = a.files
    sizes, keys = S.c2_files(0, n)
    lens = S.cas_msg_len(sizes)
    padded = (lens + np.uint64(127)) // np.uint64(128) * np.uint64(128)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(padded[:-1])
    total = int(offs[-1] + padded[-1]) + 64
    dev = torch.device("cuda", 0)
    eng = Engine(io_threads=a.io_threads, staging_bytes=a.staging_mib << 20)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).to(dev)
    d_blob = torch.empty(total, dtype=torch.uint8, device=dev)
    dk, ds, do, dl = t(keys), t(sizes), t(offs), t(lens)
    eng.dev_reserve(n, int(((lens + np.uint64(1023)) // np.uint64(1024)).sum()))
    eng.dev_synth_cas_messages(dk.data_ptr(), ds.data_ptr(), do.data_ptr(), n, d_blob.data_ptr())
    d_out = torch.zeros(n, dtype=torch.int64, device=dev)
    eng.dev_sync()
    eng.dev_hash_messages(d_blob.data_ptr(), do.data_ptr(), dl.data_ptr(), n, 0, d_out.data_ptr())
    eng.dev_sync()
    want = d_out.cpu().numpy().view(np.uint64)
    host = d_blob.cpu().numpy()
    del d_blob
    msg_bytes = int(lens.sum())
    out = {"workload": f"C2 files [0,{n})", "n_files": n, "message_bytes": msg_bytes,
           "staging_bytes_per_slot": a.staging_mib << 20, "io_threads": a.io_threads}

    # PCIe reference: pinned host -> HBM copy bandwidth (the roof of every
    # host-facing path)
    pin = torch.empty(256 << 20, dtype=torch.uint8).pin_memory()
    dst = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
    dst.copy_(pin, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(8):
        dst.copy_(pin, non_blocking=True)
    torch.cuda.synchronize()
    out["pcie_h2d_pinned_gbps"] = 8 * (256 << 20) / (time.perf_counter() - t0) / 1e9
    del pin, dst

    # (a) messages in host RAM
    best = None
    for _ in range(a.reps):
        t0 = time.perf_counter()
        got = eng.cas_ids_from_messages(host, offs, lens)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    out["messages"] = {"files_per_s": n / best, "gbps": msg_bytes / best / 1e9, "seconds": best,
                       "mismatches": int((got != want).sum())}

    # (a') the same messages in a pinned caller buffer: direct DMA, no copy
    pin = torch.empty(host.size, dtype=torch.uint8).pin_memory()
    pin.numpy()[:] = host
    best = None
    for _ in range(a.reps):
        t0 = time.perf_counter()
        got = eng.cas_ids_from_messages(pin.numpy(), offs, lens)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    out["messages_pinned"] = {"files_per_s": n / best, "gbps": msg_bytes / best / 1e9, "seconds": best,
                              "mismatches": int((got != want).sum())}
    del pin

    # (b) files in the page cache
    shutil.rmtree(a.dir, ignore_errors=True)
    os.makedirs(a.dir)
    paths = []
    t0 = time.perf_counter()
    for i in range(n):
        p = os.path.join(a.dir, f"{i:07d}")
        o = int(offs[i])
        with open(p, "wb") as f:
            f.write(host[o + 8:o + int(lens[i])].tobytes())
        paths.append(p)
    out["files_written_s"] = time.perf_counter() - t0
    del host
    best = None
    for _ in range(a.reps):
        t0 = time.perf_counter()
        got, st = eng.generate_cas_ids(paths, sizes)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    out["files"] = {"files_per_s": n / best, "gbps": msg_bytes / best / 1e9, "seconds": best,
                    "mismatches": int((got != want).sum()), "errors": int((st != 0).sum()),
                    "storage": "page cache (files just written)"}

    # (c) checksums of the same files
    best = None
    for _ in range(a.reps):
        t0 = time.perf_counter()
        d32, st = eng.file_checksums(paths)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    out["checksums"] = {"files_per_s": n / best, "gbps": int(sizes.sum()) / best / 1e9, "seconds": best,
                        "errors": int((st != 0).sum())}
    shutil.rmtree(a.dir, ignore_errors=True)
    eng.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
