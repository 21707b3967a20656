#!/usr/bin/env python3
"""End-to-end file_checksum (hash.rs:11-25) of big files through the C ABI
(sdcas_checksums): C4-sized files written to a local directory, read back
with the page cache (buffered) and with O_DIRECT (SDCAS_OPT_DIRECT_IO; the
page cache is dropped for these files with posix_fadvise first where it can
be), the window's 1 MiB pieces read by the I/O threads in parallel. Digests
are checked against the device-resident stream path. One JSON line."""
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
    ap.add_argument("--gib", type=int, default=8)
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "sdcas_e2e_big"))
    ap.add_argument("--io-threads", type=int, default=16)
    ap.add_argument("--staging-mib", type=int, default=256)
    a = ap.parse_args()
    import torch

    from spacedrive_amd import Engine
    from spacedrive_amd import synth as S
    MiB = 1 << 20
    sizes, keys = S.c4_files(a.gib << 30)
    dev = torch.device("cuda", 0)
    shutil.rmtree(a.dir, ignore_errors=True)
    os.makedirs(a.dir)
    eng = Engine(io_threads=a.io_threads, staging_bytes=a.staging_mib << 20)
    # generate each file in HBM, take its digest from the stream path, write it out
    paths, want = [], []
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x, dtype=np.uint64).view(np.int64)).to(dev)
    t0 = time.perf_counter()
    for i, (n, k) in enumerate(zip(sizes, keys)):
        n = int(n)
        blob = torch.empty(n + 4096, dtype=torch.uint8, device=dev)
        args = [t([k]), t([0]), t([n]), t([0])]
        torch.cuda.synchronize()
        eng.dev_synth_content(*(x.data_ptr() for x in args), 1, blob.data_ptr())
        out = torch.zeros((1, 32), dtype=torch.uint8, device=dev)
        eng.dev_stream_begin([n])
        eng.dev_stream_update([0], [0], [n], [blob.data_ptr()])
        eng.dev_stream_finish(out.data_ptr())
        eng.dev_sync()
        want.append(bytes(out.cpu().numpy()[0]))
        p = os.path.join(a.dir, f"f{i:03d}")
        blob[:n].cpu().numpy().tofile(p)
        paths.append(p)
        del blob
    res = {"files": len(paths), "bytes": int(sizes.sum()), "written_s": time.perf_counter() - t0,
           "io_threads": a.io_threads, "staging_bytes_per_slot": a.staging_mib << 20}
    eng.close()
    for mode in ("buffered", "direct"):
        if mode == "direct":
            for p in paths:  # drop what the page cache holds of the files (best effort)
                fd = os.open(p, os.O_RDONLY)
                os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
                os.close(fd)
        with Engine(io_threads=a.io_threads, staging_bytes=a.staging_mib << 20, direct_io=mode == "direct") as e:
            best = None
            for _ in range(2):
                t0 = time.perf_counter()
                d32, st = e.file_checksums(paths)
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            bad = sum(bytes(d32[i]) != want[i] for i in range(len(paths)))
        res[mode] = {"gbps": int(sizes.sum()) / best / 1e9, "seconds": best, "mismatches": int(bad),
                     "errors": int((st != 0).sum())}
    shutil.rmtree(a.dir, ignore_errors=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
