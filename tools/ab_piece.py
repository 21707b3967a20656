#!/usr/bin/env python3
"""A/B the 1 MiB-piece kernel variants of the checksum path (config C4's
kernel) in ONE process, interleaved rounds: a resident window of synthetic
1-4 GiB files hashed through sdcas_dev_stream_*; per variant the median / min
piece-kernel ms (HIP events) and GB/s; every variant's digests must agree."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=16, help="window size (GiB of file bytes)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", default="14,15")
    ap.add_argument("--ablation", action="store_true",
                    help="bind libsdcas_ablate.so (variants 0-13: round 1/2's losing and DIAGNOSTIC kernels)")
    a = ap.parse_args()
    import torch

    from spacedrive_amd import Engine
    from spacedrive_amd import synth as S
    if a.ablation:
        from spacedrive_amd import _native as N
        N.use_ablation_library()
    MiB = 1 << 20
    sizes, keys = S.c4_files(int(a.gib) << 30)
    dev = torch.device("cuda", 0)
    offs = np.zeros(sizes.size, np.uint64)
    padded = (sizes + np.uint64(MiB - 1)) // np.uint64(MiB) * np.uint64(MiB)
    offs[1:] = np.cumsum(padded[:-1])
    total = int(offs[-1] + padded[-1]) + 4096
    blob = torch.empty(total, dtype=torch.uint8, device=dev)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x, dtype=np.uint64).view(np.int64)).to(dev)
    eng = Engine()
    z = np.zeros(sizes.size, np.uint64)
    # keep every argument tensor alive until the kernel has run (a temporary's
    # block returns to torch's cache at once and the next one may reuse it)
    args = [t(keys), t(z), t(sizes), t(offs)]
    torch.cuda.synchronize()
    eng.dev_synth_content(*(x.data_ptr() for x in args), sizes.size, blob.data_ptr())
    eng.dev_sync()
    del args
    out = torch.zeros((sizes.size, 32), dtype=torch.uint8, device=dev)
    files = np.arange(sizes.size, dtype=np.uint64)
    addrs = np.uint64(blob.data_ptr()) + offs
    vl = [int(v) for v in a.variants.split(",")]
    res = {v: [] for v in vl}
    digests = {}
    for r in range(a.rounds):
        for v in vl:
            assert eng.dev_set_piece_variant(v), v
            eng.dev_profile(True)
            for _ in range(a.reps):
                eng.dev_stream_begin(sizes)
                eng.dev_stream_update(files, z, sizes, addrs)
                eng.dev_stream_finish(out.data_ptr())
            ms, _ = eng.dev_kernel_ms()
            eng.dev_profile(False)
            eng.dev_sync()
            res[v].append(ms)
            if r == 0:
                digests[v] = out.cpu().numpy().copy()
    ref = digests[vl[0]]
    nbytes = int(sizes.sum())
    for v in vl:
        x = sorted(res[v])
        print(f"piece variant {v}: med {x[len(x) // 2]:.2f} ms min {x[0]:.2f} ms "
              f"({nbytes / x[0] / 1e6:.0f} GB/s best), agree={np.array_equal(digests[v], ref)}", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
