#!/usr/bin/env python3
"""A/B the leaf/tree kernel variants on the C2 workload, interleaved rounds in
ONE process (cdna_hip_programming.md §5.4 rule 24). Prints per-variant median
and min leaf-kernel ms (HIP events) and checks all variants agree bit-exactly.

Binds the ablation library (libsdcas_ablate.so: `make -C spacedrive_amd/csrc
ablate`), which holds every variant of round 1's A/B runs, the DIAGNOSTIC ones
(wrong digests) included; --product binds libsdcas.so (product variants only)."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=1_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="")
    ap.add_argument("--align", type=int, default=128, help="message start alignment in HBM")
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "c5"])
    ap.add_argument("--sorts", default="1", help="comma list of slot orders to try: 1 length-sorted, 0 caller order")
    ap.add_argument("--product", action="store_true", help="bind libsdcas.so instead of the ablation library")
    a = ap.parse_args()
    import torch
    from spacedrive_amd import Engine
    from spacedrive_amd import _native as N
    if not a.product:
        N.use_ablation_library()
    dev = torch.device("cuda", 0)
    n = a.files
    sizes, keys, _ = bench.files_of(a.workload, 0, n)
    lens = bench.S.cas_msg_len(sizes)
    A = np.uint64(a.align)
    padded = (lens + A - np.uint64(1)) // A * A
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(padded[:-1])
    total = int(offs[-1] + padded[-1]) + 64 + (1 << 17)  # + 128 KiB: diagnostic 57 reads 64 KiB past a wave base
    chunks = int(np.maximum(np.uint64(1), (lens + np.uint64(1023)) // np.uint64(1024)).sum())
    eng = Engine()
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).to(dev)
    d_blob = torch.empty(total, dtype=torch.uint8, device=dev)
    dk, ds, do, dl = t(keys), t(sizes), t(offs), t(lens)
    eng.dev_reserve(n, chunks)
    sp = torch.cuda.current_stream().cuda_stream
    eng.dev_synth_cas_messages(dk.data_ptr(), ds.data_ptr(), do.data_ptr(), n, d_blob.data_ptr(), sp)
    vl = [int(v) for v in a.variants.split(",")] if a.variants else [v for v in range(64) if eng.dev_set_leaf_variant(v)]
    for v in vl:
        assert eng.dev_set_leaf_variant(v), f"variant {v} is not in {N.ABLATION_LIB_PATH if not a.product else N.LIB_PATH}"
    vs = [(v, int(so)) for v in vl for so in a.sorts.split(",")]
    outs = {}
    res = {v: [] for v in vs}
    for r in range(a.rounds):
        for v in vs:
            eng.dev_set_leaf_variant(v[0])
            eng.dev_set_sort(v[1])
            out = torch.zeros(n, dtype=torch.int64, device=dev)
            eng.dev_hash_messages(d_blob.data_ptr(), do.data_ptr(), dl.data_ptr(), n, 0, out.data_ptr(), sp)
            eng.dev_sync(sp)
            eng.dev_profile(True)
            for _ in range(a.reps):
                eng.dev_hash_messages(d_blob.data_ptr(), do.data_ptr(), dl.data_ptr(), n, 0, out.data_ptr(), sp)
            leaf, seq = eng.dev_kernel_ms()
            eng.dev_profile(False)
            res[v].append((leaf, seq))
            if r == 0:
                outs[v] = out.cpu().numpy()
    ref = outs[vs[0]]
    msg = int(lens.sum())
    for v in vs:
        leafs = sorted(x[0] for x in res[v])
        seqs = sorted(x[1] for x in res[v])
        same = np.array_equal(outs[v], ref)
        print(f"variant {v[0]} sort {v[1]}: leaf med {leafs[len(leafs)//2]:.3f} min {leafs[0]:.3f} ms "
              f"({msg / leafs[0] / 1e6:.0f} GB/s), seq med {seqs[len(seqs)//2]:.3f} ms, agree={same}",
              flush=True)
    eng.close()


if __name__ == "__main__":
    main()
