#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X content-identification engine.

Metric (BASELINE.json): cas_id files/s + BLAKE3 GB/s hashed, per node.
Workload at N=1: config C2 — 1,000,000 synthetic files per GPU, size ~
Uniform{1024..102400} (seed 0x5D0002), so every file takes the whole-file
cas_id branch of core/src/object/cas.rs:27-29: message = le64(size) || file.
Messages are generated in HBM before timing (include/sdcas_synth.h); one
"step" = one batched cas_id pass over all of a GPU's files through the C ABI
(sdcas_dev_hash_messages: chunk scan, tile map, leaf+tree kernel, finish
kernel), keys left in HBM.

Multi-GPU (torchrun): files are sharded, rank r owns global files
[r*n, (r+1)*n) — independent units, no collective on the data path
(SURVEY.md §8e); value = all ranks' files / max-over-ranks time.

Extra fields: blake3_gbps, roofline (leaf/tree kernel, HIP events on its
stream, vs HBM peak; plus the VALU roofline the kernel is actually bound by),
cpu_baseline (rank 0, N=1: the reference's shape — one hashing thread, SIMD
BLAKE3 — on a bounded sample, via the oracle; its keys double as a parity
check of the GPU keys).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "cas_id files/sec + BLAKE3 GB/s hashed (node) at 1/2/4/8 MI355X"
SEED_C2 = 0x5D0002
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# VALU: 256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz (MI355X_MICROARCH.md: SIMD-32,
# a wave64 VALU op issues over 2 cycles) = 7.86e13 int32 ops/s
VALU_PEAK_OPS = 256 * 4 * 32 * 2.4e9
OPS_PER_COMPRESSION = 680  # 7 rounds x 8 G x 12 (add3, xor, alignbit) + 8 feed-forward xor


def mix64(x):
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def c2_files(seed, lo, hi):
    """sizes and content keys of C2 files [lo, hi) (include/sdcas_synth.h)"""
    i = np.arange(lo, hi, dtype=np.uint64)
    with np.errstate(over="ignore"):
        raw = mix64(np.uint64(seed) ^ np.uint64(0xC2C2C2C2) ^ (i << np.uint64(20)) ^ (i >> np.uint64(44)))
        sizes = np.uint64(1024) + raw % np.uint64(102400 - 1024 + 1)
        keys = mix64(np.uint64(seed) ^ (i * np.uint64(0xD1B54A32D192ED03)))
    return sizes, keys


def compressions(lens):
    n = lens.astype(np.int64)
    C = np.maximum(1, (n + 1023) // 1024)
    last = n - 1024 * (C - 1)
    return 16 * (C - 1) + np.maximum(1, (last + 63) // 64) + (C - 1)


def load_traffic(workload):
    """HBM bytes per launch of the leaf kernel from the committed rocprofv3
    PMC pass (profiles/*pmc*.json, written by tools/pmc_summarize.py), if any."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("workload") == workload and d.get("kernel", "").startswith("k_leaf_tree"):
            best = d
    return best


def cpu_baseline(gpu_keys, sample, threads):
    from tests._oracle import load_oracle
    o = load_oracle()
    f = o.lib.oracle_cpu_bench_c2
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_uint64, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                  ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int),
                  ctypes.c_char_p]
    keys = np.zeros(sample, np.uint64)
    nbytes = ctypes.c_uint64(0)
    secs = (ctypes.c_double * 2)()
    kind = ctypes.c_int(0)
    ver = ctypes.create_string_buffer(32)
    rc = f(SEED_C2, sample, threads, 1, keys.ctypes.data, ctypes.byref(nbytes), secs, ctypes.byref(kind), ver)
    if rc != 0:
        return None, None
    hasher = f"upstream BLAKE3 C {ver.value.decode()} SIMD (llvm_blake3 in ROCm libclang-cpp)" if kind.value \
        else "scalar BLAKE3 restatement (oracle/blake3_ref.c)"
    mismatches = int((keys != gpu_keys[:sample]).sum())
    base = {
        "value": sample / secs[0], "unit": "files/s", "cores": 1, "kind": "port",
        "sample": f"C2 files [0,{sample}) = {nbytes.value / 1e9:.2f} GB of cas messages in host RAM, "
                  f"hashed by the cas.rs message + {hasher}, one thread (the reference hashes a step's "
                  f"files on one runtime thread); storage I/O excluded",
        "gbps": nbytes.value / secs[0] / 1e9, "seconds": secs[0],
        "all_cores": {"value": sample / secs[1], "cores": threads, "gbps": nbytes.value / secs[1] / 1e9},
    }
    parity = {"checked_files": sample, "mismatches": mismatches, "oracle": hasher}
    return base, parity


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--files", type=int, default=1_000_000, help="files per GPU (C2: 1M)")
    ap.add_argument("--cpu-sample", type=int, default=200_000)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    if distributed:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from spacedrive_amd import Engine

    n = args.files
    lo = rank * n
    sizes, keys = c2_files(SEED_C2, lo, lo + n)
    lens = sizes + np.uint64(8)
    offs = np.zeros(n, np.uint64)
    # messages start on 128-byte lines (the L2/HBM line): a chunk then spans
    # 8 lines instead of 9 (the layout of device memory is ours to choose)
    padded = (lens + np.uint64(127)) // np.uint64(128) * np.uint64(128)
    offs[1:] = np.cumsum(padded[:-1])
    total_bytes = int(offs[-1] + padded[-1]) + 64
    chunks = int(((lens + np.uint64(1023)) // np.uint64(1024)).sum())
    msg_bytes = int(lens.sum())
    comp = int(compressions(lens).sum())

    eng = Engine(device=dev.index)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
    d_blob = torch.empty(total_bytes, dtype=torch.uint8, device=dev)
    d_keys, d_sizes, d_offs, d_lens = t(keys), t(sizes), t(offs), t(lens)
    d_out = torch.zeros(n, dtype=torch.int64, device=dev)
    eng.dev_reserve(n, chunks)
    eng.dev_synth_cas_messages(d_keys.data_ptr(), d_sizes.data_ptr(), d_offs.data_ptr(), n, d_blob.data_ptr(), sp)
    torch.cuda.synchronize()

    def step():
        eng.dev_hash_messages(d_blob.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, 0, d_out.data_ptr(), sp)

    for _ in range(args.warmup):
        step()
    eng.dev_sync(sp)
    eng.dev_profile(True)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    dt = time.perf_counter() - t0
    leaf_ms, seq_ms = eng.dev_kernel_ms()
    eng.dev_profile(False)
    eng.dev_sync(sp)
    if distributed:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        lt = torch.tensor([leaf_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(lt, op=dist.ReduceOp.MAX)
        leaf_ms = float(lt.item())

    files_total = n * world * args.steps
    value = files_total / dt
    gbps = msg_bytes * world * args.steps / dt / 1e9
    leaf_s = leaf_ms / 1e3
    achieved_gbs = msg_bytes / leaf_s / 1e9 if leaf_s > 0 else None
    traffic = load_traffic("C2")
    roof = {
        "bound": "hbm", "kernel": "k_leaf_tree (leaf chunks + in-tile tree)",
        "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": achieved_gbs / HBM_PEAK_GBS if achieved_gbs else None,
        "traffic": traffic.get("hbm_bytes_per_launch") if traffic else None,
        "algorithmic_bytes_per_launch": msg_bytes,
        "leaf_ms": leaf_ms, "sequence_ms": seq_ms,
        "valu": {
            "compressions_per_launch": comp,
            "achieved_compressions_per_s": comp / leaf_s if leaf_s > 0 else None,
            "peak_compressions_per_s": VALU_PEAK_OPS / OPS_PER_COMPRESSION,
            "frac": (comp / leaf_s) / (VALU_PEAK_OPS / OPS_PER_COMPRESSION) if leaf_s > 0 else None,
            "note": "BLAKE3 is integer ARX: ~680 VALU ops per 64-byte compression; the VALU roof "
                    "(7.4 TB/s of message bytes) sits just under the HBM roof",
        },
    }
    if traffic:
        roof["traffic_source"] = traffic.get("source")

    out = {
        "metric": METRIC, "value": value, "unit": "files/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic: C2 corpus generated in HBM (splitmix64 content per file, seed 0x5D0002)",
        "config": {"workload": "C2: 1M files x Uniform{1..100 KiB}, whole-file cas_id (cas.rs:27-29)",
                   "files_per_gpu": n, "message_bytes_per_gpu": msg_bytes, "chunks_per_gpu": chunks,
                   "parallelism": f"files sharded over {world} GPU(s), no collective"},
        "blake3_gbps": gbps, "roofline": roof,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        gk = d_out[: args.cpu_sample].cpu().numpy().view(np.uint64)
        base, parity = cpu_baseline(gk, min(args.cpu_sample, n), args.cpu_threads)
        out["cpu_baseline"] = base
        out["parity"] = parity
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
