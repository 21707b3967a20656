#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X content-identification engine.

Metric (BASELINE.json): cas_id files/s + BLAKE3 GB/s hashed, per node.

Default workload (N=1 headline): config C2 — 1,000,000 synthetic files per
GPU, size ~ Uniform{1024..102400} (seed 0x5D0002), so every file takes the
whole-file cas_id branch of core/src/object/cas.rs:27-29: message =
le64(size) || file. Messages are generated in HBM before timing
(include/sdcas_synth.h); one "step" = one batched cas_id pass over all of a
GPU's files through the C ABI (sdcas_dev_hash_messages: chunk scan, tile map,
leaf+tree kernel, finish kernel), keys left in HBM.

Other workloads (--workload; reported the same way):
  c3  1.25M mixed files per GPU (75% whole-file log-uniform 1 B..100 KiB, 25%
      sampled 100 KiB..64 GiB, 15% duplicates); step = cas_id pass + the
      node-wide identifier dedup (spacedrive_amd.dist_dedup: combine, RCCL
      all-to-all, resolve, all-to-all back, apply)
  c5  6.25M files per GPU from the 50M Zipf-skewed corpus (60% duplicate
      files); same step as c3 — the dedup shuffle under heavy hitters

Multi-GPU (torchrun): files are sharded, rank r owns global files
[r*n, (r+1)*n) (c5: the contents of corpus files r, r+8, r+16, ... so every
GPU sees the corpus' mix; orphan ordinals r*n .. (r+1)*n-1) — independent
units for hashing (no collective), one all-to-all exchange for the c3/c5
dedup; value = all ranks' files / max-over-ranks time.

Extra fields: blake3_gbps, roofline (leaf/tree kernel, HIP events on its
stream; bound "valu": BLAKE3 is integer ARX, so achieved = compressions x
680 int32 lane-ops / kernel time against the spec VALU rate 256 CU x 4 SIMD
x 32 lanes x 2.4 GHz = 78.6 T/s; the HBM figures in roofline.hbm),
cpu_baseline (rank 0, N=1: the reference's shape — one hashing thread,
SIMD BLAKE3 — over the whole workload from RAM, via the oracle; its keys
double as a parity check of every GPU key; plus `reference_faithful`: the
identifier job's CPU shape over real files, 100-file steps in series with
cas.rs's reads, on a 200 k-file subset), e2e (c2, rank 0, N=1: the host-facing
C ABI from a pinned host buffer and from files, timed outside the on-device
loop; never `value`), parity.dedup (c3/c5 at N=1: every link and both counts
against the chunked oracle); at N > 1, parity = a sample of about 2000 files
per rank against the oracle, summed over the ranks.
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from spacedrive_amd import synth as S  # noqa: E402

METRIC = "cas_id files/sec + BLAKE3 GB/s hashed (node) at 1/2/4/8 MI355X"
SEED_C2 = S.SEED_C2
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# VALU: 256 CU x 4 SIMD-32 x 2.4 GHz (MI355X_MICROARCH.md: a wave64 VALU op
# issues over 2 cycles) = 7.86e13 int32 lane-ops/s
VALU_PEAK_OPS = 256 * 4 * 32 * 2.4e9
OPS_PER_COMPRESSION = 680  # 7 rounds x 8 G x 12 (add3, xor, alignbit) + 8 feed-forward xor
# tools/ubench_compress.hip on MI355X (profiles/r02_ubench_compress.txt): the
# best register-only compression loop (each G one asm block with s_nop 0
# after every v_alignbit_b32, the leaf kernels' B3_G_ASM) sustains 67 G
# compressions/s at 8 waves/SIMD (the compiler-scheduled G: 58.5 G/s)
VALU_ROOF_MEASURED = 67.0e9
# the VALU roofline of this instruction mix at the spec clock: one compression
# is 56 G x (2 v_add3_u32 + 4 v_alignbit_b32, 4 issue cycles each per wave64)
# + 56 G x (4 v_xor_b32 + 2 v_add_u32) + 8 feed-forward v_xor_b32 (2 cycles
# each) = 2032 SIMD cycles per 64 lanes; 1024 SIMDs x 2.4 GHz x 64 / 2032
ISSUE_CYCLES_PER_COMPRESSION = 56 * (6 * 4 + 6 * 2) + 8 * 2
VALU_PEAK_ISA = 256 * 4 * 2.4e9 * 64 / ISSUE_CYCLES_PER_COMPRESSION
TOPS_UNIT = "T int32 VALU lane-ops/s (680 per BLAKE3 compression)"

WORKLOADS = {
    "c2": dict(files=1_000_000, dedup=False,
               desc="C2: 1M files x Uniform{1..100 KiB}, whole-file cas_id (cas.rs:27-29)"),
    "c3": dict(files=1_250_000, dedup=True,
               desc="C3: 10M mixed files over 8 GPUs (1.25M/GPU): 75% whole-file 1 B..100 KiB, 25% sampled "
                    "100 KiB..64 GiB (cas.rs:30-59), 15% duplicates; cas_id + identifier dedup via RCCL all-to-all"),
    "c4": dict(files=0, dedup=False,
               desc="C4: full-file BLAKE3 (file_checksum, hash.rs:11-25) of 256 GiB of 1-4 GiB files (~102 files), "
                    "tree-parallel 1 MiB pieces streamed through resident HBM windows"),
    "c5": dict(files=6_250_000, dedup=True,
               desc="C5: 50M-file Zipf(1.1) corpus over 8 GPUs (6.25M/GPU), 60% duplicate files, bounded-Pareto "
                    "sizes 1 KiB..1 GiB; cas_id + identifier dedup via RCCL all-to-all"),
}


def c2_files(seed, lo, hi):
    """sizes and content keys of C2 files [lo, hi) (include/sdcas_synth.h)"""
    return S.c2_files(lo, hi, seed)


C5_CORPUS = 50_000_000  # 50 M files (the first 20 M distinct contents, then Zipf draws)


def c5_share(rank, n, world):
    """C5 corpus file indices of rank `rank`'s n files in a world of `world`:
    the world's n * world files sampled evenly over the whole corpus (global
    sample g -> file floor(g * 50 M / (n * world))), rank r taking samples r,
    r + world, r + 2 * world, ... So every rank's mix — 40 % first copies,
    60 % Zipf draws, the Zipf head (content 0) among them — is the corpus'
    at ANY n and world: 20 000 files per rank still carry duplicates, within
    a rank and across ranks. At n * world = 50 M (6.25 M files per GPU at
    N = 8) the sample is the corpus itself, file 8i + r, as before; a world
    asking more than the corpus takes files [0, n * world), the Zipf part
    continuing past 50 M."""
    g = np.arange(n, dtype=np.int64) * world + rank
    tot = n * world
    return g * C5_CORPUS // tot if tot < C5_CORPUS else g


def files_of(workload, rank, n, world=1):
    """(sizes, content keys, global orphan ordinals) of this rank's files"""
    if workload == "c2":
        s, k = S.c2_files(rank * n, (rank + 1) * n)
        return s, k, np.arange(rank * n, (rank + 1) * n, dtype=np.int64)
    if workload == "c3":
        s, k, _ = S.c3_files(rank * n, (rank + 1) * n)
        return s, k, np.arange(rank * n, (rank + 1) * n, dtype=np.int64)
    if workload == "c5":
        # an even sample of the corpus per rank (c5_share); the orphan
        # ordinals (the job's id order) are contiguous per rank
        fi = c5_share(rank, n, world)
        cid = S.c5_content_ids_at(fi.astype(np.uint64))
        return S.c5_sizes_of(cid), S.content_key(S.SEED_C5, cid), np.arange(rank * n, (rank + 1) * n, dtype=np.int64)
    raise ValueError(workload)


PAGE_CACHE_CLEAN = "page cache (files just written, then synced: clean pages, as files at rest)"


def settle_files():
    """write the just-written files back (os.sync) before their timed reads:
    the reads then meet clean page-cache pages, as an indexed library's files
    are, instead of racing the kernel's writeback; -> seconds it took"""
    t0 = time.perf_counter()
    os.sync()
    return time.perf_counter() - t0


def max_over_ranks(torch, dist, dev, vals):
    """element-wise max of a few floats over all ranks (on the GPU over RCCL;
    on the host for a gloo rehearsal)"""
    on_dev = dist.get_backend() == "nccl"
    t = torch.tensor(vals, dtype=torch.float64, device=dev if on_dev else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()]


def sum_over_ranks(torch, dist, dev, vals):
    """element-wise sum of a few integers over all ranks"""
    on_dev = dist.get_backend() == "nccl"
    t = torch.tensor(vals, dtype=torch.int64, device=dev if on_dev else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(x) for x in t.tolist()]


def digest_keys(dig):
    """first 8 bytes of each 32-byte digest, big-endian (the oracle's key)"""
    gk = np.zeros(dig.shape[0], np.uint64)
    for b in range(8):
        gk = (gk << np.uint64(8)) | dig[:, b].astype(np.uint64)
    return gk


def compressions(lens):
    n = lens.astype(np.int64)
    C = np.maximum(1, (n + 1023) // 1024)
    last = n - 1024 * (C - 1)
    return 16 * (C - 1) + np.maximum(1, (last + 63) // 64) + (C - 1)


# the library's default kernels (spacedrive_amd/csrc/b3_batch.hip
# kDefaultLeafVariant / kDefaultPieceVariant): the PMC traffic files are per kernel
# (a name prefix: round 4 added a last template argument, QD = 0, to the same kernel)
DEFAULT_LEAF_KERNEL = "k_leaf_tree<512, 279, 1, 1, 2, 2, 0, 1024u"
DEFAULT_PIECE_VARIANT = 19


def dedup_bytes(n, ne=0):
    """the bytes the identifier dedup must move at least: each file's 16-byte
    record (cas key + orphan ordinal) and 1-byte has-key flag read once, its
    8-byte link written once, and each existing Object's 16-byte record
    (cas key + DB index) read once; the group-by's table is the
    implementation's, not the algorithm's"""
    return 25 * int(n) + 16 * int(ne)


def load_dedup_traffic(workload, files):
    """HBM bytes per dedup call from the committed PMC passes
    (profiles/*pmc_dedup*.json, tools/pmc_dedup_summary.py), the latest
    round's for this workload and share size; None if none"""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_dedup*.json"))):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("workload") == workload.upper() and d.get("files") == files:
            best = d
    return best


def load_traffic(workload, kernel="k_leaf_tree"):
    """HBM bytes per launch of the dominant kernel from the committed
    rocprofv3 PMC passes (profiles/*pmc*.json, written by
    tools/pmc_summarize.py), the latest round's if several; None if none."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("workload") == workload.upper() and d.get("kernel", "").startswith(kernel):
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


def cpu_baseline_files(gpu_keys, sizes, ckeys, mode, threads, what):
    """CPU baseline over a bounded sample of any synthetic corpus (c3/c4/c5):
    mode 0 = cas messages (cas.rs:25-58), mode 1 = whole-file checksum
    (hash.rs:15-21). Messages are built untimed, then hashed on one thread and
    on `threads` threads by the oracle's SIMD-class hasher. The oracle keys
    (first 8 digest bytes) are compared with the GPU's on the same files."""
    from tests._oracle import load_oracle
    o = load_oracle()
    f = o.lib.oracle_cpu_bench_files
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                  ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_double),
                  ctypes.POINTER(ctypes.c_int), ctypes.c_char_p]
    sizes = np.ascontiguousarray(sizes, dtype=np.uint64)
    ckeys = np.ascontiguousarray(ckeys, dtype=np.uint64)
    n = sizes.size
    keys = np.zeros(n, np.uint64)
    nbytes = ctypes.c_uint64(0)
    secs = (ctypes.c_double * 2)()
    kind = ctypes.c_int(0)
    ver = ctypes.create_string_buffer(32)
    rc = f(ckeys.ctypes.data, sizes.ctypes.data, n, mode, threads, 1, keys.ctypes.data, ctypes.byref(nbytes),
           secs, ctypes.byref(kind), ver)
    if rc != 0:
        return None, None
    hasher = f"upstream BLAKE3 C {ver.value.decode()} SIMD (llvm_blake3 in ROCm libclang-cpp)" if kind.value \
        else "scalar BLAKE3 restatement (oracle/blake3_ref.c)"
    gb = nbytes.value / 1e9
    if mode == 1:
        base = {"value": gb / secs[0], "unit": "GB/s", "files_per_s": n / secs[0]}
        allc = {"value": gb / secs[1], "cores": threads, "files_per_s": n / secs[1]}
    else:
        base = {"value": n / secs[0], "unit": "files/s", "gbps": gb / secs[0]}
        allc = {"value": n / secs[1], "cores": threads, "gbps": gb / secs[1]}
    base.update({"cores": 1, "kind": "port", "seconds": secs[0], "all_cores": allc,
                 "sample": f"{what} = {gb:.2f} GB of {'file content' if mode else 'cas messages'} in host RAM, "
                           f"hashed by {hasher}, one thread (the reference hashes on one runtime thread per "
                           f"step); storage I/O excluded"})
    parity = {"checked_files": int(n), "mismatches": int((keys != gpu_keys).sum()), "oracle": hasher}
    return base, parity


def sample_parity(gpu_keys, sizes, ckeys, count, seed=1):
    """CPU oracle keys of `count` files spread over the batch (incl. sampled)"""
    from tests._oracle import load_oracle
    o = load_oracle()
    rng = np.random.default_rng(seed)
    idx = np.unique(np.concatenate([rng.integers(0, sizes.size, count),
                                    np.nonzero(sizes > S.MIN_FILE)[0][:count // 4]]))
    bad = sum(int(gpu_keys[i]) != o.synth_cas_key(int(ckeys[i]), int(sizes[i])) for i in idx)
    return {"checked_files": int(idx.size), "mismatches": int(bad),
            "oracle": "scalar BLAKE3 restatement over the synthetic cas message (oracle/cas_ref.c)"}


def e2e_c2(args, eng, torch, dev, d_blob, offs, lens, sizes, gpu_keys):
    """End-to-end (PCIe- and I/O-inclusive) C2 throughput of the host-facing
    C ABI on the first `--e2e-files` files, timed outside the on-device loop
    (it is never `value`):
      messages_pinned  sdcas_cas_ids_from_messages from a page-locked buffer
                       (direct DMA per staging slot)
      files            sdcas_cas_ids over the same files in the page cache
                       (cas.rs's reads by the library's I/O threads)
    and, on the same files, the reference-faithful CPU baseline: the
    identifier job's shape (100-file steps in series; per step the reads on an
    I/O pool, BLAKE3 on one thread; oracle/cpu_bench.c)."""
    import shutil
    import tempfile
    m = min(int(args.e2e_files), int(lens.size))
    msg_bytes = int(lens[:m].sum())
    end = int(offs[m - 1] + lens[m - 1])
    out = {"workload": f"C2 files [0,{m})", "files": m, "message_bytes": msg_bytes,
           "io_threads": args.cpu_threads, "staging_bytes_per_slot": 256 << 20}
    pin = torch.empty(end + 64, dtype=torch.uint8).pin_memory()
    pin.copy_(d_blob[: end + 64])
    host = pin.numpy()
    want = gpu_keys[:m]
    with type(eng)(device=dev.index, io_threads=args.cpu_threads, staging_bytes=256 << 20) as e:
        probe = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
        probe.copy_(pin[: 256 << 20], non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(4):
            probe.copy_(pin[: 256 << 20], non_blocking=True)
        torch.cuda.synchronize()
        out["pcie_h2d_pinned_gbps"] = 4 * (256 << 20) / (time.perf_counter() - t0) / 1e9
        del probe
        best, got = None, None
        for _ in range(3):
            t0 = time.perf_counter()
            got = e.cas_ids_from_messages(host, offs[:m], lens[:m])
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        out["messages_pinned"] = {"files_per_s": m / best, "gbps": msg_bytes / best / 1e9, "seconds": best,
                                  "mismatches": int((got != want).sum())}
        if args.no_faithful:
            return out
        root = tempfile.mkdtemp(prefix="sdcas_e2e_", dir=os.environ.get("TMPDIR", "/tmp"))
        try:
            paths = []
            t0 = time.perf_counter()
            for i in range(m):
                p = os.path.join(root, f"{i:07d}")
                o = int(offs[i])
                with open(p, "wb") as f:
                    f.write(host[o + 8:o + int(lens[i])])
                paths.append(p)
            out["files_written_s"] = time.perf_counter() - t0
            out["files_synced_s"] = settle_files()
            best = None
            for _ in range(2):
                t0 = time.perf_counter()
                got, st = e.generate_cas_ids(paths, sizes[:m])
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            out["files"] = {"files_per_s": m / best, "gbps": msg_bytes / best / 1e9, "seconds": best,
                            "mismatches": int((got != want).sum()), "errors": int((st != 0).sum()),
                            "storage": PAGE_CACHE_CLEAN}
            from tests._oracle import load_oracle
            keys, st, secs, hasher = load_oracle().cpu_faithful(paths, sizes[:m], 100, args.cpu_threads)
            out["reference_faithful"] = {
                "value": m / secs, "unit": "files/s", "cores": 1, "io_threads": args.cpu_threads, "kind": "port",
                "gbps": msg_bytes / secs / 1e9, "seconds": secs, "mismatches": int((keys != want).sum()),
                "errors": int((st != 0).sum()),
                "sample": f"C2 files [0,{m}) as files in the page cache: the identifier job's CPU shape — 100-file "
                          f"steps in series (job/mod.rs:559-673), per step metadata + cas.rs reads on "
                          f"{args.cpu_threads} I/O threads and {hasher} on ONE thread "
                          f"(file_identifier/mod.rs:105-147); DB writes excluded",
                "gpu_same_files_speedup": (m / out["files"]["seconds"]) / (m / secs)}
        finally:
            shutil.rmtree(root, ignore_errors=True)
    return out


def e2e_c3(args, eng, torch, dev, d_blob, offs, lens, sizes, gpu_keys):
    """End-to-end C3 from files (never `value`): the first `--e2e-files` C3
    files written to disk as SPARSE files holding only the bytes cas.rs reads
    — the whole file up to 100 KiB, else the 8 KiB header, the four 10 KiB
    samples at 8192 + k * ((size - 16384) / 4) and the 8 KiB footer
    (cas.rs:30-59) — at their full apparent sizes (up to 64 GiB), taken from
    the same cas messages the on-device loop hashes. Timed:
      files              sdcas_cas_ids (open + one read, or open + six reads at
                         the sampled offsets, by the library's I/O threads)
      reference_faithful the identifier job's CPU shape over the same files
                         (100-file steps in series, cas.rs's reads on an I/O
                         pool, BLAKE3 on ONE thread; oracle/cpu_bench.c)"""
    import shutil
    import tempfile
    from tests._oracle import load_oracle
    m = min(int(args.e2e_files), int(lens.size))
    end = int(offs[m - 1] + lens[m - 1])
    host = d_blob[:end].cpu().numpy()
    want = gpu_keys[:m]
    sampled = int((sizes[:m] > S.MIN_FILE).sum())
    out = {"workload": f"C3 files [0,{m}) ({sampled} sampled-branch files as sparse files)", "files": m,
           "message_bytes": int(lens[:m].sum()), "io_threads": args.cpu_threads}
    root = tempfile.mkdtemp(prefix="sdcas_e2e_c3_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        paths = []
        t0 = time.perf_counter()
        for i in range(m):
            p = os.path.join(root, f"{i:07d}")
            o, size = int(offs[i]), int(sizes[i])
            msg = host[o + 8:o + int(lens[i])]
            with open(p, "wb") as f:
                if size <= S.MIN_FILE:
                    f.write(msg)
                else:
                    jump = (size - 16384) // 4
                    f.truncate(size)
                    f.write(msg[:8192])
                    for k in range(4):
                        f.seek(8192 + k * jump)
                        f.write(msg[8192 + k * 10240:8192 + (k + 1) * 10240])
                    f.seek(size - 8192)
                    f.write(msg[8192 + 40960:])
            paths.append(p)
        out["files_written_s"] = time.perf_counter() - t0
        out["files_synced_s"] = settle_files()
        best = None
        for _ in range(2):
            t0 = time.perf_counter()
            got, st = eng.generate_cas_ids(paths, sizes[:m])
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        out["files"] = {"files_per_s": m / best, "seconds": best, "mismatches": int((got != want).sum()),
                        "errors": int((st != 0).sum()), "storage": PAGE_CACHE_CLEAN}
        keys, st, secs, hasher = load_oracle().cpu_faithful(paths, sizes[:m], 100, args.cpu_threads)
        out["reference_faithful"] = {
            "value": m / secs, "unit": "files/s", "cores": 1, "io_threads": args.cpu_threads, "kind": "port",
            "seconds": secs, "mismatches": int((keys != want).sum()), "errors": int((st != 0).sum()),
            "sample": f"C3 files [0,{m}) as sparse files in the page cache: the identifier job's CPU shape — "
                      f"100-file steps in series (job/mod.rs:559-673), per step metadata + cas.rs reads on "
                      f"{args.cpu_threads} I/O threads and {hasher} on ONE thread (file_identifier/mod.rs:105-147)",
            "gpu_same_files_speedup": (m / out["files"]["seconds"]) / (m / secs)}
    finally:
        shutil.rmtree(root, ignore_errors=True)
    return out


def e2e_c4(args, torch, dev, blob, sizes, win, out32, local):
    """End-to-end C4 (file_checksum, hash.rs:11-25) on a bounded sample of the
    corpus (the first whole files of the resident window up to --c4-e2e-gib),
    timed outside the on-device passes (never `value`):
      messages_pinned  sdcas_hash_messages from a page-locked host buffer
                       (the files' bytes DMA'd slot by slot, 1 MiB pieces)
      files            sdcas_checksums over the same files written to TMPDIR
                       and read back from the page cache (1 MiB pieces read in
                       parallel by the library's I/O threads)
    Digests are compared with the resident passes' out32."""
    import shutil
    import tempfile
    from spacedrive_amd import Engine
    pick, acc = [], 0
    for f, moff, ln, boff in win:
        if moff != 0 or ln != int(sizes[f]):
            continue
        if acc and acc + ln > (int(args.c4_e2e_gib) << 30):
            break
        pick.append((f, boff, ln))
        acc += ln
    if not pick:
        return None
    lens = np.array([ln for _, _, ln in pick], np.uint64)
    offs = np.zeros(len(pick), np.uint64)
    offs[1:] = np.cumsum((lens[:-1] + np.uint64(4095)) // np.uint64(4096) * np.uint64(4096))
    total = int(offs[-1] + lens[-1])
    pin = torch.empty(total + 4096, dtype=torch.uint8).pin_memory()
    for (f, boff, ln), ho in zip(pick, offs):
        pin[int(ho):int(ho) + ln].copy_(blob[boff:boff + ln])
    torch.cuda.synchronize()
    host = pin.numpy()
    want = out32.cpu().numpy()[[local[f] for f, _, _ in pick]]
    out = {"workload": f"C4 files {[f for f, _, _ in pick]} ({len(pick)} files, {acc / 2**30:.2f} GiB)",
           "files": len(pick), "bytes": acc, "io_threads": args.cpu_threads, "staging_bytes_per_slot": 256 << 20}
    with Engine(device=dev.index, io_threads=args.cpu_threads, staging_bytes=256 << 20) as e:
        best, got = None, None
        for _ in range(2):
            t0 = time.perf_counter()
            got = e.hash_messages(host, offs, lens)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        out["messages_pinned"] = {"gbps": acc / best / 1e9, "seconds": best,
                                  "mismatches": int((got != want).any(axis=1).sum())}
        del host, pin
        if args.no_faithful:
            return out
        root = tempfile.mkdtemp(prefix="sdcas_e2e_c4_", dir=os.environ.get("TMPDIR", "/tmp"))
        try:
            paths = []
            t0 = time.perf_counter()
            for f, boff, ln in pick:
                p = os.path.join(root, f"c4_{f:03d}")
                blob[boff:boff + ln].cpu().numpy().tofile(p)
                paths.append(p)
            out["files_written_s"] = time.perf_counter() - t0
            out["files_synced_s"] = settle_files()
            best = None
            for _ in range(2):
                t0 = time.perf_counter()
                got, st = e.file_checksums(paths)
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            out["files"] = {"gbps": acc / best / 1e9, "seconds": best,
                            "mismatches": int((got != want).any(axis=1).sum()), "errors": int((st != 0).sum()),
                            "storage": PAGE_CACHE_CLEAN}
        finally:
            shutil.rmtree(root, ignore_errors=True)
    return out


def c4_assign(sizes, world):
    """largest-first greedy assignment of files to ranks"""
    load = [0] * world
    own = [[] for _ in range(world)]
    for i in sorted(range(len(sizes)), key=lambda i: -int(sizes[i])):
        r = min(range(world), key=lambda r: load[r])
        own[r].append(i)
        load[r] += int(sizes[i])
    return [sorted(o) for o in own]


def c4_windows(sizes, files, window):
    """cut the rank's files into windows of <= `window` bytes of whole 1 MiB
    pieces: per window a list of (file, msg_off, len, blob_off)"""
    MiB = 1 << 20
    wins, cur, used = [], [], 0
    for f in files:
        off, size = 0, int(sizes[f])
        while off < size:
            take = min(size - off, window - used)
            if take < size - off:
                take -= take % MiB
            if take <= 0:
                wins.append(cur)
                cur, used = [], 0
                continue
            cur.append((f, off, take, used))
            used += (take + MiB - 1) // MiB * MiB
            off += take
            if used >= window:
                wins.append(cur)
                cur, used = [], 0
    if cur:
        wins.append(cur)
    return wins


def run_c4(args, torch, dist, dev, rank, world, distributed, out_f):
    """C4: file_checksum of 256 GiB of 1-4 GiB files (strong scaling: the node
    hashes the whole corpus), hashed as 1 MiB pieces.

    Split over ranks (--c4-split): `pieces` (default at N > 1) cuts the
    concatenation of all files' pieces into N equal ranges; each rank hashes
    its range and one all-reduce of the 32-byte piece nodes lets every rank
    finish every file (spacedrive_amd/dist_checksum.py); `files` assigns
    whole files largest-first (no collective, up to one file of imbalance).
    A rank's share is generated in HBM once, before the timed region, when it
    fits (the whole 256 GiB does, in one MI355X's 288 GB); value = bytes /
    max-over-ranks wall time of the timed passes. Otherwise (`files` only)
    the share is cut into windows regenerated (untimed) inside each pass and
    value = bytes / summed piece-kernel time (HIP events)."""
    from spacedrive_amd import Engine
    from spacedrive_amd.dist_checksum import checksums_split, split_pieces
    sizes, ckeys = S.c4_files(int(args.c4_total_gib) << 30)
    MiB = 1 << 20
    split = args.c4_split if args.c4_split != "auto" else ("pieces" if world > 1 else "files")
    free, _ = torch.cuda.mem_get_info(dev)
    if split == "pieces":
        segs = split_pieces(sizes, world)[rank]
        need = int(sum((ln + MiB - 1) // MiB * MiB for _, _, ln in segs))
        assert need + (6 << 30) < free, "the rank's piece range must be resident in HBM"
        mine = sorted({f for f, _, _ in segs})
        window, wins = need, None
    else:
        mine = c4_assign(sizes, world)[rank]
        need = int(sum((int(sizes[f]) + MiB - 1) // MiB * MiB for f in mine))
        if args.window_gib > 0:
            window = int(args.window_gib) << 30
        else:
            window = need if need + (6 << 30) < free else 64 << 30
        wins = c4_windows(sizes, mine, window)
        segs = None
    resident = split == "pieces" or len(wins) == 1
    eng = Engine(device=dev.index)
    if args.piece_variant >= 0:
        assert eng.dev_set_piece_variant(args.piece_variant), args.piece_variant
    s = torch.cuda.Stream(dev)
    sp = s.cuda_stream
    blob = torch.empty(window + (2 << 20), dtype=torch.uint8, device=dev)
    base = blob.data_ptr()
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)
    if split == "pieces":
        offs, pos = [], 0
        for _, _, ln in segs:
            offs.append(pos)
            pos += (ln + MiB - 1) // MiB * MiB
        f = np.array([x[0] for x in segs], np.uint64)
        gen = [dict(keys=t(ckeys[f]), starts=t([x[1] for x in segs]), lens=t([x[2] for x in segs]), offs=t(offs))]
        addrs = [base + o for o in offs]
        out32 = torch.zeros((sizes.size, 32), dtype=torch.uint8, device=dev)
        my_bytes = int(sum(ln for _, _, ln in segs))
        local = {f: f for f in range(sizes.size)}
        launches = 1
    else:
        out32 = torch.zeros((max(len(mine), 1), 32), dtype=torch.uint8, device=dev)
        local = {f: k for k, f in enumerate(mine)}
        gen = []
        for w in wins:
            f = np.array([x[0] for x in w], np.uint64)
            gen.append(dict(
                keys=t(ckeys[f]), starts=t([x[1] for x in w]), lens=t([x[2] for x in w]), offs=t([x[3] for x in w]),
                seg=(np.array([local[x[0]] for x in w], np.uint64), np.array([x[1] for x in w], np.uint64),
                     np.array([x[2] for x in w], np.uint64), np.array([base + x[3] for x in w], np.uint64))))
        my_bytes = int(sum(int(sizes[f]) for f in mine))
        launches = len(gen)

    def generate(a):
        eng.dev_synth_content(a["keys"].data_ptr(), a["starts"].data_ptr(), a["lens"].data_ptr(),
                              a["offs"].data_ptr(), a["keys"].numel(), base, sp)

    def one_pass():
        if split == "pieces":
            checksums_split(eng, sizes, segs, addrs, out32)
            return
        eng.dev_stream_begin(sizes[mine])
        for a in gen:
            if not resident:
                generate(a)
            eng.dev_stream_update(*a["seg"], stream=sp)
        eng.dev_stream_finish(out32.data_ptr(), sp)

    torch.cuda.synchronize()  # the argument tensors are on the device before the side stream reads them
    if resident:
        generate(gen[0])
    eng.dev_sync(sp)

    for _ in range(args.warmup):
        one_pass()
    eng.dev_sync(sp)
    torch.cuda.synchronize()
    eng.dev_profile(True)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_pass()
    eng.dev_sync(sp)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    wall = time.perf_counter() - t0
    mean_ms, _ = eng.dev_kernel_ms()
    eng.dev_profile(False)
    hash_s = mean_ms / 1e3 * launches * args.steps
    if distributed:
        hash_s, wall = max_over_ranks(torch, dist, dev, [hash_s, wall])
    total = int(sizes.sum()) * args.steps
    comp = int(sum(int(compressions(np.array([x], np.uint64))[0]) for x in sizes)) * args.steps
    timed = wall if resident else hash_s
    gbs = total / timed / 1e9
    out = {
        "metric": METRIC, "value": gbs, "unit": "GB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": timed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic: C4 corpus (seed 0x5D0004) generated in HBM " +
                ("once, before the timed region" if resident else "window by window (untimed)"),
        "config": {"workload": WORKLOADS["c4"]["desc"], "files": int(sizes.size), "bytes": int(sizes.sum()),
                   "window_bytes": window, "launches_per_pass_rank0": launches, "resident": resident,
                   "split": split,
                   "parallelism": (f"files' 1 MiB pieces split evenly over {world} GPU(s), one all-reduce of "
                                   f"the 32-byte piece nodes" if split == "pieces" else
                                   f"files assigned largest-first over {world} GPU(s), no collective")},
        "timing": "wall time of the timed passes (max over ranks)" if resident else
                  "summed piece-kernel time (HIP events; the windows are regenerated between launches)",
        "blake3_gbps": gbs,
        "hash_kernel_gbps": total / hash_s / 1e9 if hash_s > 0 else None,
        "roofline": {
            "bound": "valu", "kernel": ("k_piece_l4 + k_piece_top (1 MiB pieces -> level-4 nodes -> level-10 nodes)"
                                   if (DEFAULT_PIECE_VARIANT if args.piece_variant < 0 else args.piece_variant) == 19
                                   else "k_piece_tree (1 MiB pieces -> level-10 nodes)"),
            "achieved": comp / hash_s / world * OPS_PER_COMPRESSION / 1e12 if hash_s > 0 else None,
            "peak": VALU_PEAK_OPS / 1e12, "unit": TOPS_UNIT,
            "traffic": None, "algorithmic_bytes_per_launch": my_bytes,
            "compressions_per_launch": comp // args.steps,
            "hbm": {"achieved": my_bytes * args.steps / (hash_s) / 1e9 if hash_s > 0 else None, "peak": HBM_PEAK_GBS,
                    "unit": "GB/s"},
            "valu": {"compressions_per_s_node": comp / hash_s,
                     "peak_compressions_per_s_spec": VALU_PEAK_OPS / OPS_PER_COMPRESSION,
                     "frac_of_spec_per_gpu": comp / hash_s / world / (VALU_PEAK_OPS / OPS_PER_COMPRESSION),
                     "peak_compressions_per_s_isa": VALU_PEAK_ISA,
                     "frac_of_isa_peak_per_gpu": comp / hash_s / world / VALU_PEAK_ISA,
                     "roof_compressions_per_s_measured": VALU_ROOF_MEASURED,
                     "frac_of_measured_roof_per_gpu": comp / hash_s / world / VALU_ROOF_MEASURED},
        },
        "parity": {"note": "digests of the streamed path are checked bit-exactly against the oracle in "
                           "tests/test_gpu_stream.py (multi-piece messages up to 4 GiB + 1) and the split "
                           "path in tests/test_gpu_multiproc.py"},
    }
    out["roofline"]["frac"] = out["roofline"]["achieved"] / (VALU_PEAK_OPS / 1e12) if out["roofline"]["achieved"] \
        else None
    hb = out["roofline"]["hbm"]
    hb["frac"] = hb["achieved"] / HBM_PEAK_GBS if hb["achieved"] else None
    # PMC traffic of the kernel this run launched (the default piece kernel
    # unless --piece-variant chose another)
    piece_kernels = {17: "k_piece_tree<259, 6, 1, 0, 10>", 19: "k_piece_l4<259, 6>"}
    pv = DEFAULT_PIECE_VARIANT if args.piece_variant < 0 else args.piece_variant
    tr = load_traffic("c4", piece_kernels[pv]) if pv in piece_kernels else None
    if tr and resident and tr.get("algorithmic_bytes_per_launch") == my_bytes:
        out["roofline"]["traffic"] = tr["hbm_bytes_per_launch"]
        out["roofline"]["traffic_source"] = tr.get("source")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # bounded sample: the first files (in corpus order) up to c4_cpu_gib
        pick, acc = [], 0
        for f in mine:
            if acc >= int(args.c4_cpu_gib) << 30:
                break
            pick.append(f)
            acc += int(sizes[f])
        gk = digest_keys(out32.cpu().numpy()[[local[f] for f in pick]])
        base, parity = cpu_baseline_files(gk, sizes[pick], ckeys[pick], 1, args.cpu_threads,
                                          f"C4 files {pick[0]}..{pick[-1]} ({len(pick)} files)")
        out["cpu_baseline"] = base
        out["parity"]["cpu_baseline_sample"] = parity
    elif distributed:
        # every rank checks the smallest file it holds a digest of (with the
        # piece split: every file, through the all-reduce) against the oracle
        cand = list(range(sizes.size)) if split == "pieces" else list(mine)
        checked = bad = 0
        if cand:
            f = min(cand, key=lambda x: int(sizes[x]))
            gk = digest_keys(out32.cpu().numpy()[[local[f]]])
            _, p = cpu_baseline_files(gk, sizes[[f]], ckeys[[f]], 1, 4, f"C4 file {f}")
            checked, bad = 1, (p["mismatches"] if p else 1)
        checked, bad = sum_over_ranks(torch, dist, dev, [checked, bad])
        out["parity"].update({"checked_files": checked, "mismatches": bad, "ranks": world,
                              "sample": "each rank: its smallest file, whole-file checksum vs the oracle"})
    if rank == 0 and world == 1 and resident and split == "files" and not args.no_e2e:
        out["e2e"] = e2e_c4(args, torch, dev, blob, sizes, wins[0], out32, local)
    if args.c4_full_parity:
        # every file this rank holds a digest of, against the oracle's
        # checksum of the same synthetic content (scalar restatement, one
        # file per thread; ctypes releases the GIL)
        from concurrent.futures import ThreadPoolExecutor
        from tests._oracle import load_oracle
        o = load_oracle()
        # with the piece split every rank holds every digest: rank r checks files r, r + N, ...
        cand = [f for f in range(sizes.size) if f % world == rank] if split == "pieces" else list(mine)
        dig = out32.cpu().numpy()
        with ThreadPoolExecutor(max(1, args.cpu_threads)) as ex:
            want = list(ex.map(lambda f: o.synth_checksum(int(ckeys[f]), int(sizes[f])), cand))
        bad = sum(bytes(dig[local[f]]).hex() != w for f, w in zip(cand, want))
        nbytes = int(sum(int(sizes[f]) for f in cand))
        checked, bad, nbytes = (sum_over_ranks(torch, dist, dev, [len(cand), bad, nbytes]) if distributed
                                else (len(cand), bad, nbytes))
        out["parity"]["all_files"] = {"checked_files": checked, "mismatches": bad, "bytes": nbytes,
                                      "oracle": "scalar BLAKE3 restatement of each file's synthetic content "
                                                "(oracle/cas_ref.c oracle_synth_checksum)"}
    if rank == 0:
        emit(out_f, out)
    eng.close()


def _json_stdout():
    """The contract's ONE JSON line goes to the process's stdout; everything
    else that C libraries print there (RCCL's version banner at communicator
    setup) is moved to stderr: fd 1 becomes a copy of fd 2, and the JSON is
    written to the saved original."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(saved, "w")


def emit(out_f, obj):
    out_f.write(json.dumps(obj) + "\n")
    out_f.flush()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv, script=None):
    """`bench.py --gpus N` started without a launcher (no WORLD_SIZE in the
    environment): start N rank processes of this same script, one per GPU,
    with the torchrun environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_*),
    and return the worst exit status. This parent never touches the GPU (it
    has not imported torch); rank 0's JSON line reaches stdout through the
    inherited descriptor. If a rank fails, the others are stopped."""
    import signal
    import subprocess
    env = dict(os.environ, WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=os.environ.get("MASTER_PORT") or str(_free_port()))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = []
    for r in range(n):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r), GROUP_RANK="0")
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + argv, env=e))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    old = {s: signal.signal(s, lambda sig, fr: (stop(), sys.exit(128 + sig))) for s in (signal.SIGTERM, signal.SIGINT)}
    worst = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                rc = p.poll()
                if rc is None:
                    continue
                live.remove(p)
                if rc != 0:
                    worst = worst or (rc if rc > 0 else 128 - rc)
                    print(f"bench.py: rank {procs.index(p)} exited with {rc}; stopping the other ranks",
                          file=sys.stderr)
                    stop()
            time.sleep(0.05)
        for p in procs:
            p.wait(timeout=60)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    return worst


def check_world(gpus, env):
    """The launch must agree with --gpus: None when this process is a rank of
    an N = --gpus job (or the one process of N = 1), 'spawn' when bench.py
    must start the ranks itself, else the error to exit with."""
    ws = env.get("WORLD_SIZE")
    if gpus < 1:
        return f"--gpus must be >= 1 (got {gpus})"
    if ws is None:
        return "spawn" if gpus > 1 else None
    if int(ws) != gpus:
        return f"--gpus {gpus} but WORLD_SIZE={ws}: the launch and the flag disagree"
    return None


def main():
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=1)
    known, _ = pre.parse_known_args()
    how = check_world(known.gpus, os.environ)
    if how == "spawn":
        sys.exit(launch_ranks(known.gpus, sys.argv[1:]))
    if how is not None:
        print(f"bench.py: {how}", file=sys.stderr)
        sys.exit(2)
    out_f = _json_stdout()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--files", type=int, default=0, help="files per GPU (default: the workload's)")
    ap.add_argument("--cpu-sample", type=int, default=0, help="files in the CPU-baseline sample (0: all of rank 0's)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--c4-total-gib", type=int, default=256)
    ap.add_argument("--window-gib", type=int, default=0, help="c4: HBM window (0: the whole share when it fits)")
    ap.add_argument("--c4-cpu-gib", type=int, default=16, help="C4 CPU-baseline sample size")
    ap.add_argument("--c4-e2e-gib", type=int, default=8, help="C4 end-to-end sample size (pinned buffer, files)")
    ap.add_argument("--msg-align", type=int, default=128, choices=[16, 32, 64, 128],
                    help="c2/c3/c5: byte alignment of each message in HBM")
    ap.add_argument("--e2e-files", type=int, default=200_000, help="c2: files in the end-to-end / faithful leg")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--sustain-s", type=float, default=6.0,
                    help="after the timed steps, the same steps back to back for this long (untimed by the "
                         "contract; reported as `sustained`): the rate the card holds at its power limit, and "
                         "a window long enough for a GPU-busy sampler to see (0: skip)")
    ap.add_argument("--no-bind-stream", action="store_true",
                    help="A/B: leave the step's stream unbound (every device call then waits on the previous "
                         "call's event even on the same stream, sdcas_dev_bind_stream)")
    ap.add_argument("--no-faithful", action="store_true", help="e2e without the page-cache files legs")
    ap.add_argument("--piece-variant", type=int, default=-1, help="c4: piece kernel variant (-1 default)")
    ap.add_argument("--c4-full-parity", action="store_true",
                    help="c4: check every file's checksum against the oracle (16 CPU threads, about a minute)")
    ap.add_argument("--c4-split", default="auto", choices=["auto", "pieces", "files"],
                    help="c4 over N GPUs: split the files' pieces (auto at N > 1) or assign whole files")
    args = ap.parse_args()
    W = WORKLOADS[args.workload]

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    # one rank per GPU; the modulo only matters for a rehearsal of the N > 1
    # path with more ranks than GPUs (SDCAS_BENCH_BACKEND=gloo: RCCL refuses
    # two ranks on one device), never on a node with a GPU per rank
    torch.cuda.set_device((local % torch.cuda.device_count()) if distributed else 0)
    dev = torch.device("cuda", torch.cuda.current_device())
    backend = os.environ.get("SDCAS_BENCH_BACKEND", "nccl")
    if distributed:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    elif W["dedup"]:
        # the dedup driver is collective code: a world of one over RCCL
        dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)

    if args.workload == "c4":
        run_c4(args, torch, dist, dev, rank, world, distributed, out_f)
        if dist.is_initialized():
            dist.destroy_process_group()
        return

    from spacedrive_amd import Engine
    from spacedrive_amd.dist_dedup import DeviceStages, identifier_dedup_distributed

    n = args.files or W["files"]
    sizes, keys, ids = files_of(args.workload, rank, n, world)
    lens = S.cas_msg_len(sizes)
    offs = np.zeros(n, np.uint64)
    # messages start on 128-byte lines (the L2/HBM line): a chunk then spans
    # 8 lines instead of 9 (the layout of device memory is ours to choose);
    # --msg-align 16 packs them at the ABI's minimum instead (A/B)
    al = np.uint64(args.msg_align)
    padded = (lens + al - np.uint64(1)) // al * al
    offs[1:] = np.cumsum(padded[:-1])
    total_bytes = int(offs[-1] + padded[-1]) + 64
    chunks = int(np.maximum(np.uint64(1), (lens + np.uint64(1023)) // np.uint64(1024)).sum())
    msg_bytes = int(lens.sum())
    comp = int(compressions(lens).sum())

    eng = Engine(device=dev.index)
    # one real stream for the whole run: torch's default stream is the legacy
    # NULL stream (handle 0), which the library reads as "the context's own
    # stream" — the hash would then run unordered with the events recorded
    # here, and the dedup's HIP-event span would swallow the hash
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    assert sp != 0
    if not args.no_bind_stream:
        eng.dev_bind_stream(sp)  # consecutive calls on it (hash, dedup) skip the scratch fence's event wait
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
    d_blob = torch.empty(total_bytes, dtype=torch.uint8, device=dev)
    d_keys, d_sizes, d_offs, d_lens = t(keys), t(sizes), t(offs), t(lens)
    d_out = torch.zeros(n, dtype=torch.int64, device=dev)
    eng.dev_reserve(n, chunks)
    eng.dev_synth_cas_messages(d_keys.data_ptr(), d_sizes.data_ptr(), d_offs.data_ptr(), n, d_blob.data_ptr(), sp)
    torch.cuda.synchronize()

    dd = None
    if W["dedup"]:
        d_has = (d_sizes != 0).to(torch.uint8)  # mod.rs:78-86: empty files have no cas_id
        d_ids = torch.from_numpy(ids).to(dev)
        # the dedup's stages on the step's own stream (no cross-stream waits)
        stages = DeviceStages(eng, dev.index, same_stream=True)
        dd = {}

    def dedup_call():
        # a world of one leaves the counts on the device (read after the
        # timed steps): the call enqueues without a host wait
        return identifier_dedup_distributed(stages, d_out, d_has, None, d_ids, 100, counts_on_device=not distributed)

    def step():
        eng.dev_hash_messages(d_blob.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, 0, d_out.data_ptr(), sp)
        if dd is not None:
            # the dedup's stages are ordered after the hash on the stream (no
            # host wait in between, no event: one would idle the GPU ~6-8 us)
            dd["last"] = dedup_call()

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
        dt, leaf_ms, seq_ms = max_over_ranks(torch, dist, dev, [dt, leaf_ms, seq_ms])
    sustained = None
    if args.sustain_s > 0:
        # the same steps for a few seconds more, outside the timed region: the
        # steady-state rate (clock and power settled); the count follows from
        # the timed steps' max-over-ranks time, so every rank runs as many
        k = max(16, int(math.ceil(args.sustain_s / (dt / args.steps))))
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(k):
            step()
        torch.cuda.synchronize()
        st = time.perf_counter() - t1
        if distributed:
            st = max_over_ranks(torch, dist, dev, [st])[0]
        sustained = {"steps": k, "seconds": st, "value": n * world * k / st, "ms_per_step": st / k * 1e3,
                     "note": "the timed steps' workload repeated back to back after them, untimed by the "
                             "contract (not part of `value`)"}
    if dd is not None:
        # the dedup's share of a step: the same calls on the same resident
        # inputs, `steps` of them back to back between one pair of HIP events
        # (and, at N > 1, the exchange's own events), after the timed steps
        stages.time_exchange = distributed
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.steps):
            dd["last"] = dedup_call()
        e1.record(stream)
        torch.cuda.synchronize()
        dd["ms"] = e0.elapsed_time(e1) / args.steps

    files_total = n * world * args.steps
    value = files_total / dt
    gbps = msg_bytes * world * args.steps / dt / 1e9
    leaf_s = leaf_ms / 1e3
    achieved_gbs = msg_bytes / leaf_s / 1e9 if leaf_s > 0 else None
    traffic = load_traffic(args.workload, DEFAULT_LEAF_KERNEL)
    valu_rate = comp / leaf_s if leaf_s > 0 else None
    tops = valu_rate * OPS_PER_COMPRESSION / 1e12 if valu_rate else None
    roof = {
        # the binding roof: BLAKE3 is integer ARX, so the dominant kernel is
        # priced in VALU lane-ops (680 per compression) against the spec rate
        "bound": "valu", "kernel": "k_leaf_tree (leaf chunks + in-tile tree)",
        "achieved": tops, "peak": VALU_PEAK_OPS / 1e12, "unit": TOPS_UNIT,
        "frac": tops / (VALU_PEAK_OPS / 1e12) if tops else None,
        "traffic": traffic.get("hbm_bytes_per_launch") if traffic else None,
        "algorithmic_bytes_per_launch": msg_bytes, "compressions_per_launch": comp,
        "leaf_ms": leaf_ms, "sequence_ms": seq_ms,
        "hbm": {"achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS if achieved_gbs else None},
        "valu": {
            "compressions_per_launch": comp,
            "achieved_compressions_per_s": valu_rate,
            "peak_compressions_per_s_spec": VALU_PEAK_OPS / OPS_PER_COMPRESSION,
            "frac_of_spec": valu_rate / (VALU_PEAK_OPS / OPS_PER_COMPRESSION) if valu_rate else None,
            "peak_compressions_per_s_isa": VALU_PEAK_ISA,
            "frac_of_isa_peak": valu_rate / VALU_PEAK_ISA if valu_rate else None,
            "roof_compressions_per_s_measured": VALU_ROOF_MEASURED,
            "frac_of_measured_roof": valu_rate / VALU_ROOF_MEASURED if valu_rate else None,
            "note": "BLAKE3 is integer ARX (no MFMA): the kernel is VALU-bound (and power-held: it runs at "
                    "~1.9 GHz), not HBM-bound. spec peak = 680 ops/compression as if every op issued at the "
                    "full VALU lane rate at 2.4 GHz; isa peak = round 1's issue model of the same 680 "
                    "instructions (VOP3 4 cycles, VOP2 2 cycles per wave64) at 2.4 GHz, an upper bound; "
                    "measured roof = the best register-only compression loop (asm G blocks, "
                    "tools/ubench_compress.hip, 67 G/s)",
        },
    }
    if traffic:
        roof["traffic_source"] = traffic.get("source")

    out = {
        "metric": METRIC, "value": value, "unit": "files/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": f"synthetic: {args.workload.upper()} corpus generated in HBM (splitmix64 content per file, "
                f"include/sdcas_synth.h, spacedrive_amd/synth.py)",
        "config": {"workload": W["desc"], "files_per_gpu": n, "message_bytes_per_gpu": msg_bytes,
                   "chunks_per_gpu": chunks,
                   "parallelism": f"files sharded over {world} GPU(s)" +
                                  (", dedup: one RCCL all-to-all exchange" if W["dedup"] else ", no collective")},
        "blake3_gbps": gbps, "roofline": roof, "sustained": sustained,
    }
    if dd is not None:
        ms = med = float(dd["ms"])
        if distributed:
            ms, med = max_over_ranks(torch, dist, dev, [ms, med])
        last = dd["last"]
        if len(last) == 2:  # (link, counts on the device)
            c = last[1].tolist()
            last = (last[0], int(c[0]), int(c[1]))
            dd["last"] = last
        _, created, linked = last
        out["dedup"] = {"ms_per_step": ms, "ms_median": med, "objects_created": created, "files_linked": linked,
                        "records_per_gpu": n, "protocol": getattr(stages, "last_protocol", None),
                        "timing": "HIP events around `steps` back-to-back dedup calls on the step's stream, "
                                  "after the timed steps, on the same resident inputs (an event pair inside "
                                  "every step would idle the GPU ~6-8 us per event); ms_median = ms_per_step"}
        # the dedup is HBM-bound; priced on the bytes it must
        # move (dedup_bytes) over its time, the PMC-measured bytes beside them
        algo = dedup_bytes(n)
        dr = {"bound": "hbm", "achieved": algo / med / 1e6, "peak": HBM_PEAK_GBS, "unit": "GB/s",
              "frac": algo / med / 1e6 / HBM_PEAK_GBS, "algorithmic_bytes_per_step": algo,
              "algorithmic": "25 B per file (16-B record in, 1-B has-key flag in, 8-B link out)",
              "traffic": None}
        tr = load_dedup_traffic(args.workload, n) if world == 1 else None
        if tr:
            dr["traffic"] = tr["hbm_bytes_per_call"]
            dr["traffic_over_algorithmic"] = tr["hbm_bytes_per_call"] / algo
            dr["traffic_gbps"] = tr["hbm_bytes_per_call"] / med / 1e6
            dr["traffic_frac"] = dr["traffic_gbps"] / HBM_PEAK_GBS
            dr["traffic_source"] = tr.get("source")
        out["dedup"]["roofline"] = dr
        xs = getattr(stages, "last_exchange", None)
        if xs is not None:
            # the exchange (RCCL all-to-alls) of the last step: bytes this
            # rank sent and the HIP-event time of its collectives
            xms = sum(a.elapsed_time(b) for a, b in xs["events"])
            xb, xoff, xms = max_over_ranks(torch, dist, dev, [xs["bytes"], xs["bytes_off_rank"], xms])
            out["dedup"]["exchange"] = {"bytes_per_rank": xb, "bytes_off_rank": xoff, "ms": xms,
                                        "gbps_off_rank": xoff / xms / 1e6 if xms > 0 else None,
                                        "timing": "HIP events around the all-to-alls on the step's stream, "
                                                  "max over ranks",
                                        "link_peak_gbps_per_peer": 153.6}
    if rank == 0 and world == 1:
        gk = d_out.cpu().numpy().view(np.uint64)
        if args.workload == "c2" and not args.no_cpu_baseline:
            base, parity = cpu_baseline(gk, min(args.cpu_sample or n, n), args.cpu_threads)
            out["cpu_baseline"] = base
            out["parity"] = parity
        elif not args.no_cpu_baseline:
            m = min(args.cpu_sample or n, n)
            base, parity = cpu_baseline_files(gk[:m], sizes[:m], keys[:m], 0, args.cpu_threads,
                                              f"{args.workload.upper()} files [0,{m}) of rank 0")
            out["cpu_baseline"] = base
            out["parity"] = parity
        else:
            out["parity"] = sample_parity(gk, sizes, keys, 2000)
        if dd is not None:
            from tests._oracle import load_oracle
            link = dd["last"][0].cpu().numpy()
            # the oracle walks ordinals 0..n-1 in chunks of 100 (rank 0's
            # ordinals at N = 1), over the GPU's keys (checked above)
            want, wc, wl = load_oracle().identifier_dedup(gk, (sizes != 0).astype(np.uint8), None, 100)
            out["parity"]["dedup"] = {"files": n, "link_mismatches": int((link != want).sum()),
                                      "counts_match": (wc, wl) == (dd["last"][1], dd["last"][2]),
                                      "oracle": "chunked restatement of file_identifier/mod.rs:149-254 "
                                                "(oracle/cas_ref.c)"}
        if args.workload == "c3" and not args.no_e2e:
            out["e2e"] = e2e_c3(args, eng, torch, dev, d_blob, offs, lens, sizes, gk)
        if args.workload == "c2" and not args.no_e2e:
            out["e2e"] = e2e_c2(args, eng, torch, dev, d_blob, offs, lens, sizes, gk)
            if "cpu_baseline" in out and out["e2e"].get("reference_faithful"):
                out["cpu_baseline"]["reference_faithful"] = out["e2e"].pop("reference_faithful")
    elif distributed:
        # every rank checks a sample of its own files against the oracle (the
        # full checks above need the whole corpus on one host: N = 1 only)
        gk = d_out.cpu().numpy().view(np.uint64)
        p = sample_parity(gk, sizes, keys, 2000, seed=1 + rank)
        checked, bad = sum_over_ranks(torch, dist, dev, [p["checked_files"], p["mismatches"]])
        out["parity"] = {"checked_files": checked, "mismatches": bad, "ranks": world,
                         "sample": "about 2000 files per rank (incl. sampled-branch files)", "oracle": p["oracle"]}
        if dd is not None:
            # the exchange's result over the whole job: every rank's keys and
            # links (global ordinals rank * n + i) to rank 0, checked against
            # the chunked oracle over the concatenated corpus
            on_dev = dist.get_backend() == "nccl"
            loc = lambda t: t if on_dev else t.cpu()
            parts = [loc(torch.empty(2 * n, dtype=torch.int64, device=dev)) for _ in range(world)]
            dist.all_gather(parts, loc(torch.cat([d_out, dd["last"][0]])))
            if rank == 0:
                from tests._oracle import load_oracle
                allk = np.concatenate([x.cpu().numpy()[:n] for x in parts]).view(np.uint64)
                alll = np.concatenate([x.cpu().numpy()[n:] for x in parts])
                has = np.concatenate([(files_of(args.workload, r, n, world)[0] != 0) for r in range(world)]).astype(np.uint8)
                want, wc, wl = load_oracle().identifier_dedup(allk, has, None, 100)
                out["parity"]["dedup"] = {"files": int(alll.size), "link_mismatches": int((alll != want).sum()),
                                          "counts_match": (wc, wl) == (dd["last"][1], dd["last"][2]),
                                          "oracle": "chunked restatement of file_identifier/mod.rs:149-254 over "
                                                    "all ranks' files (oracle/cas_ref.c)"}
    if rank == 0:
        emit(out_f, out)
    eng.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
