"""file_checksum (core/src/object/validation/hash.rs:11-25) of big files whose
1 MiB pieces are split over the GPUs of a node (a file larger
than one GPU's share; config C4 at N > 1).

BLAKE3's tree makes every full 1 MiB piece of a file a node of its tree (a
level-10 subtree at chunk counter 1024 q), independent of every other piece.
So the concatenation of all files' pieces is cut into `world` contiguous
ranges of equal piece counts; every rank hashes its range into the session's
node list (sdcas_dev_stream_update), the lists — zero where a rank hashed
nothing — are summed by one all-reduce (32 B per piece: 8 MB for C4's
256 GiB), and every rank merges the complete lists into the roots
(sdcas_dev_stream_finish). One collective per batch, no data moves between
GPUs. Whole-file assignment (bench.py's `files` split) needs no collective
but leaves up to one file of imbalance; the piece split balances to one piece.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

MiB = 1 << 20


def split_pieces(sizes, world):
    """-> per rank a list of segments (file, msg_off, length) covering a
    contiguous range of the files' pieces (file order, then piece order),
    every rank within one piece of sizes' total pieces / world"""
    sizes = [int(s) for s in sizes]
    npc = [(s + MiB - 1) // MiB for s in sizes]
    total = sum(npc)
    cuts = [total * r // world for r in range(world + 1)]
    out = [[] for _ in range(world)]
    base = 0  # global index of the file's first piece
    for f, (s, n) in enumerate(zip(sizes, npc)):
        for r in range(world):
            lo, hi = max(cuts[r], base), min(cuts[r + 1], base + n)
            if lo < hi:
                off = (lo - base) * MiB
                end = min(s, (hi - base) * MiB)
                out[r].append((f, off, end - off))
        base += n
    return out


def checksums_split(eng, sizes, segments, dev_addrs, out32, group=None):
    """This rank's share of the split checksum session. sizes: every file's
    length (> 1 MiB each, the same list on every rank); segments: this rank's
    (file, msg_off, length) from split_pieces; dev_addrs: the device address
    of each segment's bytes (written before the call on the current stream).
    Collective. Writes all files' 32-byte digests to out32 (device,
    len(sizes) x 32) on every rank, ordered before anything the caller
    enqueues next on its current stream."""
    dev = out32.device
    cur = torch.cuda.current_stream(dev)
    # the library's calls, the export / import copies and the all-reduce all
    # run on one side stream ordered after the caller's work (torch's default
    # stream is the legacy NULL stream, which libsdcas would read as "the
    # context's own stream", so it is never handed over as is)
    s = torch.cuda.Stream(dev)
    s.wait_stream(cur)
    sp = s.cuda_stream
    eng.dev_stream_begin(np.asarray(sizes, np.uint64))
    if segments:
        f, o, ln = (np.array([x[i] for x in segments], np.uint64) for i in range(3))
        eng.dev_stream_update(f, o, ln, np.asarray(dev_addrs, np.uint64), stream=sp)
    nbytes = eng.dev_stream_node_bytes()
    with torch.cuda.stream(s):
        nodes = torch.empty(nbytes // 8, dtype=torch.int64, device=dev)
        eng.dev_stream_export(nodes.data_ptr(), nbytes, sp)
        dist.all_reduce(nodes, group=group)  # each entry is nonzero on exactly one rank
        eng.dev_stream_import(nodes.data_ptr(), nbytes, sp)
        eng.dev_stream_finish(out32.data_ptr(), sp)
    out32.record_stream(s)
    cur.wait_stream(s)


__all__ = ["split_pieces", "checksums_split"]
