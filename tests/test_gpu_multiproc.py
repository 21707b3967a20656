"""The multi-rank dedup path as real device code in real processes
(SURVEY.md §8e): two processes, one Engine and DeviceStages each (libsdcas's
HIP kernels on cuda:0), exchanging through torch.distributed. Two RCCL ranks
on one GPU are refused by RCCL, so the processes use gloo, whose collectives
take the same device tensors (staged through the host); the protocol code is
the one bench.py runs over RCCL. Each rank's links are compared with the
chunked oracle of file_identifier/mod.rs:149-254, for the exact protocol
(first call) and the one-synchronisation bucket protocol (second call),
with and without existing Objects.

Also: two streams sharing one context's device scratch (sdcas.h "Threading").
"""
import os
import socket
import tempfile
import time

import numpy as np
import pytest
import torch

from tests._dist_stages import make_corpus, shard

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _corpus(existing_mode):
    keys, has, status, existing = make_corpus(4242, 60000, pool=9000, n_existing=1 if existing_mode == "sparse"
                                              else 400)
    if existing_mode == "none":
        existing = existing[:0]
    return keys, has, status, existing


def _worker(rank, world, port, outdir, existing_mode):
    import torch.distributed as dist

    from spacedrive_amd import Engine
    from spacedrive_amd.dist_dedup import DeviceStages, identifier_dedup_distributed
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    eng = Engine(device=0)
    try:
        keys, has, status, existing = _corpus(existing_mode)
        shards, ex = shard(keys, has, status, existing, world, device="cuda")
        k, h, s, ids = shards[rank]
        ek, eids = ex[rank] if existing_mode != "none" else (None, None)
        st = DeviceStages(eng, 0)
        out = {}
        for call in range(2):
            link, c, l = identifier_dedup_distributed(st, k, h, s, ids, 100, ek, eids)
            out[f"link{call}"] = link.cpu().numpy()
            out[f"count{call}"] = np.array([c, l])
            out[f"proto{call}"] = np.array(st.last_protocol)
        np.savez(os.path.join(outdir, f"r{rank}.npz"), **out)
    finally:
        eng.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("existing_mode", ["full", "none", "sparse"])
def test_two_process_device_dedup(oracle, existing_mode):
    import torch.multiprocessing as mp
    world = 2
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.start_processes(_worker, args=(world, _free_port(), d, existing_mode), nprocs=world, join=False,
                                 start_method="spawn")
        deadline = time.time() + 100
        try:
            while not ctx.join(timeout=5):
                assert time.time() < deadline, "ranks did not finish"
        finally:
            for p in ctx.processes:
                if p.is_alive():
                    p.terminate()
        parts = [np.load(os.path.join(d, f"r{r}.npz")) for r in range(world)]
    keys, has, status, existing = _corpus(existing_mode)
    want, wc, wl = oracle.identifier_dedup(keys, has, status, 100, existing)
    for call in range(2):
        assert np.array_equal(np.concatenate([p[f"link{call}"] for p in parts]), want), call
        for p in parts:
            assert tuple(int(x) for x in p[f"count{call}"]) == (wc, wl)
    # the first call takes the buckets (capacities from the all-gathered file
    # counts) unless a rank holds more rows that stay orphans than the first
    # call's gather of them takes (256): it then reruns the exact protocol;
    # the second call uses what the first learned
    cuts = [keys.size * r // world for r in range(world + 1)]
    stays = [int(((status[a:b] != 0) | (has[a:b] == 0)).sum()) for a, b in zip(cuts, cuts[1:])]
    first = "buckets-overflow" if max(stays) > 256 else "buckets"
    assert [str(p["proto0"]) for p in parts] == [first] * world
    assert [str(p["proto1"]) for p in parts] == ["buckets"] * world


@pytest.mark.parametrize("bind", ["unbound", "bound", "rebound"])
def test_two_streams_share_one_context(oracle, bind):
    """dedup_local on two raw streams of one context, enqueued back to back
    with no ordering between the streams on the caller's side: the second
    call clears the shared resolve table while the first may still run, so
    the library must order them (sdcas_ctx::fence_in). Both results exact —
    also with both streams bound to tokens (sdcas_dev_bind_stream: the wait
    is skipped only between calls on one bound stream), and with one stream's
    handle bound to a token, then rebound to another (as after the caller
    re-created a stream whose handle came back)"""
    from spacedrive_amd import Engine
    eng = Engine()
    try:
        corpora = [make_corpus(s, 400_000, pool=50_000) for s in (1, 2)]
        dev = torch.device("cuda", 0)
        s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        if bind != "unbound":
            eng.dev_bind_stream(s1.cuda_stream)
            eng.dev_bind_stream(s2.cuda_stream)
        bufs = []
        for keys, has, status, existing in corpora:
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
            bufs.append(dict(k=t(keys.view(np.int64)), h=t(has), s=t(status),
                             ids=torch.arange(keys.size, dtype=torch.int64, device=dev),
                             ek=t(existing.view(np.int64)),
                             eids=torch.arange(existing.size, dtype=torch.int64, device=dev),
                             link=torch.empty(keys.size, dtype=torch.int64, device=dev),
                             cnt=torch.zeros(2, dtype=torch.int64, device=dev)))
        torch.cuda.synchronize()
        for rep in range(3):
            for b in bufs:
                b["cnt"].zero_()
            torch.cuda.synchronize()
            if bind == "rebound":
                eng.dev_bind_stream(s1.cuda_stream)  # a fresh token: the next call on s1 waits again
            for b, s in zip(bufs, (s1, s2)):
                rc = eng.L.sdcas_dev_dedup_local(eng.ctx, b["k"].data_ptr(), b["h"].data_ptr(), b["s"].data_ptr(),
                                                 b["ids"].data_ptr(), b["k"].numel(), b["ek"].data_ptr(),
                                                 b["eids"].data_ptr(), b["ek"].numel(), 100, 0, 0, 0,
                                                 b["link"].data_ptr(), b["cnt"].data_ptr(), None, s.cuda_stream)
                eng._check(rc, "sdcas_dev_dedup_local")
            torch.cuda.synchronize()
            for (keys, has, status, existing), b in zip(corpora, bufs):
                want, wc, wl = oracle.identifier_dedup(keys, has, status, 100, existing)
                assert np.array_equal(b["link"].cpu().numpy(), want), rep
                assert tuple(b["cnt"].tolist()) == (wc, wl)
    finally:
        eng.close()


# ---- big-file checksums with the pieces split over ranks (dist_checksum.py) ----

MiB = 1 << 20
SPLIT_SIZES = [5 * MiB + 3, 17 * MiB, 2 * MiB + 1, 33 * MiB - 1, 9 * MiB + 4095]


def _split_keys():
    from tests._oracle import content_key
    return [content_key(0x5D0004, 500 + i) for i in range(len(SPLIT_SIZES))]


def _rank_blob(segments, keys, dev):
    """this rank's segments' bytes generated in HBM -> (blob, device addresses)"""
    from tests._oracle import content
    offs, parts, pos = [], [], 0
    for f, off, ln in segments:
        offs.append(pos)
        parts.append(content("synth", off, ln, keys[f]))
        pos += (ln + MiB - 1) // MiB * MiB
    blob = torch.zeros(pos + 4096, dtype=torch.uint8, device=dev)
    for o, p in zip(offs, parts):
        blob[o:o + p.size].copy_(torch.from_numpy(p))
    return blob, [blob.data_ptr() + o for o in offs]


def test_split_checksum_virtual_ranks(oracle):
    """three contexts hash disjoint piece ranges of the same files; their node
    lists, summed, finish to the oracle's digests on every context"""
    from spacedrive_amd import Engine
    from spacedrive_amd.dist_checksum import split_pieces
    keys = _split_keys()
    R = 3
    parts = split_pieces(SPLIT_SIZES, R)
    engs = [Engine() for _ in range(R)]
    try:
        lists, blobs = [], []
        for r in range(R):
            blob, addrs = _rank_blob(parts[r], keys, "cuda")
            blobs.append(blob)
            torch.cuda.synchronize()
            e = engs[r]
            e.dev_stream_begin(SPLIT_SIZES)
            seg = parts[r]
            e.dev_stream_update([x[0] for x in seg], [x[1] for x in seg], [x[2] for x in seg], addrs)
            nb = e.dev_stream_node_bytes()
            t = torch.empty(nb // 8, dtype=torch.int64, device="cuda")
            e.dev_stream_export(t.data_ptr(), nb)
            e.dev_sync()
            lists.append(t)
        total = sum(lists)
        torch.cuda.synchronize()
        for r in range(R):
            out = torch.zeros((len(SPLIT_SIZES), 32), dtype=torch.uint8, device="cuda")
            engs[r].dev_stream_import(total.data_ptr(), total.numel() * 8)
            engs[r].dev_stream_finish(out.data_ptr())
            engs[r].dev_sync()
            got = out.cpu().numpy()
            for i, (k, n) in enumerate(zip(keys, SPLIT_SIZES)):
                assert bytes(got[i]).hex() == oracle.synth_checksum(k, n), (r, n)
    finally:
        for e in engs:
            e.close()


def _split_worker(rank, world, port, outdir):
    import torch.distributed as dist

    from spacedrive_amd import Engine
    from spacedrive_amd.dist_checksum import checksums_split, split_pieces
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    eng = Engine(device=0)
    try:
        keys = _split_keys()
        seg = split_pieces(SPLIT_SIZES, world)[rank]
        blob, addrs = _rank_blob(seg, keys, "cuda")
        out = torch.zeros((len(SPLIT_SIZES), 32), dtype=torch.uint8, device="cuda")
        checksums_split(eng, SPLIT_SIZES, seg, addrs, out)
        np.save(os.path.join(outdir, f"r{rank}.npy"), out.cpu().numpy())
    finally:
        eng.close()
        dist.destroy_process_group()


def test_split_checksum_two_processes(oracle):
    """two processes (gloo, the collective bench.py runs over RCCL) split the
    files' pieces; both end with every file's exact digest"""
    import torch.multiprocessing as mp
    world = 2
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.start_processes(_split_worker, args=(world, _free_port(), d), nprocs=world, join=False,
                                 start_method="spawn")
        deadline = time.time() + 100
        try:
            while not ctx.join(timeout=5):
                assert time.time() < deadline, "ranks did not finish"
        finally:
            for p in ctx.processes:
                if p.is_alive():
                    p.terminate()
        outs = [np.load(os.path.join(d, f"r{r}.npy")) for r in range(world)]
    for got in outs:
        for i, (k, n) in enumerate(zip(_split_keys(), SPLIT_SIZES)):
            assert bytes(got[i]).hex() == oracle.synth_checksum(k, n), n


@pytest.mark.parametrize("launcher", ["torchrun", "plain"])
@pytest.mark.parametrize("workload", ["c2", "c5", "c4"])
def test_bench_two_ranks(workload, launcher):
    """bench.py as the driver launches it at N > 1 — under
    torch.distributed.run, or as a plain `python3 bench.py --gpus 2` that
    starts its two ranks itself — on the one GPU with gloo standing in for
    RCCL: ONE line that reports both ranks, every rank's oracle sample
    matches, and the c5 dedup exchange gives the chunked oracle's links over
    both ranks' files"""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SDCAS_BENCH_BACKEND="gloo", OMP_NUM_THREADS="4")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    args = ["bench.py", "--gpus", "2", "--workload", workload, "--files", "20000", "--steps", "2", "--warmup", "1",
            "--sustain-s", "0.5", "--c4-total-gib", "4"]
    if launcher == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    else:
        cmd = [sys.executable] + args
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if '{"metric"' in l]
    if launcher == "plain":
        assert len(lines) == 1 and lines[0].startswith('{"metric"'), r.stdout[-2000:]
    line = lines[-1]
    d = json.loads(line[line.index('{"metric"'):])  # torchrun may prefix a rank tag
    assert d["n_gpus"] == 2 and d["value"] > 0
    if workload != "c4":  # the untimed sustained phase, as many steps on every rank
        assert d["sustained"]["steps"] >= 16 and d["sustained"]["value"] > 0
    assert d["parity"]["ranks"] == 2 and d["parity"]["checked_files"] >= (2 if workload == "c4" else 2000)
    assert d["parity"]["mismatches"] == 0
    if workload == "c5":
        assert d["dedup"]["records_per_gpu"] == 20000
        pd = d["parity"]["dedup"]  # both ranks' links against the oracle over the whole corpus
        assert pd["files"] == 40000 and pd["link_mismatches"] == 0 and pd["counts_match"]
        # the shares carry the corpus' duplicates at this size (bench.c5_share):
        # the exchange links files, the Zipf head's among them
        assert d["dedup"]["files_linked"] > 0
        # the dedup priced: bytes over time against HBM, and the exchange's
        # bytes and collective time
        assert d["dedup"]["roofline"]["bound"] == "hbm" and d["dedup"]["roofline"]["frac"] > 0
        x = d["dedup"]["exchange"]
        assert x["bytes_per_rank"] >= 20000 * 16 and 0 < x["bytes_off_rank"] < x["bytes_per_rank"] and x["ms"] > 0
