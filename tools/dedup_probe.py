#!/usr/bin/env python3
"""Price the identifier dedup (file_identifier/mod.rs:149-254 inside the job's
steps) on one GPU: the C3 or C5 share bench.py builds, hashed once, then the
world-of-one dedup (sdcas_dev_dedup_local: stays select, plan walk, table
memset, k_solo_insert, k_solo_apply) run --reps times, each bracketed by HIP
events on the stream it runs on. One JSON line: ms per dedup, the bytes it
must move at least (bench.dedup_bytes) and that figure over the time against
the HBM peak. Run under rocprofv3 --pmc (tools/pmc_dedup.sh) for the bytes
it does move: every kernel after the hash belongs to the dedup.

usage: dedup_probe.py [--workload c5] [--files N] [--reps 20] [--existing K]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def settings(spec):
    """'N=v1,v2' -> [{N: v1}, {N: v2}]; 'N1=a+N2=b,N1=c' -> [{N1: a, N2: b}, {N1: c}]"""
    if spec.count("=") == 1:
        name, vals = spec.split("=")
        return [{name: v} for v in vals.split(",")]
    return [dict(kv.split("=") for kv in part.split("+")) for part in spec.split(",")]


def label(env):
    return "+".join(f"{k}={v}" for k, v in env.items())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c5", choices=["c3", "c5"])
    ap.add_argument("--files", type=int, default=0)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--existing", type=int, default=0, help="existing Objects (cas keys of the first K files)")
    ap.add_argument("--tables", default="", help="A/B: comma-separated SDCAS_DEDUP_TABLE values, interleaved per rep")
    ap.add_argument("--ab", default="",
                    help="A/B of settings, interleaved per rep: 'NAME=v1,v2' or 'N1=a+N2=b,N1=c+N2=d' (environment "
                         "values each library call reads), e.g. SDCAS_DEDUP_TABLE=tile,idx")
    ap.add_argument("--world", type=int, default=1,
                    help="> 1: one rank's device stages of the bucket protocol at this world size (combine_buckets, "
                         "resolve_buckets over its own buckets as if received, apply), each timed; no exchange")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    import bench
    from spacedrive_amd import Engine
    from spacedrive_amd import synth as S
    from spacedrive_amd.dist_dedup import DeviceStages
    n = a.files or bench.WORKLOADS[a.workload]["files"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    sizes, keys, ids = bench.files_of(a.workload, 0, n)
    lens = S.cas_msg_len(sizes)
    padded = (lens + np.uint64(127)) // np.uint64(128) * np.uint64(128)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(padded[:-1])
    total = int(offs[-1] + padded[-1]) + 64
    chunks = int(np.maximum(np.uint64(1), (lens + np.uint64(1023)) // np.uint64(1024)).sum())
    eng = Engine(device=0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).to(dev)
    d_blob = torch.empty(total, dtype=torch.uint8, device=dev)
    d_keys, d_sizes, d_offs, d_lens = t(keys), t(sizes), t(offs), t(lens)
    d_out = torch.zeros(n, dtype=torch.int64, device=dev)
    # every device input of the dedup exists before the hash, so that under
    # rocprofv3 every dispatch after the hash's last kernel is the dedup's
    d_has = (d_sizes != 0).to(torch.uint8)
    d_ids = torch.from_numpy(ids).to(dev)
    ei = torch.arange(a.existing, dtype=torch.int64, device=dev) if a.existing else None
    ek = torch.empty(a.existing, dtype=torch.int64, device=dev) if a.existing else None
    eng.dev_reserve(n, chunks)
    eng.dev_synth_cas_messages(d_keys.data_ptr(), d_sizes.data_ptr(), d_offs.data_ptr(), n, d_blob.data_ptr(), sp)
    eng.dev_hash_messages(d_blob.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, 0, d_out.data_ptr(), sp)
    if a.existing:  # the first K files' keys stand for K existing Objects
        ek.copy_(d_out[: a.existing])
    torch.cuda.synchronize()
    del d_blob
    stages = DeviceStages(eng, 0)
    if a.world > 1:
        W = a.world
        cap = int(n / W * 1.125) + 256
        combines = settings(a.ab) if a.ab else [{}]
        combines = {label(c): c for c in combines}
        tm = {c: {"combine_buckets": [], "resolve_buckets": [], "apply": []} for c in combines}
        links = {}
        ovf = None
        for r in range(a.reps + 2):
            for c, env in combines.items():
                os.environ.update(env)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                ev[0].record(stream)
                send, slot, cnt, ovf = stages.combine_buckets(d_out, d_has, None, d_ids, W, cap)
                ev[1].record(stream)
                res = stages.resolve_buckets(send, cap, cnt, None, 0, None, W)
                ev[2].record(stream)
                link, counts = stages.apply(d_ids, slot, res, 100)
                ev[3].record(stream)
                if r >= 2:
                    for k, (x, y) in zip(tm[c], zip(ev[:-1], ev[1:])):
                        tm[c][k].append((x, y))
                if r == a.reps + 1:
                    links[c] = (link.clone(), counts.clone())
        torch.cuda.synchronize()
        out = {c: {k: float(np.median([x.elapsed_time(y) for x, y in v])) for k, v in t.items()} for c, t in tm.items()}
        l0, c0 = links[next(iter(combines))]
        print(json.dumps({"workload": a.workload.upper(), "files": n, "world": W, "bucket_cap": cap,
                          "overflow": int(ovf.item()), "ms_median": out,
                          "ms_total": {c: sum(v.values()) for c, v in out.items()},
                          "equal": all(torch.equal(l0, l) and torch.equal(c0, x) for l, x in links.values())}),
              flush=True)
        eng.close()
        dist.destroy_process_group()
        return
    if a.ab:
        tables = {label(c): c for c in settings(a.ab)}
    else:
        tables = {t: {"SDCAS_DEDUP_TABLE": t} for t in a.tables.split(",") if t} or {"": {}}
    ev = {t: [] for t in tables}
    links = {}
    link = counts = None
    for r in range(a.reps + 2):
        for t, env in tables.items():
            os.environ.update(env)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            link, counts = stages.local(d_out, d_has, None, d_ids, 100, ek, ei)
            e1.record(stream)
            if r >= 2:
                ev[t].append((e0, e1))
            if r == a.reps + 1 and len(tables) > 1:
                links[t] = (link.clone(), counts.clone())
    torch.cuda.synchronize()
    per = {t: [x.elapsed_time(y) for x, y in v] for t, v in ev.items()}
    ms = per[list(tables)[-1]]
    gk = d_out.cpu().numpy().view(np.uint64)
    distinct = int(np.unique(gk[sizes != 0]).size)
    algo = bench.dedup_bytes(n, a.existing)
    med = float(np.median(ms))
    res = {"workload": a.workload.upper(), "files": n, "existing": a.existing, "distinct_keys": distinct,
           "reps": a.reps, "ms_median": med, "ms_mean": float(np.mean(ms)), "ms_min": float(np.min(ms)),
           "algorithmic_bytes": algo, "algorithmic_gbps": algo / med / 1e6,
           "frac_of_hbm_peak": algo / med / 1e6 / bench.HBM_PEAK_GBS,
           "created_linked": [int(x) for x in counts.tolist()]}
    if len(tables) > 1:
        res["ab"] = {t: {"ms_median": float(np.median(v)), "ms_min": float(np.min(v))} for t, v in per.items()}
        l0, c0 = links[next(iter(tables))]
        res["ab_equal"] = all(torch.equal(l0, l) and torch.equal(c0, c) for l, c in links.values())
    print(json.dumps(res), flush=True)
    eng.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
