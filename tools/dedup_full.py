#!/usr/bin/env python3
"""The identifier dedup (file_identifier/mod.rs:149-254 inside the job's
cursor steps) over a WHOLE BASELINE corpus on one GPU: C3's 10 M files or C5's
50 M (bench.py shards them over 8 GPUs; here one world-of-one call takes the
lot, the largest group-by one sd-core job would hand one device).

Every file's cas key is made on the device (spacedrive_amd.synth messages,
sdcas_dev_hash_messages), --chunk files at a time, into one resident key
array; a sample of the keys is checked against upstream BLAKE3 C (the
oracle). Then:
  * sdcas_dev_dedup_local (the bench's N = 1 path) --reps times, each
    bracketed by HIP events on its stream: ms per call, the bytes the
    group-by must move at least (bench.dedup_bytes) over that time;
  * unless --no-parity: every link and both counts against the oracle's
    chunked dedup (oracle/cas_ref.c), for the device call AND for the host
    C ABI sd-core binds (sdcas_dedup: host keys in, links out), the latter
    timed too.
Run under rocprofv3 --pmc with --no-parity (tools/pmc_dedup.sh W REPS full;
tools/pmc_dedup_summary.py with CALLS = REPS + 1) for the HBM bytes: every
dispatch after the last hash kernel is the dedup's.

usage: dedup_full.py [--workload c5] [--files N] [--reps 5] [--existing K] [--errors F]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FULL = {"c3": 10_000_000, "c5": 50_000_000}
CHUNK = {"c3": 1_250_000, "c5": 6_250_000}  # bench.py's per-GPU shares


def corpus(workload, n):
    """(sizes, content keys) of the corpus' first n files (C5: the corpus in
    file order — bench.c5_share at world 1 with n = 50 M is the identity)"""
    import bench
    s, k, _ = bench.files_of(workload, 0, n, 1)
    return s, k


def device_keys(eng, torch, dev, sizes, ckeys, chunk, stream=0):
    """cas keys of the files (int64 device tensor), made chunk by chunk"""
    from spacedrive_amd import synth as S
    n = sizes.size
    out = torch.empty(n, dtype=torch.int64, device=dev)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).to(dev)
    blob = None
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        sz, ck = sizes[lo:hi], ckeys[lo:hi]
        lens = S.cas_msg_len(sz)
        padded = (lens + np.uint64(127)) // np.uint64(128) * np.uint64(128)
        offs = np.zeros(hi - lo, np.uint64)
        offs[1:] = np.cumsum(padded[:-1])
        total = int(offs[-1] + padded[-1]) + 64
        if blob is None or blob.numel() < total:
            blob = None
            blob = torch.empty(total, dtype=torch.uint8, device=dev)
        dk, ds, do, dl = t(ck), t(sz), t(offs), t(lens)
        eng.dev_reserve(hi - lo, int(np.maximum(np.uint64(1), (lens + np.uint64(1023)) // np.uint64(1024)).sum()))
        eng.dev_synth_cas_messages(dk.data_ptr(), ds.data_ptr(), do.data_ptr(), hi - lo, blob.data_ptr(), stream)
        eng.dev_hash_messages(blob.data_ptr(), do.data_ptr(), dl.data_ptr(), hi - lo, 0, out[lo:hi].data_ptr(), stream)
        eng.dev_sync(stream)
    del blob
    return out


def run(workload="c5", files=0, reps=5, existing=0, errors=0.0, parity=True, host_abi=True, sample=20000,
        chunk=0, seed=17, ab="", log=print):
    import torch

    import bench
    from spacedrive_amd import Engine
    from spacedrive_amd.dist_dedup import DeviceStages
    n = files or FULL[workload]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    t0 = time.perf_counter()
    sizes, ckeys = corpus(workload, n)
    log(f"[dedup_full] {workload} {n} files generated on the host in {time.perf_counter() - t0:.1f} s")
    eng = Engine(device=0)
    res = {"workload": workload.upper(), "files": n}
    try:
        # every device input but the keys exists before the hash, so that under
        # rocprofv3 every dispatch after the hash's last kernel is the dedup's
        rng = np.random.default_rng(seed)
        has = (sizes != 0).astype(np.uint8)  # mod.rs:78-86: an empty file has no cas_id
        status = np.where(rng.random(n) < errors, 5, 0).astype(np.int32) if errors else None
        d_has = torch.from_numpy(has).to(dev)
        d_status = torch.from_numpy(status).to(dev) if status is not None else None
        d_ids = torch.arange(n, dtype=torch.int64, device=dev)
        t0 = time.perf_counter()
        d_keys = device_keys(eng, torch, dev, sizes, ckeys, chunk or CHUNK[workload])
        res["keys_s"] = time.perf_counter() - t0
        keys = d_keys.cpu().numpy().view(np.uint64) if (parity or existing) else None
        ex = np.zeros(0, np.uint64)
        if existing:  # existing Objects: keys of random files and keys nobody carries, in DB order
            ex = np.concatenate([keys[rng.choice(n, existing - existing // 6, replace=False)],
                                 rng.integers(0, 2**64, existing // 6, dtype=np.uint64)])
        d_ek = torch.from_numpy(ex.view(np.int64)).to(dev) if ex.size else None
        d_ei = torch.arange(ex.size, dtype=torch.int64, device=dev) if ex.size else None
        log(f"[dedup_full] keys on the device in {res['keys_s']:.1f} s")
        stream = torch.cuda.Stream(dev)
        st = DeviceStages(eng, 0, same_stream=True)
        # A/B: settings (environment values the library reads per call)
        # interleaved per rep; the last setting is the one reported
        settings = [dict(kv.split("=") for kv in part.split("+")) for part in ab.replace("/", ",").split(",")] \
            if ab else [{}]
        per = {i: [] for i in range(len(settings))}
        outs = {}
        link = counts = None
        with torch.cuda.stream(stream):
            for r in range(reps + 1):
                for i, env in enumerate(settings):
                    os.environ.update(env)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    link, counts = st.local(d_keys, d_has, d_status, d_ids, 100, d_ek, d_ei)
                    e1.record(stream)
                    e1.synchronize()
                    if r:  # the first call sizes the workspace
                        per[i].append(e0.elapsed_time(e1))
                    if r == reps and len(settings) > 1:
                        outs[i] = (link.clone(), counts.clone())
        torch.cuda.synchronize()
        ms = per[len(settings) - 1]
        if len(settings) > 1:
            res["ab"] = {"+".join(f"{k}={v}" for k, v in env.items()): {"ms_median": float(np.median(per[i])),
                                                                      "ms_min": float(np.min(per[i]))}
                         for i, env in enumerate(settings)}
            l0, c0 = outs[0]
            res["ab_equal"] = all(torch.equal(l0, l) and torch.equal(c0, c) for l, c in outs.values())
            log(f"[dedup_full] A/B {res['ab']} equal {res['ab_equal']}")
        med = float(np.median(ms)) if ms else float("nan")
        algo = bench.dedup_bytes(n, ex.size)
        res.update({"existing": int(ex.size), "errors_frac": errors, "reps": reps, "ms_median": med,
                    "ms_min": float(np.min(ms)) if ms else None, "ms_all": ms, "algorithmic_bytes": algo,
                    "algorithmic_gbps": algo / med / 1e6, "frac_of_hbm_peak": algo / med / 1e6 / bench.HBM_PEAK_GBS,
                    "created_linked": [int(x) for x in counts.tolist()],
                    "files_per_s": n / med * 1e3})
        log(f"[dedup_full] device dedup {med:.3f} ms per call (median of {reps})")
        if parity:
            from tests._oracle import load_oracle
            oracle = load_oracle()
            # a sample of the keys against upstream BLAKE3 C
            pick = np.sort(rng.choice(n, min(sample, n), replace=False))
            want_k, hasher = oracle.synth_cas_keys(ckeys[pick], sizes[pick], threads=16)
            res["key_sample"] = {"checked": int(pick.size), "mismatches": int((keys[pick] != want_k).sum()),
                                 "hasher": hasher}
            t0 = time.perf_counter()
            want, wc, wl = oracle.identifier_dedup(keys, has, status, 100, ex)
            res["oracle_s"] = time.perf_counter() - t0
            got = link.cpu().numpy()
            res["device"] = {"links_equal": bool(np.array_equal(got, want)),
                             "mismatches": int((got != want).sum()),
                             "counts_equal": [int(x) for x in counts.tolist()] == [wc, wl]}
            res["oracle_created_linked"] = [wc, wl]
            log(f"[dedup_full] oracle {res['oracle_s']:.1f} s, device links equal: {res['device']['links_equal']}")
            del got
            if host_abi:
                t0 = time.perf_counter()
                hl, hc, hlk = eng.identifier_dedup(keys, has, status, 100, ex)
                res["host_abi"] = {"s": time.perf_counter() - t0, "links_equal": bool(np.array_equal(hl, want)),
                                   "counts_equal": (hc, hlk) == (wc, wl)}
                log(f"[dedup_full] sdcas_dedup (host arrays) {res['host_abi']['s']:.2f} s, "
                    f"links equal: {res['host_abi']['links_equal']}")
        res["distinct_keys"] = int(np.unique(keys[has != 0]).size) if keys is not None else None
    finally:
        eng.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c5", choices=["c3", "c5"])
    ap.add_argument("--files", type=int, default=0, help="0: the whole corpus (C3 10 M, C5 50 M)")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--existing", type=int, default=0)
    ap.add_argument("--errors", type=float, default=0.0, help="fraction of files with an I/O error")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-host-abi", action="store_true")
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--ab", default="", help="A/B: 'N1=a+N2=b,N1=c' (or '/' for ',') settings interleaved per rep")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    res = run(a.workload, a.files, a.reps, a.existing, a.errors, not a.no_parity, not a.no_host_abi,
              chunk=a.chunk, ab=a.ab, log=lambda s: print(s, file=sys.stderr, flush=True))
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
