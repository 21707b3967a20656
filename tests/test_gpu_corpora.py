"""Configs C3 and C5 (BASELINE.json) through the HIP path, against the oracle.

A 200 k-file subset of each synthetic corpus (spacedrive_amd.synth, the
definition bench.py uses) is generated in HBM, hashed by the device API
(sdcas_dev_hash_messages: both cas.rs branches, the sampled one for every
file > 100 KiB), and EVERY key is compared with the oracle's (upstream
BLAKE3 C through oracle_synth_cas_keys_mt). The keys then go through the
identifier dedup (file_identifier/mod.rs:190-254, chunks of 100) on the
device — the fused single-rank path, the host-array C ABI (sdcas_dedup) and
the multi-rank bucket protocol over virtual ranks — and every link and both
counts are compared with oracle.identifier_dedup.

C5's subset is every 31st file of bench.py's rank-0 share of the 50 M-file
corpus (stride 8 over the whole corpus), so its mix of first copies (40 %)
and Zipf(1.1) duplicates (60 %, heavy hitters included) is the corpus's.
Orphan ordinals are positions in the subset (the job's id order).
"""
import numpy as np
import pytest
import torch

from spacedrive_amd import synth as S
from tests._dist_stages import dedup_virtual_buckets

pytestmark = pytest.mark.gpu
N_SUBSET = 200_000


@pytest.fixture(scope="module")
def eng():
    from spacedrive_amd import Engine
    e = Engine()
    yield e
    e.close()


def c3_subset(n=N_SUBSET):
    sizes, ckeys, _ = S.c3_files(0, n)
    return sizes, ckeys


def c5_subset(share=6_250_000, step=31):
    ids = (np.arange(share, dtype=np.uint64) * np.uint64(8))[::step]
    cid = S.c5_content_ids_at(ids)
    return S.c5_sizes_of(cid), S.content_key(S.SEED_C5, cid)


def device_keys(eng, sizes, ckeys):
    """cas keys of synthetic files, messages generated and hashed in HBM"""
    n = sizes.size
    lens = S.cas_msg_len(sizes)
    padded = (lens + np.uint64(127)) // np.uint64(128) * np.uint64(128)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(padded[:-1])
    total = int(offs[-1] + padded[-1]) + 64
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
    blob = torch.empty(total, dtype=torch.uint8, device=dev)
    dk, ds, do, dl = t(ckeys), t(sizes), t(offs), t(lens)
    out = torch.zeros(n, dtype=torch.int64, device=dev)
    eng.dev_reserve(n, int(np.maximum(np.uint64(1), (lens + np.uint64(1023)) // np.uint64(1024)).sum()))
    eng.dev_synth_cas_messages(dk.data_ptr(), ds.data_ptr(), do.data_ptr(), n, blob.data_ptr())
    eng.dev_hash_messages(blob.data_ptr(), do.data_ptr(), dl.data_ptr(), n, 0, out.data_ptr())
    eng.dev_sync()
    return out.cpu().numpy().view(np.uint64)


def check_dedup(eng, oracle, keys, sizes, rng):
    from spacedrive_amd.dist_dedup import DeviceStages
    n = keys.size
    has = (sizes != 0).astype(np.uint8)  # mod.rs:78-86: empty files have no cas_id
    status = np.where(rng.random(n) < 0.002, 5, 0).astype(np.int32)  # a few I/O errors
    existing = np.concatenate([keys[rng.choice(n, 3000, replace=False)],
                               rng.integers(0, 2**64, 500, dtype=np.uint64)])
    dev = torch.device("cuda", 0)
    tk = torch.from_numpy(keys.view(np.int64)).to(dev)
    th, ts = torch.from_numpy(has).to(dev), torch.from_numpy(status).to(dev)
    ids = torch.arange(n, dtype=torch.int64, device=dev)
    ek = torch.from_numpy(existing.view(np.int64)).to(dev)
    eids = torch.arange(existing.size, dtype=torch.int64, device=dev)
    st = DeviceStages(eng)
    for ex in (False, True):
        exk = existing if ex else np.zeros(0, np.uint64)
        want, wc, wl = oracle.identifier_dedup(keys, has, status, 100, exk)
        # fused single-rank device path (bench.py at N = 1)
        link, cnt = st.local(tk, th, ts, ids, 100, ek if ex else None, eids if ex else None)
        assert np.array_equal(link.cpu().numpy(), want)
        assert tuple(cnt.tolist()) == (wc, wl)
        # the host-array C ABI sd-core binds (sdcas_dedup)
        got, gc, gl = eng.identifier_dedup(keys, has, status, 100, exk)
        assert np.array_equal(got, want) and (gc, gl) == (wc, wl)
        # the multi-rank bucket protocol, 4 virtual ranks (contiguous shares)
        R = 4
        cuts = [n * r // R for r in range(R + 1)]
        shards = [(tk[cuts[r]:cuts[r + 1]], th[cuts[r]:cuts[r + 1]], ts[cuts[r]:cuts[r + 1]],
                   ids[cuts[r]:cuts[r + 1]]) for r in range(R)]
        exs = [(ek[r::R].contiguous(), eids[r::R].contiguous()) for r in range(R)] if ex else None
        caps = (n // R + 1, existing.size // R + 1)
        links, c, l, over = dedup_virtual_buckets(lambda r: st, shards, 100, exs, caps)
        assert not over
        assert np.array_equal(np.concatenate([x.cpu().numpy() for x in links]), want)
        assert (c, l) == (wc, wl)


@pytest.mark.parametrize("config", ["c3", "c5"])
def test_corpus_subset_keys_and_dedup(eng, oracle, config):
    sizes, ckeys = c3_subset() if config == "c3" else c5_subset()
    assert sizes.size >= N_SUBSET
    sampled = int((sizes > np.uint64(S.MIN_FILE)).sum())
    assert sampled > 1000  # both cas.rs branches are exercised
    got = device_keys(eng, sizes, ckeys)
    want, hasher = oracle.synth_cas_keys(ckeys, sizes, threads=16)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (hasher, bad[:10], sizes[bad[:10]])
    # the corpus really duplicates: C3 ~15 % duplicate files, C5 ~60 %
    dup_frac = 1 - np.unique(want).size / want.size
    assert dup_frac > (0.1 if config == "c3" else 0.3), dup_frac
    check_dedup(eng, oracle, got, sizes, np.random.default_rng(17 if config == "c3" else 19))
