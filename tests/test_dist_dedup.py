"""Multi-GPU dedup: the collective protocol of
spacedrive_amd.dist_dedup against the chunked CPU oracle of
file_identifier/mod.rs:149-254 (oracle_identifier_dedup).

CPU: the real torch.distributed protocol under gloo (world 2 and 4, one
process per rank) with the numpy stages (tests/_dist_stages.py), and the
virtual-rank protocol with the numpy stages.
GPU: the device stages (libsdcas HIP kernels) under the virtual-rank protocol
for R = 1..8, and the real protocol over RCCL at world 1.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch

from tests._dist_stages import NumpyStages, dedup_virtual, make_corpus, shard

INT64_MIN = np.iinfo(np.int64).min


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_corpus(seed, n, existing_mode):
    # "full": ~350 existing Objects; "sparse": one, so most ranks' shares are
    # empty; "none": the caller passes no existing Objects at all
    keys, has, status, existing = make_corpus(seed, n, n_existing=1 if existing_mode == "sparse" else 300)
    if existing_mode == "none":
        existing = existing[:0]
    return keys, has, status, existing


def _gloo_worker(rank, world, port, outdir, seed, n, chunk_size, existing_mode="full", caps=None, grow=1):
    import torch.distributed as dist

    from spacedrive_amd.dist_dedup import identifier_dedup_distributed
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        st = NumpyStages()
        if caps is not None:
            st.force_caps = caps  # the first call's capacities
        # the same stages object twice: the first call seeds its bucket
        # capacities from the all-gathered file counts (or takes the given
        # caps), the second rescales the first's fills to its own load
        # (`grow` times the first's files)
        out = {}
        for call in range(2):
            keys, has, status, existing = _gloo_corpus(seed + call, n * (grow if call else 1), existing_mode)
            shards, ex = shard(keys, has, status, existing, world)
            k, h, s, ids = shards[rank]
            ek, eids = ex[rank] if existing_mode != "none" else (None, None)
            link, created, linked = identifier_dedup_distributed(st, k, h, s, ids, chunk_size, ek, eids)
            out[f"link{call}"] = link.numpy()
            out[f"count{call}"] = np.array([created, linked])
            out[f"proto{call}"] = np.array(st.last_protocol)
        np.savez(os.path.join(outdir, f"r{rank}.npz"), **out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,chunk_size,existing_mode,grow", [
    (1, 100, "full", 1), (2, 100, "full", 1), (4, 7, "full", 1), (3, 1, "full", 1), (1, 100, "none", 1),
    (2, 100, "none", 1), (3, 100, "sparse", 1), (2, 100, "full", 3), (3, 100, "none", 3)])
def test_gloo_protocol_vs_oracle(oracle, world, chunk_size, existing_mode, grow):
    """fixed-capacity buckets from the first call on (one device sync per
    call), also when the second call carries 3x the first's files"""
    import torch.multiprocessing as mp
    seed, n = 1000 + world, 3000
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_gloo_worker, args=(world, _free_port(), d, seed, n, chunk_size, existing_mode, None,
                                               grow),
                           nprocs=world, join=True, start_method="spawn")
        parts = [np.load(os.path.join(d, f"r{r}.npz")) for r in range(world)]
    for call in range(2):
        keys, has, status, existing = _gloo_corpus(seed + call, n * (grow if call else 1), existing_mode)
        want, wc, wl = oracle.identifier_dedup(keys, has, status, chunk_size, existing)
        got = np.concatenate([p[f"link{call}"] for p in parts])
        assert np.array_equal(got, want)
        for p in parts:  # node-wide totals on every rank
            assert tuple(int(x) for x in p[f"count{call}"]) == (wc, wl)
    if world > 1:
        assert [str(p["proto0"]) for p in parts] == ["buckets"] * world
        assert [str(p["proto1"]) for p in parts] == ["buckets"] * world


@pytest.mark.parametrize("caps", [(8, 8), (100_000, 100_000, 3)])
def test_gloo_bucket_overflow_falls_back(oracle, caps):
    """buckets too small for the records (or the stays gather too small for
    the rows that stay orphans): the overflow flag travels with the totals,
    every rank reruns the exact protocol, links still exact"""
    import torch.multiprocessing as mp
    world, seed, n = 3, 77, 3000
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_gloo_worker, args=(world, _free_port(), d, seed, n, 100, "full", caps),
                           nprocs=world, join=True, start_method="spawn")
        parts = [np.load(os.path.join(d, f"r{r}.npz")) for r in range(world)]
    for call in range(2):
        keys, has, status, existing = _gloo_corpus(seed + call, n, "full")
        want, wc, wl = oracle.identifier_dedup(keys, has, status, 100, existing)
        assert np.array_equal(np.concatenate([p[f"link{call}"] for p in parts]), want)
        for p in parts:
            assert tuple(int(x) for x in p[f"count{call}"]) == (wc, wl)
    assert [str(p["proto0"]) for p in parts] == ["buckets-overflow"] * world
    assert [str(p["proto1"]) for p in parts] == ["buckets"] * world


@pytest.mark.parametrize("R", [1, 2, 5, 8])
def test_virtual_protocol_numpy_vs_oracle(oracle, R):
    keys, has, status, existing = make_corpus(7 + R, 2500)
    shards, ex = shard(keys, has, status, existing, R)
    links, c, l = dedup_virtual(lambda r: NumpyStages(), shards, 100, ex)
    want, wc, wl = oracle.identifier_dedup(keys, has, status, 100, existing)
    assert np.array_equal(np.concatenate([x.numpy() for x in links]), want)
    assert (c, l) == (wc, wl)


def _numpy_window(keys, has, status, existing, cs, max_steps=0, more=False):
    """one rank's numpy stages with the job window -> (link, created, linked, plan header)"""
    st = NumpyStages()
    (k, h, s, ids), = shard(keys, has, status, existing, 1)[0]
    ek = torch.from_numpy(np.ascontiguousarray(existing).view(np.int64))
    eids = torch.arange(existing.size, dtype=torch.int64)
    rec, slot, _ = st.combine(k, h, s, ids, 1)
    erec, _, _ = st.combine(ek, None, None, eids, 1)
    ans = st.resolve(rec, erec)
    stays, _ = st.stays(h, s, ids, max(keys.size, 1))
    plan = st.plan(stays, keys.size, cs, max_steps, more)
    link, cnt = st.apply(ids, slot, ans, cs, plan)
    return link.numpy(), int(cnt[0]), int(cnt[1]), plan.numpy()[:12]


@pytest.mark.parametrize("seed", range(60))
def test_step_plan_matches_literal_step_loop(oracle, seed):
    """the plan's closed form (re-reads from the stays ordinals, positions,
    limit, repeated rows) against the oracle's literal cursor loop, on small
    dense cases: every chunk size from 1, stays rows at chunk ends, budgets
    above and below what the rows need, windows with more rows to come"""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 60))
    cs = int(rng.choice([1, 2, 3, 4, 7, 10, 100]))
    pool = rng.integers(0, 2**64, max(2, n // 3), dtype=np.uint64)
    keys = pool[rng.integers(0, pool.size, n)]
    has = (rng.random(n) > rng.random() * 0.5).astype(np.uint8)
    status = np.where(rng.random(n) < rng.random() * 0.4, 5, 0).astype(np.int32)
    existing = pool[rng.integers(0, pool.size, int(rng.integers(0, 4)))]
    for max_steps, more in ((0, False), (int(rng.integers(1, 2 * n + 2)), False),
                            (int(rng.integers(1, 2 * n + 2)), True), (0, True)):
        want, wc, wl, ww = oracle.identifier_job(keys, has, status, cs, existing, max_steps, more)
        got, gc, gl, head = _numpy_window(keys, has, status, existing, cs, max_steps, more)
        case = (n, cs, max_steps, more)
        assert np.array_equal(got, want), case
        assert (gc, gl) == (wc, wl), case
        assert (int(head[2]), int(head[3]), int(head[8])) == (ww["steps"], ww["rows"], ww["rereads"]), case


def collision_corpus(seed=11, n=8000):
    """keys drawn from 40 top-32-bit prefixes x 4 low values: many distinct
    keys share their top 32 bits (the combine's sort key)"""
    rng = np.random.default_rng(seed)
    hi = rng.integers(0, 2**32, 40, dtype=np.uint64) << np.uint64(32)
    pool = (hi[rng.integers(0, 40, 600)] | rng.integers(0, 4, 600, dtype=np.uint64)).astype(np.uint64)
    keys = pool[rng.integers(0, pool.size, n)]
    has = (rng.random(n) > 0.02).astype(np.uint8)
    status = np.where(rng.random(n) < 0.01, 5, 0).astype(np.int32)
    return keys, has, status, pool[:25].copy()


@pytest.mark.parametrize("R", [1, 3])
def test_virtual_protocol_numpy_top32_collisions(oracle, R):
    keys, has, status, existing = collision_corpus()
    shards, ex = shard(keys, has, status, existing, R)
    links, c, l = dedup_virtual(lambda r: NumpyStages(), shards, 100, ex)
    want, wc, wl = oracle.identifier_dedup(keys, has, status, 100, existing)
    assert np.array_equal(np.concatenate([x.numpy() for x in links]), want)
    assert (c, l) == (wc, wl)


def test_owner_is_monotone_and_covers_ranks():
    from spacedrive_amd.dist_dedup import owner_of
    k = np.sort(np.random.default_rng(0).integers(0, 2**64, 10000, dtype=np.uint64))
    for w in (1, 2, 3, 8, 16):
        o = owner_of(k, w)
        assert np.all(np.diff(o) >= 0) and o.min() == 0 and o.max() == w - 1
    assert owner_of(np.array([2**64 - 1], np.uint64), 8)[0] == 7


# ---- GPU: device stages ------------------------------------------------------

@pytest.fixture(scope="module")
def eng():
    from spacedrive_amd import Engine
    e = Engine()
    yield e
    e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("R,chunk_size", [(1, 100), (2, 100), (3, 7), (8, 100), (8, 1)])
def test_device_stages_virtual_vs_oracle(eng, oracle, R, chunk_size):
    from spacedrive_amd.dist_dedup import DeviceStages
    keys, has, status, existing = make_corpus(50 + R, 40000, pool=6000)
    shards, ex = shard(keys, has, status, existing, R, device="cuda")
    st = DeviceStages(eng)
    links, c, l = dedup_virtual(lambda r: st, shards, chunk_size, ex)
    want, wc, wl = oracle.identifier_dedup(keys, has, status, chunk_size, existing)
    got = np.concatenate([x.cpu().numpy() for x in links])
    assert np.array_equal(got, want)
    assert (c, l) == (wc, wl)


@pytest.mark.gpu
@pytest.mark.parametrize("R", [1, 3])
def test_device_stages_on_callers_stream(eng, oracle, R):
    """same_stream=True (the bench's setting): the stages enqueue on the
    caller's current stream, with no cross-stream waits; same links"""
    from spacedrive_amd.dist_dedup import DeviceStages
    keys, has, status, existing = make_corpus(70 + R, 30000, pool=5000)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        shards, ex = shard(keys, has, status, existing, R, device="cuda")
        st = DeviceStages(eng, same_stream=True)
        assert st._current() is not None and st._enter() == s.cuda_stream
        links, c, l = dedup_virtual(lambda r: st, shards, 100, ex)
        got = np.concatenate([x.cpu().numpy() for x in links])
    want, wc, wl = oracle.identifier_dedup(keys, has, status, 100, existing)
    assert np.array_equal(got, want)
    assert (c, l) == (wc, wl)


@pytest.mark.gpu
def test_device_stages_match_numpy_stages(eng):
    """stage by stage, device vs numpy restatement (records, slots, answers):
    the device combine's records within an owner's range come in no
    particular order (a hash table), so records are compared as per-owner
    sets and slots through the records they name"""
    from spacedrive_amd.dist_dedup import DeviceStages
    keys, has, status, existing = make_corpus(5, 20000)
    keys[:3] = np.uint64(2**64 - 1)  # the table's empty marker is a legal key
    (k, h, s, ids), = shard(keys, has, status, existing, 1, device="cuda")[0]
    st, ns = DeviceStages(eng), NumpyStages()
    for world in (1, 4, 7):
        rec_d, slot_d, starts_d = st.combine(k, h, s, ids, world)
        rec_n, slot_n, starts_n = ns.combine(k.cpu(), h.cpu(), s.cpu(), ids.cpu(), world)
        assert starts_d == starts_n
        rd, rn = rec_d.cpu().numpy(), rec_n.numpy()
        for r in range(world):
            a, b = rd[starts_d[r]:starts_d[r + 1]], rn[starts_n[r]:starts_n[r + 1]]
            assert np.array_equal(a[np.lexsort(a.T[::-1])], b[np.lexsort(b.T[::-1])]), r
        sd, sn = slot_d.cpu().numpy().view(np.uint32), slot_n.numpy().view(np.uint32)
        keyed = sn < 0xFFFFFFFE
        assert np.array_equal(sd[~keyed], sn[~keyed])
        assert np.array_equal(rd[sd[keyed]], rn[sn[keyed]])
    ek = torch.from_numpy(existing.view(np.int64)).cuda()
    eids = torch.arange(existing.size, dtype=torch.int64, device="cuda")
    erec_d, _, _ = st.combine(ek, None, None, eids, 1)
    ans_d = st.resolve(rec_d, erec_d)
    ans_n = ns.resolve(rec_d.cpu(), erec_d.cpu())
    assert torch.equal(ans_d.cpu(), ans_n)


def _owner_np(keys, world):
    return ((keys >> np.uint64(52)).astype(np.uint64) * np.uint64(world)) >> np.uint64(12)


@pytest.mark.gpu
@pytest.mark.parametrize("corpus", ["default", "collisions"])
def test_combine_contract_one_record_per_key(eng, corpus):
    """sdcas.h's combine contract (ABI 5), checked against numpy directly
    rather than against the numpy stages: owner r's range
    [starts[r], starts[r+1]) holds, as a multiset, exactly one (key, lowest
    id) record per distinct key of a keyed, unerrored file whose owner is r
    (no duplicate, no order assumed), and every such file's slot names its
    key's record; the same through sdcas_dev_dedup_combine_async with the
    starts left on the device"""
    import ctypes

    from spacedrive_amd.dist_dedup import DeviceStages
    if corpus == "default":
        keys, has, status, _ = make_corpus(23, 25000)
        keys[:3] = np.uint64(2**64 - 1)
    else:
        keys, has, status, _ = collision_corpus()
    (k, h, s, ids), = shard(keys, has, status, keys[:0], 1, device="cuda")[0]
    ok = (has != 0) & (status == 0)
    st = DeviceStages(eng)
    for world in (1, 3, 8):
        rec, slot, starts = st.combine(k, h, s, ids, world)
        n = keys.size
        rec2 = torch.empty((n, 2), dtype=torch.int64, device="cuda")
        slot2 = torch.empty(n, dtype=torch.int32, device="cuda")
        d_starts = torch.empty(world + 1, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        rc = eng.L.sdcas_dev_dedup_combine_async(eng.ctx, k.data_ptr(), h.data_ptr(), s.data_ptr(), ids.data_ptr(),
                                                 n, world, rec2.data_ptr(), slot2.data_ptr(), d_starts.data_ptr(),
                                                 None)
        eng._check(rc, "sdcas_dev_dedup_combine_async")
        eng._check(eng.L.sdcas_dev_sync(eng.ctx, None), "sdcas_dev_sync")
        starts2 = d_starts.cpu().numpy().view(np.uint32).astype(np.int64).tolist()
        uk, first = np.unique(keys[ok], return_index=True)
        want_id = np.flatnonzero(ok)[first]
        own = _owner_np(uk, world)
        for got_rec, got_slot, got_starts in ((rec, slot, starts), (rec2, slot2, starts2)):
            rd = got_rec[: got_starts[world]].cpu().numpy()
            assert got_starts[world] == uk.size, world
            for r in range(world):
                a = rd[got_starts[r]:got_starts[r + 1]]
                sel = own == r
                assert a.shape[0] == int(sel.sum()), (world, r)
                ak = a[:, 0].view(np.uint64)
                o = np.argsort(ak, kind="stable")
                assert np.array_equal(ak[o], uk[sel]), (world, r)  # each key once
                assert np.array_equal(a[o, 1], want_id[sel]), (world, r)
            sl = got_slot[:n].cpu().numpy().view(np.uint32)
            assert np.all(sl[~ok & (status != 0)] == 0xFFFFFFFE)
            assert np.all(sl[(status == 0) & (has == 0)] == 0xFFFFFFFF)
            assert np.array_equal(rd[sl[ok], 0].view(np.uint64), keys[ok]), world


@pytest.mark.gpu
@pytest.mark.parametrize("chunk_size", [100, 7, 2])
def test_device_reread_index(eng, oracle, chunk_size, monkeypatch):
    """round 6: the applies count the re-reads below an ordinal through a
    coarse index of the plan's re-read list (k_rr_index, built for lists of
    64 or more and stamped with its plan). 8 % stays rows over 200 K files
    (hundreds to thousands of re-reads; at chunk size 1 the first stays row
    would be read by every later step, a loop, not re-reads): every link and both counts
    against the oracle with the index and without it (SDCAS_RR_INDEX=0), on
    the world-of-one path and on the staged path (combine, resolve, stays,
    plan, apply); and a plan whose index was replaced by a later plan's on
    the same stages (stamps differ) falls back to the full search"""
    from spacedrive_amd.dist_dedup import DeviceStages
    n = 200_000
    keys, has, status, existing = make_corpus(4242 + chunk_size, n, pool=n // 4, p_none=0.04, p_err=0.04)
    want, wc, wl = oracle.identifier_dedup(keys, has, status, chunk_size, existing)
    (k, h, s, ids), = shard(keys, has, status, existing, 1, device="cuda")[0]
    ek = torch.from_numpy(np.ascontiguousarray(existing).view(np.int64)).cuda()
    eids = torch.arange(existing.size, dtype=torch.int64, device="cuda")
    keys2, has2, status2, _ = make_corpus(99 + chunk_size, n, pool=n // 4, p_none=0.2, p_err=0.0)
    (_, h2, s2, ids2), = shard(keys2, has2, status2, existing, 1, device="cuda")[0]
    for flag in ("1", "0"):
        monkeypatch.setenv("SDCAS_RR_INDEX", flag)
        st = DeviceStages(eng)
        link, cnt = st.local(k, h, s, ids, chunk_size, ek, eids)
        assert np.array_equal(link.cpu().numpy(), want), flag
        assert tuple(cnt.tolist()) == (wc, wl), flag
        rec, slot, _ = st.combine(k, h, s, ids, 1)
        erec, _, _ = st.combine(ek, None, None, eids, 1)
        ans = st.resolve(rec, erec)
        stays, _ = st.stays(h, s, ids, n)
        plan = st.plan(stays, n, chunk_size)
        if flag == "1":
            assert int(plan[1]) >= 64 and int(plan[9]) != 0  # indexed
            stays2, _ = st.stays(h2, s2, ids2, n)
            plan2 = st.plan(stays2, n, chunk_size)  # the workspace's index is plan2's now
            assert int(plan2[9]) not in (0, int(plan[9]))
        else:
            assert int(plan[9]) == 0
        link, cnt = st.apply(ids, slot, ans, chunk_size, plan)
        assert np.array_equal(link.cpu().numpy(), want), flag
        assert tuple(cnt.tolist()) == (wc, wl), flag


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1024 * 7 + 1, 1024 * 7 + 63, 1024 * 7 + 65, 1024 * 29 + 1000, 1024 * 300 + 17])
@pytest.mark.parametrize("chunk_size", [100, 7])
def test_device_local_stays_in_partial_last_tile(eng, oracle, n, chunk_size):
    """stays rows (no cas_id, and errored) in the last, partial stays tile
    (kStayTile = 1024 rows, dist_dedup.hip): the insert counts them per tile,
    the writer places them after the tiles before, the plan walk sums every
    tile — the round-5 hazard was those three disagreeing on the tile (the
    counts are kept per tile and per group of 64 tiles: n = 300 K spans five
    groups). The
    last rows are stays rows at step ends, so a miscounted tile shows as
    DEFERRED or missing re-reads; every link, both counts and the plan's
    steps / rows / rereads against the oracle's literal step loop"""
    from spacedrive_amd.dist_dedup import DeviceStages
    keys, has, status, existing = make_corpus(1000 + n, n, pool=max(50, n // 5), p_none=0.05, p_err=0.05)
    tail = n - (n // 1024) * 1024
    lo = n - tail
    has[lo:] = 1
    status[lo:] = 0
    # in the partial tile: rows without cas_id and errored rows, among them the
    # very last row and rows at step ends
    pick = np.unique(np.concatenate([[n - 1, n - 2, lo], np.arange(lo + chunk_size - 1, n, chunk_size),
                                     lo + np.random.default_rng(n).integers(0, tail, max(1, tail // 8))]))
    pick = pick[(pick >= lo) & (pick < n)]
    has[pick[::2]] = 0
    status[pick[1::2]] = 5
    st = DeviceStages(eng)
    header = torch.zeros(12, dtype=torch.int64, device="cuda")
    (k, h, s, ids), = shard(keys, has, status, existing, 1, device="cuda")[0]
    ek = torch.from_numpy(existing.view(np.int64)).cuda()
    eids = torch.arange(existing.size, dtype=torch.int64, device="cuda")
    want, wc, wl, ww = oracle.identifier_job(keys, has, status, chunk_size, existing)
    for _ in range(2):  # the second call over a dirty workspace
        link, cnt = st.local(k, h, s, ids, chunk_size, ek, eids, header=header)
        assert np.array_equal(link.cpu().numpy(), want)
        assert tuple(cnt.tolist()) == (wc, wl)
        hd = header.cpu().numpy()
        assert (int(hd[2]), int(hd[3]), int(hd[8])) == (ww["steps"], ww["rows"], ww["rereads"])
    got, gc, gl, gw = eng.identifier_dedup_window(keys, has, status, chunk_size, existing, 0, False)
    assert np.array_equal(got, want) and (gc, gl) == (wc, wl) and gw == ww


@pytest.mark.gpu
@pytest.mark.parametrize("R", [1, 3])
def test_device_stages_top32_collisions(eng, oracle, R):
    """keys sharing their top 32 bits interleave in the combine's sort and
    split into several records; the links still equal the oracle's"""
    from spacedrive_amd.dist_dedup import DeviceStages
    keys, has, status, existing = collision_corpus()
    shards, ex = shard(keys, has, status, existing, R, device="cuda")
    st = DeviceStages(eng)
    links, c, l = dedup_virtual(lambda r: st, shards, 100, ex)
    want, wc, wl = oracle.identifier_dedup(keys, has, status, 100, existing)
    assert np.array_equal(np.concatenate([x.cpu().numpy() for x in links]), want)
    assert (c, l) == (wc, wl)


@pytest.mark.gpu
@pytest.mark.parametrize("R", [1, 4])
def test_device_stages_clustered_keys_wrap(eng, oracle, R):
    """the resolve table's home slot is the key's top bits: keys packed at the
    top of the key space (and at its bottom) make long probe chains that wrap
    past the table's end; the links still equal the oracle's"""
    from spacedrive_amd.dist_dedup import DeviceStages
    rng = np.random.default_rng(23)
    top = (np.uint64(2**64 - 2**20) + rng.integers(0, 2**20 - 1, 3000, dtype=np.uint64)).astype(np.uint64)
    low = rng.integers(0, 2**16, 1000, dtype=np.uint64)
    pool = np.concatenate([top, low, np.array([2**64 - 1, 0], np.uint64)])
    keys = pool[rng.integers(0, pool.size, 12000)]
    has = (rng.random(keys.size) > 0.02).astype(np.uint8)
    status = np.where(rng.random(keys.size) < 0.01, 5, 0).astype(np.int32)
    existing = pool[rng.integers(0, pool.size, 500)]
    shards, ex = shard(keys, has, status, existing, R, device="cuda")
    st = DeviceStages(eng)
    links, c, l = dedup_virtual(lambda r: st, shards, 100, ex)
    want, wc, wl = oracle.identifier_dedup(keys, has, status, 100, existing)
    assert np.array_equal(np.concatenate([x.cpu().numpy() for x in links]), want)
    assert (c, l) == (wc, wl)


@pytest.mark.gpu
def test_device_stages_empty_and_degenerate(eng, oracle):
    from spacedrive_amd.dist_dedup import DeviceStages
    st = DeviceStages(eng)
    # a rank with no files, a rank whose files all lack cas_ids or failed
    keys = np.array([5, 5, 6, 5, 7, 7], np.uint64)
    has = np.array([1, 0, 1, 1, 0, 1], np.uint8)
    status = np.array([0, 0, 2, 0, 0, 0], np.int32)
    shards, ex = shard(keys, has, status, np.zeros(0, np.uint64), 3, device="cuda")
    shards = [shards[0], shards[1], shards[2]]
    empty = shard(np.zeros(0, np.uint64), np.zeros(0, np.uint8), np.zeros(0, np.int32), np.zeros(0, np.uint64), 1,
                  device="cuda")[0][0]
    # ordinals stay global: splice an empty rank in front
    links, c, l = dedup_virtual(lambda r: st, [empty] + shards, 2)
    want, wc, wl = oracle.identifier_dedup(keys, has, status, 2, np.zeros(0, np.uint64))
    assert np.array_equal(np.concatenate([x.cpu().numpy() for x in links]), want)
    assert (c, l) == (wc, wl)


def _mismatches(got, want, keys, has, status, k=8):
    """the first k mismatching files, for an assertion message"""
    bad = np.nonzero(got != want)[0]
    rows = [f"{bad.size} mismatches"]
    for b in bad[:k]:
        first = int(np.nonzero(keys == keys[b])[0][0])
        rows.append(f"i={b} key={int(keys[b]):016x} has={int(has[b])} status={int(status[b])} got={got[b]} "
                    f"want={want[b]} first_with_key={first}")
    return "\n".join(rows)


@pytest.mark.gpu
def test_rccl_world1(eng, oracle):
    """the real collective path (backend nccl = RCCL) at world size 1"""
    import torch.distributed as dist

    from spacedrive_amd.dist_dedup import DeviceStages, identifier_dedup_distributed
    keys, has, status, existing = make_corpus(77, 30000)
    (k, h, s, ids), = shard(keys, has, status, existing, 1, device="cuda")[0]
    ek = torch.from_numpy(existing.view(np.int64)).cuda()
    eids = torch.arange(existing.size, dtype=torch.int64, device="cuda")
    store = dist.HashStore()
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        stages = DeviceStages(eng)
        link, c, l = identifier_dedup_distributed(stages, k, h, s, ids, 100, ek, eids)
        # the same with the counts left on the device (no host wait in the call)
        link2, cnt = identifier_dedup_distributed(stages, k, h, s, ids, 100, ek, eids, counts_on_device=True)
    finally:
        dist.destroy_process_group()
    want, wc, wl = oracle.identifier_dedup(keys, has, status, 100, existing)
    got = link.cpu().numpy()
    assert np.array_equal(got, want), _mismatches(got, want, keys, has, status)
    assert (c, l) == (wc, wl)
    assert cnt.is_cuda and cnt.tolist() == [wc, wl]
    assert np.array_equal(link2.cpu().numpy(), want)


@pytest.mark.gpu
@pytest.mark.parametrize("table", ["idx", "idx-r0", "idx-r1", "idx-r8", "idx-c0", "idx-xslot", "idx-pplain", "idx4",
                                   "kv"])
@pytest.mark.parametrize("corpus,chunk_size", [("default", 100), ("default", 7), ("default", 1),
                                               ("collisions", 100), ("clustered", 100)])
def test_device_local_vs_oracle(eng, oracle, corpus, chunk_size, table, monkeypatch):
    """the fused single-rank path (sdcas_dev_dedup_local: no combine, files and
    existing Objects straight into the resolve table) against the oracle, with
    every table: the compact u32 table (the default; since round 5 the
    insert also counts the stays rows per 1024-row tile, five launches),
    the same table behind round 4's eight launches, round 3's 16-byte kv
    table; the default table's apply with 0 (the grid-stride form), 1 and 8
    files per thread beside the default 4 (`idx-rN`, SDCAS_APPLY_R), every
    first ordinal read instead of taken from the index (`idx-c0`), the
    existing Objects' minima by table slot instead of by claiming Object
    (`idx-xslot`, round 5's form), the files' insert probing with ordinary
    loads (`idx-pplain`, SDCAS_PROBE=plain, round 6's A/B); and the
    existing Objects passed in DB order and shuffled (their DB indices then
    not ascending: the first Object is the lowest DB index, not the first
    entry)"""
    from spacedrive_amd.dist_dedup import DeviceStages
    table, _, knob = table.partition("-")
    monkeypatch.setenv("SDCAS_DEDUP_TABLE", table)
    if knob:
        monkeypatch.setenv({"r": "SDCAS_APPLY_R", "c": "SDCAS_CONTIG", "x": "SDCAS_EXIST_MIN",
                            "p": "SDCAS_PROBE"}[knob[0]], knob[1:])
    if corpus == "default":
        keys, has, status, existing = make_corpus(91, 40000, pool=6000)
        keys[:2] = np.uint64(2**64 - 1)  # the table's empty marker is a legal key
        existing = np.concatenate([existing, np.array([2**64 - 1], np.uint64)])
    elif corpus == "collisions":
        keys, has, status, existing = collision_corpus()
    else:
        rng = np.random.default_rng(29)
        pool = np.concatenate([(np.uint64(2**64 - 2**20) + rng.integers(0, 2**20 - 1, 3000, dtype=np.uint64)),
                               rng.integers(0, 2**16, 1000, dtype=np.uint64),
                               np.array([2**64 - 1, 0], np.uint64)]).astype(np.uint64)
        keys = pool[rng.integers(0, pool.size, 12000)]
        has = (rng.random(keys.size) > 0.02).astype(np.uint8)
        status = np.where(rng.random(keys.size) < 0.01, 5, 0).astype(np.int32)
        existing = pool[rng.integers(0, pool.size, 500)]
    (k, h, s, ids), = shard(keys, has, status, existing, 1, device="cuda")[0]
    ek = torch.from_numpy(existing.view(np.int64)).cuda()
    eids = torch.arange(existing.size, dtype=torch.int64, device="cuda")
    st = DeviceStages(eng)
    # dirty the workspace first: a larger batch with dense stays rows leaves
    # its stays list and tile counts behind (round 5: a tiled insert counted
    # its last tile's lanes past n as stays rows, and the walk read that
    # call's stale entries)
    dk, dh, ds, _ = make_corpus(3, 3 * keys.size + 1000, p_none=0.3, p_err=0.3)
    (dk, dh, ds, dids), = shard(dk, dh, ds, existing, 1, device="cuda")[0]
    st.local(dk, dh, ds, dids, chunk_size)
    order = torch.from_numpy(np.random.default_rng(5).permutation(existing.size)).cuda()
    for with_existing in (True, "shuffled", False):
        e_k, e_i = (ek, eids) if with_existing is True else (ek[order], eids[order])
        link, cnt = st.local(k, h, s, ids, chunk_size, e_k if with_existing else None,
                             e_i if with_existing else None)
        want, wc, wl = oracle.identifier_dedup(keys, has, status, chunk_size,
                                               existing if with_existing else np.zeros(0, np.uint64))
        assert np.array_equal(link.cpu().numpy(), want)
        assert tuple(cnt.tolist()) == (wc, wl)
    # degenerate: no files; files without cas_ids or with errors only
    z = torch.zeros(0, dtype=torch.int64, device="cuda")
    link, cnt = st.local(z, z.to(torch.uint8), z.to(torch.int32), z, 100)
    assert link.numel() == 0 and cnt.tolist() == [0, 0]
    k2 = torch.tensor([5, 5, 6], dtype=torch.int64, device="cuda")
    h2 = torch.tensor([0, 1, 1], dtype=torch.uint8, device="cuda")
    s2 = torch.tensor([0, 3, 3], dtype=torch.int32, device="cuda")
    i2 = torch.arange(3, dtype=torch.int64, device="cuda")
    link, cnt = st.local(k2, h2, s2, i2, 100)
    want, wc, wl = oracle.identifier_dedup(np.array([5, 5, 6], np.uint64), np.array([0, 1, 1], np.uint8),
                                           np.array([0, 3, 3], np.int32), 100, np.zeros(0, np.uint64))
    assert np.array_equal(link.cpu().numpy(), want) and tuple(cnt.tolist()) == (wc, wl)


def _plan_cases(count, seed0=0):
    """small dense cases of the step plan: every chunk size from 1, stays rows
    at step ends, budgets above and below what the rows need, windows"""
    for seed in range(seed0, seed0 + count):
        rng = np.random.default_rng(seed)
        n = int(rng.integers(1, 60))
        cs = int(rng.choice([1, 2, 3, 4, 7, 10, 100]))
        pool = rng.integers(0, 2**64, max(2, n // 3), dtype=np.uint64)
        keys = pool[rng.integers(0, pool.size, n)]
        has = (rng.random(n) > rng.random() * 0.5).astype(np.uint8)
        status = np.where(rng.random(n) < rng.random() * 0.4, 5, 0).astype(np.int32)
        existing = pool[rng.integers(0, pool.size, int(rng.integers(0, 4)))]
        for max_steps, more in ((0, False), (int(rng.integers(1, 2 * n + 2)), False),
                                (int(rng.integers(1, 2 * n + 2)), True), (0, True)):
            yield keys, has, status, existing, cs, max_steps, more



@pytest.mark.gpu
def test_device_local_ordinals_not_contiguous(eng, oracle, monkeypatch):
    """the fused apply takes a key's first ordinal from its first file's index
    only when every ordinal is ids[0] + index: offset ordinals (a rank's
    share) take the shortcut, one moved ordinal must send the apply back to
    reading them (checked against the reading path, SDCAS_CONTIG=0)"""
    from spacedrive_amd.dist_dedup import DeviceStages
    keys, has, status, existing = make_corpus(17, 30000, pool=3000)
    (k, h, s, ids), = shard(keys, has, status, existing, 1, device="cuda")[0]
    st = DeviceStages(eng)
    # a first file of a duplicated key: its ordinal is what its key's other files link to
    _, first, counts = np.unique(keys, return_index=True, return_counts=True)
    f = int(first[np.argmax(counts)])
    for name, d_ids in (("offset", ids + 1000), ("moved", ids.clone())):
        if name == "moved":
            d_ids[f] += 5
        monkeypatch.setenv("SDCAS_CONTIG", "1")
        got, gc = st.local(k, h, s, d_ids, 100)
        got = got.cpu().numpy().copy()
        monkeypatch.setenv("SDCAS_CONTIG", "0")
        ref, rc = st.local(k, h, s, d_ids, 100)
        assert np.array_equal(got, ref.cpu().numpy()), name
        assert gc.tolist() == rc.tolist(), name
    want, _, _ = oracle.identifier_dedup(keys, has, status, 100, np.zeros(0, np.uint64))
    got, _ = st.local(k, h, s, ids, 100)
    assert np.array_equal(got.cpu().numpy(), want)

@pytest.mark.gpu
def test_device_step_plan_matches_literal_step_loop(eng, oracle):
    """the device's plan (k_plan_walk) through sdcas_dedup_window and through
    sdcas_dev_dedup_local, against the oracle's literal cursor loop"""
    from spacedrive_amd.dist_dedup import DeviceStages
    st = DeviceStages(eng)
    header = torch.zeros(12, dtype=torch.int64, device="cuda")
    for keys, has, status, existing, cs, max_steps, more in _plan_cases(300):
        want, wc, wl, ww = oracle.identifier_job(keys, has, status, cs, existing, max_steps, more)
        case = (keys.size, cs, max_steps, more)
        got, gc, gl, gw = eng.identifier_dedup_window(keys, has, status, cs, existing, max_steps, more)
        assert np.array_equal(got, want) and (gc, gl) == (wc, wl), case
        assert gw == ww, case
        (k, h, s, ids), = shard(keys, has, status, existing, 1, device="cuda")[0]
        ek = torch.from_numpy(existing.view(np.int64)).cuda()
        eids = torch.arange(existing.size, dtype=torch.int64, device="cuda")
        link, cnt = st.local(k, h, s, ids, cs, ek, eids, keys.size, max_steps, more, header=header)
        assert np.array_equal(link.cpu().numpy(), want) and tuple(cnt.tolist()) == (wc, wl), case
        hd = header.cpu().numpy()
        assert (int(hd[2]), int(hd[3]), int(hd[8])) == (ww["steps"], ww["rows"], ww["rereads"]), case


@pytest.mark.gpu
@pytest.mark.parametrize("R,chunk_size", [(1, 100), (3, 100), (8, 7), (2, 1)])
def test_device_stages_dense_stays_vs_oracle(eng, oracle, R, chunk_size):
    """a corpus where many rows stay orphans (20 % errors, 20 % without a
    cas_id), so most steps re-read their predecessor's last row: the device
    stays + plan + combine + resolve + apply over R virtual ranks"""
    from spacedrive_amd.dist_dedup import DeviceStages
    keys, has, status, existing = make_corpus(300 + R, 30000, pool=3000, p_none=0.2, p_err=0.2)
    want, wc, wl, ww = oracle.identifier_job(keys, has, status, chunk_size, existing)
    assert ww["rereads"] > 10 or chunk_size == 1
    shards, ex = shard(keys, has, status, existing, R, device="cuda")
    st = DeviceStages(eng)
    links, c, l = dedup_virtual(lambda r: st, shards, chunk_size, ex)
    got = np.concatenate([x.cpu().numpy() for x in links])
    assert np.array_equal(got, want)
    assert (c, l) == (wc, wl)


@pytest.mark.gpu
@pytest.mark.parametrize("m", [1, 2, 300, 4096, 4097, 50_000])
def test_device_plan_sorts_gathered_stays(eng, oracle, m):
    """sdcas_dev_dedup_plan over every rank's stays ordinals concatenated in
    no order, padded with all-ones entries: up to 4096 entries one
    workgroup's bitonic sort, more a bitmap over the job's ordinals read back
    in order (round 5; round 4: hipCUB's radix sort) — the plan equals the
    one from the sorted list, and the oracle's for a job whose stays rows
    are exactly those ordinals"""
    from spacedrive_amd import _native as N
    from spacedrive_amd.dist_dedup import DeviceStages
    rng = np.random.default_rng(m)
    n_total = max(2 * m, 1000) + 17
    stays = np.sort(rng.choice(n_total, m, replace=False)).astype(np.int64)
    shuffled = np.concatenate([rng.permutation(stays), np.full(m // 7 + 3, -1, np.int64)])
    rng.shuffle(shuffled)
    st = DeviceStages(eng)
    for cs, max_steps, more in ((100, 0, False), (7, 0, True), (100, 3, False), (1, 0, False)):
        got = st.plan(torch.from_numpy(shuffled).cuda(), n_total, cs, max_steps, more).cpu().numpy()
        ref = st.plan(torch.from_numpy(np.concatenate([stays, np.full(4, -1, np.int64)])).cuda(), n_total, cs,
                      max_steps, more).cpu().numpy()
        h = N.SDCAS_PLAN_HEADER_WORDS
        nr = int(got[1])
        # word 9: the stamp of the re-read list's coarse index, one per plan built (0: none)
        assert (got[9] != 0) == (nr >= 64) and (ref[9] != 0) == (nr >= 64)
        got[9] = ref[9] = 0
        assert np.array_equal(got[:h], ref[:h]) and np.array_equal(got[h:h + nr], ref[h:h + nr]), (cs, max_steps)
        # the oracle: rows without a cas_id at exactly those ordinals
        has = np.ones(n_total, np.uint8)
        has[stays] = 0
        keys = rng.integers(0, 2**64, n_total, dtype=np.uint64)
        _, _, _, ww = oracle.identifier_job(keys, has, None, cs, np.zeros(0, np.uint64), max_steps, more)
        assert (int(got[2]), int(got[3]), int(got[8])) == (ww["steps"], ww["rows"], ww["rereads"]), (cs, max_steps)


# ---- the piece split of big-file checksums (spacedrive_amd/dist_checksum.py) ----

@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_split_pieces_covers_every_piece_once(world):
    from spacedrive_amd.dist_checksum import MiB, split_pieces
    rng = np.random.default_rng(world)
    sizes = [int(x) for x in rng.integers(MiB + 1, 40 * MiB, 13)] + [4 * MiB, MiB + 1]
    parts = split_pieces(sizes, world)
    seen = {}
    for r, segs in enumerate(parts):
        for f, off, ln in segs:
            assert off % MiB == 0 and ln > 0 and off + ln <= sizes[f]
            assert ln % MiB == 0 or off + ln == sizes[f]  # whole pieces, or the file's tail
            for q in range(off // MiB, (off + ln + MiB - 1) // MiB):
                assert (f, q) not in seen
                seen[(f, q)] = r
    total = sum((s + MiB - 1) // MiB for s in sizes)
    assert len(seen) == total
    counts = [sum((ln + MiB - 1) // MiB for _, _, ln in segs) for segs in parts]
    assert max(counts) - min(counts) <= 1


@pytest.mark.gpu
def test_owner_resolve_with_one_owners_keys(eng, oracle):
    """what an owner receives at 8 ranks: keys whose top 12 bits all lie in
    one eighth of their range (dd_owner). The owner's table must spread them
    over all its slots — with the home slot taken from the owner bits they
    crowded into an eighth of the table and a resolve took 1000x longer. The
    answers are the per-key minima (first ordinal), and the clustered resolve
    runs about as fast as a uniform one."""
    import time
    from spacedrive_amd.dist_dedup import DeviceStages
    rng = np.random.default_rng(21)
    n, pool = 400_000, 300_000
    base = rng.integers(0, 1 << 63, pool, dtype=np.uint64) * np.uint64(2) + np.uint64(1)
    times = {}
    for name, shift in (("uniform", 0), ("one owner of 8", 3)):
        keys_pool = base >> np.uint64(shift)  # top 3 bits zero: owner 0 of 8
        pick = rng.integers(0, pool, n)
        keys = keys_pool[pick]
        ords = np.arange(n, dtype=np.int64)
        frec = torch.from_numpy(np.stack([keys.view(np.int64), ords], 1)).cuda()
        st = DeviceStages(eng, 0)
        st.resolve(frec, frec[:0])  # warm: table allocation
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            res = st.resolve(frec, frec[:0])
        torch.cuda.synchronize()
        times[name] = (time.perf_counter() - t0) / 3
        first = {}
        for k, o in zip(keys.tolist(), ords.tolist()):
            first.setdefault(k, o)
        want = np.array([first[k] for k in keys.tolist()], np.int64)
        assert (res.cpu().numpy() == want).all(), name
    assert times["one owner of 8"] < 5 * times["uniform"] + 0.002, times


def _subgroup_worker(rank, world, port, outdir):
    import torch.distributed as dist

    from spacedrive_amd import dist_dedup as D
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        sub = dist.new_group(ranks=[0, 1])
        sub2 = dist.new_group(ranks=[1, 2])
        member = rank in (0, 1)
        real = dist.get_backend
        # stand in for an RCCL subgroup on its members (the meta group is
        # only built for a non-gloo group; gloo is all this container has).
        # A rank outside `sub` holds torch's NON_GROUP_MEMBER for it, on
        # which get_backend raises: it is never asked
        D.dist.get_backend = lambda g=None: "nccl" if member and g is sub else real(g)
        res = []
        if member:
            try:
                D._meta_group(sub)
                res.append("no error")
            except RuntimeError as e:
                res.append("prepare_meta_group" in str(e))
        else:
            try:
                D.prepare_meta_group(sub)  # the handle names no ranks here
                res.append("no error")
            except ValueError as e:
                res.append("ranks=" in str(e))
        # every rank of the default group, members by handle, the other by ranks
        g1 = D.prepare_meta_group(sub) if member else D.prepare_meta_group(ranks=[0, 1])
        g2 = D.prepare_meta_group(sub2) if rank in (1, 2) else D.prepare_meta_group(ranks=[2, 1])
        res.append(g1 is not g2)  # two subgroups, two meta groups (on the non-member too)
        if member:
            g = D._meta_group(sub)
            res.append(g is g1 and real(g) == "gloo" and dist.get_world_size(g) == 2)
            t = torch.tensor([rank + 1])
            dist.all_reduce(t, group=g)
            res.append(int(t) == 3)
        D.dist.get_backend = real
        np.save(os.path.join(outdir, f"r{rank}.npy"), np.array(res, dtype=object), allow_pickle=True)
    finally:
        dist.destroy_process_group()


def test_meta_group_of_a_subgroup():
    """the host-integer group of a strict subgroup: asking for it before it
    exists raises (dist.new_group would hang: it is collective over every
    rank); prepare_meta_group on every rank creates it — members by the
    subgroup's handle, a rank outside it by the ranks (its handle names none,
    and asking with it raises instead of leaving the members blocked)"""
    import torch.multiprocessing as mp
    world = 3
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_subgroup_worker, args=(world, _free_port(), d), nprocs=world, join=True,
                           start_method="spawn")
        res = [list(np.load(os.path.join(d, f"r{r}.npy"), allow_pickle=True)) for r in range(world)]
    assert res[0] == [True, True, True, True] and res[1] == [True, True, True, True] and res[2] == [True, True]


@pytest.mark.gpu
@pytest.mark.parametrize("combine", ["tile", "tile-idx", "tile-kv", "tile-split", "tile-r0", "tile-r1", "hash",
                                     "hash-idx"])
@pytest.mark.parametrize("R,chunk_size", [(2, 100), (8, 100), (5, 7)])
def test_device_bucket_protocol_vs_oracle(eng, oracle, R, chunk_size, combine, monkeypatch):
    """the bucket protocol's device stages (combine_buckets -> equal-split
    exchange -> resolve_buckets -> apply) over R virtual ranks with existing
    Objects, both combines — round 6's per-tile LDS pre-aggregation (the
    default: a key may take one record per 2048-file tile) and round 5's
    global hash table (SDCAS_COMBINE=hash, one record per key) — and every
    resolve: the owner's u32 claim table folding the other records' values
    into the claiming record (the default), the same table with per-slot side
    minima (SDCAS_RESOLVE=idx), round 5's 16-byte (key, minimum) entries
    (SDCAS_RESOLVE=kv) and round 4's tables sized from the buckets' capacity
    (SDCAS_RESOLVE=split); the
    apply with 4 files per thread (the default), round 5's grid-stride apply
    (SDCAS_APPLY_R=0) and one file per thread (1); then buckets one record too
    small, which must raise the overflow flag (the caller then reruns the
    exact stages)"""
    from spacedrive_amd.dist_dedup import DeviceStages
    from tests._dist_stages import dedup_virtual_buckets
    comb, _, knob = combine.partition("-")
    monkeypatch.setenv("SDCAS_COMBINE", comb)
    if knob in ("split", "kv", "idx"):
        monkeypatch.setenv("SDCAS_RESOLVE", knob)
    elif knob.startswith("r"):
        monkeypatch.setenv("SDCAS_APPLY_R", knob[1:])
    keys, has, status, existing = make_corpus(700 + R, 24000, pool=5000, p_none=0.05, p_err=0.05)
    # the all-ones key (the tables' empty marker, a legal cas key) on several
    # files and ranks, once with an existing Object
    keys[[5, 4000, 17000]] = np.uint64(2**64 - 1)
    if chunk_size == 100:
        existing = np.concatenate([existing, np.array([2**64 - 1], np.uint64)])
    want, wc, wl = oracle.identifier_dedup(keys, has, status, chunk_size, existing)
    shards, ex = shard(keys, has, status, existing, R, device="cuda")
    st = DeviceStages(eng)
    n = max(int(s[3].numel()) for s in shards)
    caps = (n + 1, max(int(e[0].numel()) for e in ex) + 1)
    links, c, l, over = dedup_virtual_buckets(lambda r: st, shards, chunk_size, ex, caps)
    assert not over
    assert np.array_equal(np.concatenate([x.cpu().numpy() for x in links]), want)
    assert (c, l) == (wc, wl)
    # the largest bucket's fill, then one less capacity: overflow
    fills = []
    for (k, h, s, ids) in shards:
        _, _, cnt, _ = st.combine_buckets(k, h, s, ids, R, caps[0])
        fills.append(int(cnt.max()))
    _, _, _, over = dedup_virtual_buckets(lambda r: st, shards, chunk_size, ex, (max(fills) - 1, caps[1]))
    assert over
