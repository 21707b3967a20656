"""Multi-GPU identifier dedup: the cas_id -> Object group-by of
core/src/object/file_identifier/mod.rs:149-254 over orphan file_paths sharded
across the GPUs of a node, one process per GPU.

The reference runs this group-by 100 files at a time in one process
(file_identifier_job.rs:296-319). In canonical form it
only needs two per-key minima — the first existing Object in DB order and the
lowest orphan ordinal carrying the key — plus a per-file rule, so it shards:

  1. combine   every rank reduces its files to one (key, min ordinal) record
               per distinct key, grouped by owner rank
               (owner = top 12 key bits split into `world` ranges); existing
               Objects likewise to (key, min DB index)
  2. exchange  RCCL all-to-all of both record sets (16 B records)
  3. resolve   the owner answers each file record: -(db+1) or the key's
               global first ordinal
  4. exchange  the answers go back (8 B each, the reverse all-to-all)
  5. apply     every rank links its files: dropped / own Object / existing
               Object / the Object created by the key's first file

The device stages (1, 3, 5) are libsdcas's HIP kernels
(sdcas_dev_dedup_{combine,resolve,apply}; a world of one runs them fused
without the combine, sdcas_dev_dedup_local); the exchanges are
torch.distributed all_to_all_single (backend "nccl" = RCCL over xGMI). The
`stages` object is pluggable only so that the collective protocol can be
exercised with gloo on CPU by the test-suite's numpy stages
(tests/_dist_stages.py); the product path is `DeviceStages`.

Host synchronisations. all_to_all_single needs its split sizes on the host,
so the exact protocol waits for the host three times (the combine's owner
ranges, the received counts, the final totals). The bucket protocol sends
every owner a fixed-capacity bucket instead (equal splits, nothing for the
host to learn) and carries the valid counts on the device; its only host
synchronisation is the final totals, which also carry an overflow flag.
Capacities are agreed from the previous call's largest bucket (all ranks see
the same all-reduced maximum); the first call of a `stages` object, and any
call whose buckets overflow, takes the exact protocol.
"""
from __future__ import annotations

import ctypes
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

from . import _native as N


class DeviceStages:
    """The three device stages through the C ABI, on torch tensors in HBM.

    Every stage runs on a stream of its own, ordered after the caller's
    current stream and before anything the caller enqueues next (torch's
    default stream is the legacy NULL stream, which libsdcas would read as
    "the context's non-blocking stream", so it is never handed over as is).
    """

    def __init__(self, engine, device=None, same_stream=False):
        self.eng = engine
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self.stream = torch.cuda.Stream(self.device)
        # same_stream: enqueue on the caller's current stream when it is a
        # real stream (not the legacy NULL stream) — no cross-stream event
        # wait on either side of every stage (≈ 20 µs each, measured in the
        # C5 step's trace)
        self.same_stream = same_stream

    def _current(self):
        cur = torch.cuda.current_stream(self.device)
        return cur if self.same_stream and cur.cuda_stream else None

    def _enter(self):
        cur = self._current()
        if cur is not None:
            return cur.cuda_stream
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        return self.stream.cuda_stream

    def _leave(self, *tensors):
        if self._current() is not None:
            return
        for t in tensors:
            if t is not None and t.is_cuda:
                t.record_stream(self.stream)
        torch.cuda.current_stream(self.device).wait_stream(self.stream)

    def combine(self, keys, has_key, status, ids, world):
        """-> (rec int64[U, 2], slot int32[n] or None, starts list[world+1])"""
        n = int(ids.numel())
        dev = ids.device
        rec = torch.empty((max(n, 1), 2), dtype=torch.int64, device=dev)
        slot = torch.empty(max(n, 1), dtype=torch.int32, device=dev) if has_key is not None or status is not None \
            or keys is not None else None
        starts = (ctypes.c_uint64 * (world + 1))()
        p = lambda t: t.data_ptr() if t is not None and t.numel() else None
        rc = self.eng.L.sdcas_dev_dedup_combine(self.eng.ctx, p(keys), p(has_key), p(status), p(ids), n,
                                                world, p(rec), p(slot) if slot is not None else None, starts,
                                                self._enter())
        self._leave(keys, has_key, status, ids, rec, slot)
        self.eng._check(rc, "sdcas_dev_dedup_combine")
        st = [int(x) for x in starts]
        return rec[: st[world]], (slot[:n] if slot is not None else None), st

    def resolve(self, frec, erec):
        nf, ne = int(frec.shape[0]), int(erec.shape[0])
        result = torch.empty(max(nf, 1), dtype=torch.int64, device=frec.device)
        p = lambda t: t.data_ptr() if t.numel() else None
        rc = self.eng.L.sdcas_dev_dedup_resolve(self.eng.ctx, p(frec), nf, p(erec), ne, p(result),
                                                self._enter())
        self._leave(frec, erec, result)
        self.eng._check(rc, "sdcas_dev_dedup_resolve")
        return result[:nf]

    def local(self, keys, has_key, status, ids, chunk_size, existing_keys=None, existing_ids=None, n_total=0,
              max_steps=0, more=False, header=None):
        """stays + plan + combine + resolve + apply for a world of one (nothing
        to exchange, so no combine): -> (link int64[n], counts int64[2]) on
        the device; `header` (int64[8] device tensor) receives the plan's header"""
        n = int(ids.numel())
        link = torch.empty(max(n, 1), dtype=torch.int64, device=ids.device)
        counts = torch.zeros(2, dtype=torch.int64, device=ids.device)
        ne = int(existing_keys.numel()) if existing_keys is not None else 0
        p = lambda t: t.data_ptr() if t is not None and t.numel() else None
        rc = self.eng.L.sdcas_dev_dedup_local(self.eng.ctx, p(keys), p(has_key), p(status), p(ids), n,
                                              p(existing_keys) if ne else None, p(existing_ids) if ne else None,
                                              ne, int(chunk_size), int(n_total), int(max_steps), int(bool(more)),
                                              p(link), counts.data_ptr(), p(header), self._enter())
        self._leave(keys, has_key, status, ids, existing_keys, existing_ids, link, counts, header)
        self.eng._check(rc, "sdcas_dev_dedup_local")
        return link[:n], counts

    def stays(self, has_key, status, ids, cap):
        """-> (this rank's stays ordinals int64[cap] padded with -1 (all ones),
        their count int64[1]), on the device"""
        n = int(ids.numel())
        out = torch.empty(max(cap, 1), dtype=torch.int64, device=ids.device)
        count = torch.empty(1, dtype=torch.int64, device=ids.device)
        p = lambda t: t.data_ptr() if t is not None and t.numel() else None
        rc = self.eng.L.sdcas_dev_dedup_stays(self.eng.ctx, p(has_key), p(status), p(ids), n, int(cap), p(out),
                                              count.data_ptr(), self._enter())
        self._leave(has_key, status, ids, out, count)
        self.eng._check(rc, "sdcas_dev_dedup_stays")
        return out[:cap], count

    def plan(self, stays, n_total, chunk_size, max_steps=0, more=False):
        """every rank's stays ordinals (any order, -1 = padding) -> the job's
        step plan int64[SDCAS_PLAN_HEADER_WORDS + len] on the device"""
        m = int(stays.numel())
        plan = torch.empty(N.SDCAS_PLAN_HEADER_WORDS + m, dtype=torch.int64, device=stays.device)
        rc = self.eng.L.sdcas_dev_dedup_plan(self.eng.ctx, stays.data_ptr() if m else None, m, int(n_total),
                                             int(chunk_size), int(max_steps), int(bool(more)), plan.data_ptr(),
                                             self._enter())
        self._leave(stays, plan)
        self.eng._check(rc, "sdcas_dev_dedup_plan")
        return plan

    @property
    def combine_tiles(self):
        """the bucket combine pre-aggregates per 2048-file tile (the default;
        SDCAS_COMBINE=hash: one record per key through the rank's table): its
        buckets hold up to one record per key per tile, more than the exact
        combine's one per key"""
        return os.environ.get("SDCAS_COMBINE", "") != "hash"

    def combine_buckets(self, keys, has_key, status, ids, world, cap, need_slot=True):
        """-> (send int64[world * cap, 2], slot int32[n] or None, counts int64[world],
        overflow int32[1]), all on the device, no host synchronisation"""
        n = int(ids.numel())
        dev = ids.device
        send = torch.empty((max(world * cap, 1), 2), dtype=torch.int64, device=dev)
        slot = torch.empty(max(n, 1), dtype=torch.int32, device=dev) if need_slot else None
        counts = torch.empty(world, dtype=torch.int64, device=dev)
        overflow = torch.empty(1, dtype=torch.int32, device=dev)
        p = lambda t: t.data_ptr() if t is not None and t.numel() else None
        rc = self.eng.L.sdcas_dev_dedup_combine_buckets(self.eng.ctx, p(keys), p(has_key), p(status), p(ids), n,
                                                        world, cap, p(send), p(slot), p(counts), p(overflow),
                                                        self._enter())
        self._leave(keys, has_key, status, ids, send, slot, counts, overflow)
        self.eng._check(rc, "sdcas_dev_dedup_combine_buckets")
        return send[: world * cap], (slot[:n] if slot is not None else None), counts, overflow

    def resolve_buckets(self, frecv, fcap, fcounts, erecv, ecap, ecounts, world):
        """-> result int64[world * fcap] in the received buckets' layout"""
        result = torch.empty(max(world * fcap, 1), dtype=torch.int64, device=frecv.device)
        p = lambda t: t.data_ptr() if t is not None and t.numel() else None
        rc = self.eng.L.sdcas_dev_dedup_resolve_buckets(self.eng.ctx, p(frecv), fcap, p(fcounts), p(erecv),
                                                        ecap, p(ecounts), world, p(result), self._enter())
        self._leave(frecv, fcounts, erecv, ecounts, result)
        self.eng._check(rc, "sdcas_dev_dedup_resolve_buckets")
        return result[: world * fcap]

    def apply(self, ids, slot, result, chunk_size, plan=None):
        """-> (link int64[n], counts int64[2] = (created, linked)) on the device"""
        n = int(ids.numel())
        link = torch.empty(max(n, 1), dtype=torch.int64, device=ids.device)
        counts = torch.zeros(2, dtype=torch.int64, device=ids.device)
        p = lambda t: t.data_ptr() if t is not None and t.numel() else None
        rc = self.eng.L.sdcas_dev_dedup_apply(self.eng.ctx, p(ids), p(slot), n, p(result), int(chunk_size),
                                              p(plan), p(link), counts.data_ptr(), self._enter())
        self._leave(ids, slot, result, plan, link, counts)
        self.eng._check(rc, "sdcas_dev_dedup_apply")
        return link[:n], counts


def _exchange(send, send_counts, group, recv_counts=None):
    """all_to_all of rows grouped by destination rank -> (recv, recv_counts);
    recv_counts, when the caller knows them, saves the counts exchange (and
    its host synchronisation)"""
    dev = send.device
    if recv_counts is None:
        sc = torch.tensor(send_counts, dtype=torch.int64, device=dev)
        rc = torch.empty_like(sc)
        dist.all_to_all_single(rc, sc, group=group)
        recv_counts = [int(x) for x in rc.tolist()]
    recv = send.new_empty((sum(recv_counts),) + tuple(send.shape[1:]))
    dist.all_to_all_single(recv, send.contiguous(), recv_counts, list(send_counts), group=group)
    return recv, recv_counts


_META_GROUPS = {}  # sorted ranks -> the gloo group of host integers over them


def _ranks_of(group):
    return tuple(range(dist.get_world_size())) if group is None else tuple(sorted(dist.get_process_group_ranks(group)))


def prepare_meta_group(group=None, ranks=None):
    """Create the gloo group over `group`'s ranks that carries the host-known
    integers (file and Object counts: exchanging them never waits for the
    device). dist.new_group is collective over the WHOLE default group, so
    for a strict subgroup every rank of the default group must call this
    before the subgroup's first dedup — a member with the subgroup's handle
    (or its ranks), a rank outside it with `ranks` (its handle of the
    subgroup is torch's NON_GROUP_MEMBER, which names no ranks); the default
    group's own is created on its first dedup, which every rank reaches.
    Every rank creates the same group whatever the subgroup's backend, and
    groups are kept by their ranks, so two subgroups never share one."""
    if ranks is None:
        if group is not None and dist.distributed_c10d._rank_not_in_group(group):
            raise ValueError("prepare_meta_group: this rank is outside `group`; pass the subgroup's ranks= instead")
        key = _ranks_of(group)
    else:
        key = tuple(sorted(int(r) for r in ranks))
    if key not in _META_GROUPS:
        _META_GROUPS[key] = dist.new_group(ranks=list(key), backend="gloo")
    return _META_GROUPS[key]


def _meta_group(group):
    if dist.get_backend(group) == "gloo":
        return group
    key = _ranks_of(group)
    if key not in _META_GROUPS:
        if len(key) != dist.get_world_size():
            raise RuntimeError("identifier_dedup_distributed over a subgroup: call "
                               "dist_dedup.prepare_meta_group(group) on every member and "
                               "prepare_meta_group(ranks=...) on every other rank of the default group first "
                               "(dist.new_group is collective over all ranks)")
        _META_GROUPS[key] = dist.new_group(ranks=list(key), backend="gloo")
    return _META_GROUPS[key]


def _meta(n, ne, group):
    """every rank's (files, existing Objects) -> int64[world, 2] on the host"""
    world = dist.get_world_size(group)
    mine = torch.tensor([n, ne], dtype=torch.int64)
    parts = [torch.empty(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(parts, mine, group=_meta_group(group))
    return torch.stack(parts).numpy()


def identifier_dedup_distributed(stages, keys, has_key, status, ids, chunk_size=100,
                                 existing_keys=None, existing_ids=None, group=None, counts_on_device=False,
                                 n_total=0, max_steps=0, more=False):
    """This rank's share of the identifier group-by.

    keys/has_key/status/ids: this rank's orphan file_paths (ids = their global
    ordinals in orphan order, ascending; has_key 0 = cas_id None; status != 0
    = I/O error). existing_keys/existing_ids: this rank's share of the
    library's existing Objects (ids = global DB order; passed on every rank —
    an empty share as a zero-length tensor — or on none). Every rank must call
    this (it is collective). Returns (link int64[n], created, linked): link
    uses sdcas_dedup's encoding with global ordinals (i = creates, j = links
    to the Object created by file j, -(e+1) = existing Object e, INT64_MIN =
    dropped, INT64_MIN + 1 = deferred); created/linked are the node-wide
    totals identifier_job_step returns summed over the job's steps (mod.rs:349).

    The steps (file_identifier_job.rs:180-236; sdcas_job_window): the job's
    orphans are ordinals [0, n_total) (0: the sum of every rank's files),
    the job may run max_steps more steps (0: ceil(n_total / chunk_size)),
    more = further orphans follow ordinal n_total - 1.

    counts_on_device: in a world of one, return (link, counts) with counts an
    int64[2] device tensor (created, linked) instead of two ints, so that the
    call enqueues its work without waiting for it (a pipelined job reads the
    counts when it writes its report). With an exchange the totals are read
    on the host anyway (they carry the bucket overflow flag).
    """
    world = dist.get_world_size(group)
    # a world of one exchanges with itself: its records are already where
    # the collectives would deliver them, so the exchanges are skipped, and
    # without an exchange the combine has nothing to shrink or group: stages
    # that offer the fused single-rank path take it
    if world == 1 and hasattr(stages, "local"):
        stages.last_protocol = "local"
        link, cnt = stages.local(keys, has_key, status, ids, chunk_size, existing_keys, existing_ids,
                                 n_total or int(ids.numel()), max_steps, more)
        if counts_on_device:
            return link, cnt
        c = cnt.tolist()
        return link, int(c[0]), int(c[1])
    n, ne = int(ids.numel()), int(existing_keys.numel()) if existing_keys is not None else 0
    meta = _meta(n, ne, group) if world > 1 else np.array([[n, ne]], np.int64)
    win = dict(n_total=int(n_total) or int(meta[:, 0].sum()), max_steps=int(max_steps), more=bool(more),
               max_n=int(meta[:, 0].max()), max_ne=int(meta[:, 1].max()))
    if existing_keys is not None and int(meta[:, 1].sum()) == 0:
        existing_keys = existing_ids = None  # nobody holds an existing Object: nothing to exchange for them
    if world > 1 and hasattr(stages, "combine_buckets"):
        stages.last_protocol = "buckets"
        out = _dedup_buckets(stages, world, keys, has_key, status, ids, chunk_size, existing_keys,
                             existing_ids, group, win)
        if out is not None:
            return out
        stages.last_protocol = "buckets-overflow"
    else:
        stages.last_protocol = "exact"
    return _dedup_exact(stages, world, keys, has_key, status, ids, chunk_size, existing_keys, existing_ids, group,
                        win)


def _cap(fill, n_prev, n_now):
    """a bucket capacity for n_now items from a fill seen at n_prev items"""
    return int(fill * max(1.0, n_now / max(n_prev, 1)) * 1.125) + 256


def _caps(stages, world, win, has_ex):
    """(file, existing, stays) bucket capacities, identical on every rank
    (they follow from all-gathered counts and all-reduced fills): the last
    call's largest buckets scaled to this call's largest share, or — on a
    stages object's first call — an even split of the largest share (owners
    are key ranges of uniform BLAKE3 output) with 12.5 % + 256 headroom"""
    forced = stages.__dict__.pop("force_caps", None)  # tests: one call's capacities chosen by the caller
    if forced is not None:
        return forced[0], forced[1] if has_ex else 0, forced[2] if len(forced) > 2 else 256
    seen = getattr(stages, "bucket_seen", None)
    if seen is None:
        f = _cap(win["max_n"] / world, 1, 1)
        e = _cap(win["max_ne"] / world, 1, 1) if has_ex else 0
        s = 256
    else:
        f = _cap(seen["fill_f"], seen["max_n"], win["max_n"])
        e = _cap(max(seen["fill_e"], 0), seen["max_ne"], win["max_ne"]) if has_ex else 0
        s = _cap(seen["fill_s"], seen["max_n"], win["max_n"])
    return f, e, s


def _learn(stages, win, fill_f, fill_e, fill_s):
    """what this call's buckets held (all-reduced maxima), for the next call"""
    stages.bucket_seen = dict(fill_f=int(fill_f), fill_e=int(fill_e), fill_s=int(fill_s), max_n=win["max_n"],
                              max_ne=win["max_ne"])
    f, e, _ = _caps(stages, 1, win, True)
    stages.bucket_caps = (f, e)  # (reported by the bench; the next call rescales)


def _plan(stages, has_key, status, ids, chunk_size, win, group, world, cap, exact=False):
    """the job's step plan from every rank's stays rows: an equal-split
    all-gather of cap ordinals per rank. -> (plan or None, this rank's stays
    count (device int64[1]))"""
    if has_key is None and status is None and not win["more"] and not win["max_steps"]:
        return None, None  # no stays rows and every row within the job's steps: fixed chunks
    st, cnt = stages.stays(has_key, status, ids, cap)
    if exact:
        cs = [torch.empty_like(cnt) for _ in range(world)]
        dist.all_gather(cs, cnt, group=group)
        cap2 = max(1, max(int(c.item()) for c in cs))
        if cap2 > cap:
            st, cnt = stages.stays(has_key, status, ids, cap2)
            cap = cap2
    parts = [torch.empty_like(st) for _ in range(world)]
    dist.all_gather(parts, st.contiguous(), group=group)
    return stages.plan(torch.cat(parts), win["n_total"], chunk_size, win["max_steps"], win["more"]), cnt


def _dedup_exact(stages, world, keys, has_key, status, ids, chunk_size, existing_keys, existing_ids, group, win):
    solo = world == 1
    plan, scnt = _plan(stages, has_key, status, ids, chunk_size, win, group, world, 256, exact=True)
    rec, slot, starts = stages.combine(keys, has_key, status, ids, world)
    counts = [starts[r + 1] - starts[r] for r in range(world)]
    ecounts = [0] * world
    if existing_keys is not None:
        # collective: every rank passes its (possibly empty) share, or none does
        if existing_keys.numel():
            erec, _, estarts = stages.combine(existing_keys, None, None, existing_ids, world)
            ecounts = [estarts[r + 1] - estarts[r] for r in range(world)]
        else:
            erec = rec.new_empty((0, 2))
    if solo:
        frecv, fcounts = rec, counts
        erecv = erec if existing_keys is not None else rec.new_empty((0, 2))
    elif existing_keys is not None:
        # one counts exchange for both record streams: rank r's pair is
        # (file records, existing records) bound for r -- one host sync, not two
        sc = torch.tensor([c for r in range(world) for c in (counts[r], ecounts[r])],
                          dtype=torch.int64, device=rec.device)
        rc = torch.empty_like(sc)
        dist.all_to_all_single(rc, sc, group=group)
        pairs = rc.view(world, 2).tolist()
        frecv, fcounts = _exchange(rec, counts, group, recv_counts=[int(a) for a, _ in pairs])
        erecv = _exchange(erec, ecounts, group, recv_counts=[int(b) for _, b in pairs])[0]
    else:
        frecv, fcounts = _exchange(rec, counts, group)
        erecv = rec.new_empty((0, 2))
    answer = stages.resolve(frecv, erecv)
    # the answers retrace the file records' route: this rank receives back
    # exactly what it sent
    back = answer if solo else _exchange(answer, fcounts, group, recv_counts=counts)[0]
    link, cnt = stages.apply(ids, slot, back, chunk_size, plan)
    if solo:
        c = cnt.tolist()
        return link, int(c[0]), int(c[1])
    # totals, and the node's largest buckets for the next call's capacities
    fills = torch.stack([torch.tensor(max(counts), dtype=torch.int64),
                         torch.tensor(max(ecounts) if existing_keys is not None else -1, dtype=torch.int64),
                         (scnt.cpu()[0] if scnt is not None else torch.tensor(0, dtype=torch.int64))]).to(cnt.device)
    dist.all_reduce(cnt, group=group)
    dist.all_reduce(fills, op=dist.ReduceOp.MAX, group=group)
    c, f = cnt.tolist(), fills.tolist()
    if hasattr(stages, "combine_buckets"):
        # the exact combine's fills are one record per key; a bucket combine
        # that pre-aggregates per tile sends up to one per key per tile: learn
        # at least the first call's even split of the files then
        tiles = getattr(stages, "combine_tiles", False)
        _learn(stages, win, max(f[0], win["max_n"] // world) if tiles else f[0],
               max(f[1], win["max_ne"] // world) if tiles else f[1], f[2])
    return link, int(c[0]), int(c[1])


class _Trace:
    """SDCAS_DEDUP_TRACE=1: wall time of each bucket-protocol stage on rank 0's
    stderr, the device drained at every mark (a diagnostic: it adds host
    synchronisations the protocol itself does not have)"""
    on = bool(os.environ.get("SDCAS_DEDUP_TRACE"))

    def __init__(self):
        self.t, self.parts = time.perf_counter(), []

    def mark(self, what):
        if self.on:
            torch.cuda.synchronize()
            now = time.perf_counter()
            self.parts.append(f"{what} {1e3 * (now - self.t):.2f}")
            self.t = now

    def done(self, group):
        if self.on and dist.get_rank(group) == 0:
            print("dedup buckets ms: " + ", ".join(self.parts), file=sys.stderr, flush=True)


class _XTimer:
    """stages.time_exchange: HIP events around the bucket protocol's
    all-to-alls on the caller's stream (the collectives are ordered on it; no
    host synchronisation added) and the bytes this rank sends, left in
    stages.last_exchange for the caller to read after it synchronises"""

    def __init__(self, stages, dev):
        self.stages, self.dev = stages, dev
        self.on = bool(getattr(stages, "time_exchange", False))
        self.events = []

    def start(self):
        if self.on:
            self.events.append([torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)])
            self.events[-1][0].record(torch.cuda.current_stream(self.dev))

    def stop(self):
        if self.on:
            self.events[-1][1].record(torch.cuda.current_stream(self.dev))

    def done(self, world, *tensors):
        if self.on:
            b = sum(int(t.numel()) * t.element_size() for t in tensors if t is not None)
            self.stages.last_exchange = {"bytes": b, "bytes_off_rank": b * (world - 1) // world,
                                         "events": [tuple(e) for e in self.events]}


def _dedup_buckets(stages, world, keys, has_key, status, ids, chunk_size, existing_keys, existing_ids, group, win):
    """the exchange in fixed-capacity buckets: one host synchronisation of the
    device (the totals; the counts agreed before it are host integers); None
    when a bucket overflowed (the caller reruns the exact path)"""
    tr = _Trace()
    tr.mark("enter")
    has_ex = existing_keys is not None
    fcap, ecap, scap = _caps(stages, world, win, has_ex)
    stages.bucket_caps = (fcap, ecap)
    plan, scnt = _plan(stages, has_key, status, ids, chunk_size, win, group, world, scap)
    send, slot, fcnt, ovf = stages.combine_buckets(keys, has_key, status, ids, world, fcap)
    dev = fcnt.device
    if has_ex:
        if existing_keys.numel():
            esend, _, ecnt, eovf = stages.combine_buckets(existing_keys, None, None, existing_ids, world, ecap,
                                                          need_slot=False)
        else:
            esend = torch.zeros((world * ecap, 2), dtype=torch.int64, device=dev)
            ecnt = torch.zeros(world, dtype=torch.int64, device=dev)
            eovf = torch.zeros(1, dtype=torch.int32, device=dev)
        sc = torch.stack([fcnt, ecnt], 1).contiguous()
    else:
        sc = fcnt.view(world, 1).contiguous()
    tr.mark("stays+plan+combine")
    xev = _XTimer(stages, dev)
    xev.start()
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=group)  # equal splits: no host sizes
    tr.mark("a2a counts")
    frecv = torch.empty_like(send)
    dist.all_to_all_single(frecv, send.contiguous(), group=group)
    tr.mark(f"a2a buckets ({send.numel() * 8 >> 20} MiB)")
    if has_ex:
        erecv = torch.empty_like(esend)
        dist.all_to_all_single(erecv, esend.contiguous(), group=group)
        ercnt = rc[:, 1].contiguous()
    else:
        erecv, ercnt = None, None
    xev.stop()
    answer = stages.resolve_buckets(frecv, fcap, rc[:, 0].contiguous(), erecv, ecap if has_ex else 0, ercnt, world)
    tr.mark("resolve")
    xev.start()
    back = torch.empty_like(answer)
    dist.all_to_all_single(back, answer.contiguous(), group=group)
    xev.stop()
    xev.done(world, sc, send, esend if has_ex else None, answer)
    tr.mark("a2a answers")
    link, cnt = stages.apply(ids, slot, back, chunk_size, plan)
    tr.mark("apply")
    zero = torch.zeros((), dtype=torch.int64, device=dev)
    sfill = scnt.to(dev)[0] if scnt is not None else zero
    over = ovf.to(torch.int64) + (eovf.to(torch.int64) if has_ex else 0) + (sfill > scap).to(torch.int64)
    tot = torch.cat([cnt.to(torch.int64), over.view(1)])
    fills = torch.stack([fcnt.max(), ecnt.max() if has_ex else torch.full((), -1, dtype=torch.int64, device=dev),
                         sfill])
    dist.all_reduce(tot, group=group)
    dist.all_reduce(fills, op=dist.ReduceOp.MAX, group=group)
    tf = torch.cat([tot, fills]).tolist()  # the one host synchronisation
    tr.mark("totals")
    tr.done(group)
    t, f = tf[:3], tf[3:]
    # an overflowing call learns its true fills from the exact rerun (the
    # bucket counts here are clamped to the capacity)
    _learn(stages, win, f[0], f[1], f[2])
    if t[2]:
        return None
    return link, int(t[0]), int(t[1])


def owner_of(keys: np.ndarray, world: int) -> np.ndarray:
    """owner rank of cas keys (dist_dedup.h dd_owner): top 12 bits in `world` ranges"""
    k = np.asarray(keys, dtype=np.uint64)
    return ((k >> np.uint64(52)) * np.uint64(world) >> np.uint64(12)).astype(np.int64)


__all__ = ["DeviceStages", "identifier_dedup_distributed", "owner_of", "prepare_meta_group"]
_ = N  # the C ABI is bound by spacedrive_amd._native.load()
