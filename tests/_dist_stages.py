"""Test infrastructure: numpy restatement of the three device stages of the
multi-GPU dedup (spacedrive_amd/csrc/dist_dedup.hip), on CPU torch tensors.

Used (a) to run spacedrive_amd.dist_dedup's collective protocol under gloo on
CPU, where there is no GPU, and (b) as a second checker of the device stages.
Never used by the product path. Semantics follow
core/src/object/file_identifier/mod.rs:149-254 in the canonical form of
SURVEY.md §8a a7 (see tests/_oracle.py:identifier_dedup for the chunked loop).
"""
import numpy as np
import torch

from spacedrive_amd.dist_dedup import owner_of

NOKEY = np.uint32(0xFFFFFFFF)
ALL_ONES = np.uint64(2**64 - 1)
H = 12  # SDCAS_PLAN_HEADER_WORDS
DROPPED = np.uint32(0xFFFFFFFE)


def _u64(t):
    return t.numpy().view(np.uint64) if t is not None else None


def _t64(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64))


def virtual_exchange(send_list, counts_list):
    """all-to-all among R virtual ranks in one process: send_list[r] rows
    grouped by destination with counts_list[r][d] rows for d. Returns per
    destination (recv rows, recv counts from each source)."""
    R = len(send_list)
    out, out_counts = [], []
    offs = [np.concatenate([[0], np.cumsum(c)]).astype(np.int64) for c in counts_list]
    for d in range(R):
        parts = [send_list[s][int(offs[s][d]):int(offs[s][d + 1])] for s in range(R)]
        out.append(torch.cat(parts) if parts else send_list[0][:0])
        out_counts.append([int(counts_list[s][d]) for s in range(R)])
    return out, out_counts


def dedup_virtual(stages_for, shards, chunk_size, existing_shards=None):
    """Run the protocol of identifier_dedup_distributed for R virtual ranks in
    one process (stages_for(r) gives rank r's stage object; shards[r] =
    (keys, has_key, status, ids) tensors). Returns (per-rank links, created,
    linked)."""
    R = len(shards)
    st = [stages_for(r) for r in range(R)]
    plan = virtual_plan(st, shards, chunk_size)
    recs, slots, counts = [], [], []
    for r, (k, h, s, ids) in enumerate(shards):
        rec, slot, starts = st[r].combine(k, h, s, ids, R)
        recs.append(rec)
        slots.append(slot)
        counts.append([starts[d + 1] - starts[d] for d in range(R)])
    erecs, ecounts = [], []
    for r in range(R):
        if existing_shards is not None and existing_shards[r][0].numel():
            ek, eids = existing_shards[r]
            rec, _, starts = st[r].combine(ek, None, None, eids, R)
        else:
            rec, starts = recs[r][:0], [0] * (R + 1)
        erecs.append(rec)
        ecounts.append([starts[d + 1] - starts[d] for d in range(R)])
    frecv, fc = virtual_exchange(recs, counts)
    erecv, _ = virtual_exchange(erecs, ecounts)
    answers = [st[d].resolve(frecv[d], erecv[d]) for d in range(R)]
    # reverse exchange: destination d sends answers back grouped by source
    back, _ = virtual_exchange(answers, fc)
    links, created, linked = [], 0, 0
    for r, (k, h, s, ids) in enumerate(shards):
        link, cnt = st[r].apply(ids, slots[r], back[r], chunk_size, plan)
        links.append(link)
        c = cnt.cpu().tolist()
        created += int(c[0])
        linked += int(c[1])
    return links, created, linked


def virtual_plan(st, shards, chunk_size, n_total=None):
    """stays of every virtual rank, gathered, then one plan (every rank would
    build the same)"""
    n_total = n_total if n_total is not None else sum(int(x[3].numel()) for x in shards)
    parts = []
    for r, (k, h, s, ids) in enumerate(shards):
        out, cnt = st[r].stays(h, s, ids, max(int(ids.numel()), 1))
        parts.append(out)
    return st[0].plan(torch.cat(parts), n_total, chunk_size)


class NumpyStages:
    """Same contract as spacedrive_amd.dist_dedup.DeviceStages, on CPU."""

    def combine(self, keys, has_key, status, ids, world):
        ids_np = _u64(ids)
        n = ids_np.size
        k = _u64(keys) if keys is not None else np.zeros(n, np.uint64)
        ok = np.ones(n, bool) if status is None else status.numpy() == 0
        has = np.ones(n, bool) if has_key is None else has_key.numpy() != 0
        valid = ok & has
        slot = np.where(ok, NOKEY, DROPPED).astype(np.uint32)
        vi = np.nonzero(valid)[0]
        # one record per distinct key (its lowest id: ids ascend), key order;
        # the device combine (a hash table since round 5) emits the same
        # records grouped by owner in no particular order within an owner
        order = vi[np.argsort(k[vi], kind="stable")]
        sk = k[order]
        head = np.ones(sk.size, bool)
        head[1:] = sk[1:] != sk[:-1]
        uid = np.cumsum(head) - 1
        slot[order] = uid.astype(np.uint32)
        rec = np.stack([sk[head], ids_np[order[head]]], 1) if sk.size else np.zeros((0, 2), np.uint64)
        own = owner_of(rec[:, 0], world)
        starts = [int(x) for x in np.searchsorted(own, np.arange(world + 1), side="left")]
        starts[world] = int(rec.shape[0])
        return _t64(rec).reshape(-1, 2), torch.from_numpy(slot.view(np.int32)), starts

    def resolve(self, frec, erec):
        f = _u64(frec).reshape(-1, 2)
        e = _u64(erec).reshape(-1, 2)
        emin = {}
        for key, db in e:
            if key not in emin or db < emin[key]:
                emin[int(key)] = int(db)
        fmin = {}
        for key, i in f:
            key, i = int(key), int(i)
            if key not in fmin or i < fmin[key]:
                fmin[key] = i
        res = np.empty(f.shape[0], np.int64)
        for p, (key, _) in enumerate(f):
            key = int(key)
            res[p] = -emin[key] - 1 if key in emin else fmin[key]
        return torch.from_numpy(res)

    def combine_buckets(self, keys, has_key, status, ids, world, cap, need_slot=True):
        """the combine into world fixed-capacity buckets (dist_dedup.h
        dd_combine_buckets): record p of owner r at row r * cap + p"""
        rec, slot, starts = self.combine(keys, has_key, status, ids, world)
        r64 = _u64(rec).reshape(-1, 2)
        send = np.zeros((world * cap, 2), np.uint64)
        counts = np.zeros(world, np.int64)
        over = 0
        for r in range(world):
            c = starts[r + 1] - starts[r]
            over |= int(c > cap)
            c = min(c, cap)
            counts[r] = c
            send[r * cap: r * cap + c] = r64[starts[r]: starts[r] + c]
        if slot is not None and need_slot:
            s = slot.numpy().view(np.uint32).copy()
            v = s < DROPPED
            own = owner_of(r64[s[v], 0], world)
            st = np.array(starts, np.int64)
            pos = s[v].astype(np.int64) - st[own]
            s[v] = np.where(pos < cap, own * cap + pos, np.int64(NOKEY)).astype(np.uint32)
            slot = torch.from_numpy(s.view(np.int32))
        else:
            slot = None
        return (_t64(send).reshape(-1, 2), slot, torch.from_numpy(counts),
                torch.tensor([over], dtype=torch.int32))

    def resolve_buckets(self, frecv, fcap, fcounts, erecv, ecap, ecounts, world):
        f = frecv.reshape(-1, 2)
        fsel = np.concatenate([np.arange(r * fcap, r * fcap + int(fcounts[r])) for r in range(world)]).astype(np.int64)
        if erecv is not None and ecap:
            e = erecv.reshape(-1, 2)
            esel = np.concatenate([np.arange(r * ecap, r * ecap + int(ecounts[r]))
                                   for r in range(world)]).astype(np.int64)
            ev = e[torch.from_numpy(esel)]
        else:
            ev = f[:0]
        ans = self.resolve(f[torch.from_numpy(fsel)], ev).numpy()
        out = np.full(world * fcap, -7, np.int64)  # padding: never read
        out[fsel] = ans
        return torch.from_numpy(out)

    def stays(self, has_key, status, ids, cap):
        """ordinals of the rows that stay orphans after their step (the
        device's dd_stays): int64[cap] padded with -1, count int64[1]"""
        ids_np = _u64(ids)
        n = ids_np.size
        ok = np.ones(n, bool) if status is None else status.numpy() == 0
        has = np.ones(n, bool) if has_key is None else has_key.numpy() != 0
        s = ids_np[~(ok & has)]
        out = np.full(cap, ALL_ONES, np.uint64)
        out[:min(cap, s.size)] = s[:cap]
        return _t64(out), torch.tensor([s.size], dtype=torch.int64)

    def plan(self, stays, n_total, chunk_size, max_steps=0, more=False):
        """the job's step plan (dist_dedup.h "the job's steps"), walking the
        stays ordinals one at a time"""
        cs = int(chunk_size)
        s = np.sort(_u64(stays))
        s = [int(x) for x in s[s < np.uint64(n_total)]]
        rr = []
        if cs > 1:
            for p in s:
                if p + 1 < n_total and (p + len(rr)) % cs == cs - 1:
                    rr.append(p)
        T = int(max_steps) or -(-n_total // cs)
        loop, reads, rows = -1, 0, 0
        if cs == 1 and s and s[0] < T:
            loop, reads, steps, limit, rows = s[0], T - s[0], T, s[0], s[0] + 1
        else:
            E = n_total + len(rr)
            avail = E // cs if more else -(-E // cs)
            steps = min(avail, T)
            limit = steps * cs
            if steps:
                P = min(limit, E) - 1
                rows = P - sum(1 for k, q in enumerate(rr) if q + k + 1 <= P) + 1
            if not more and T > avail and n_total and s and s[-1] == n_total - 1:
                loop, reads, steps = n_total - 1, 1 + T - avail, T
        run = sum(1 for k, q in enumerate(rr) if q + k + 1 < limit) + (reads - 1 if loop >= 0 else 0)
        head = [limit, len(rr), steps, rows, n_total, cs, loop, reads, run, 0, 0, 0]
        assert len(head) == H
        return torch.tensor(head + rr, dtype=torch.int64)

    def apply(self, ids, slot, result, chunk_size, plan=None):
        ids_np = _u64(ids).astype(np.int64)
        s = slot.numpy().view(np.uint32)
        r = result.numpy()
        cs = int(chunk_size)
        if plan is None:
            limit, rr, loop, reads = 2**63, [], 2**63, 0
        else:
            pl = plan.numpy()
            limit, nrr = int(pl[0]), int(pl[1])
            rr = [int(x) for x in pl[H:H + nrr]]
            loop = int(pl[6]) if int(pl[6]) >= 0 else 2**63
            reads = int(pl[7])
        below = lambda x: int(np.searchsorted(np.array(rr, np.int64), x, side="left")) if rr else 0
        link = np.empty(ids_np.size, np.int64)
        created = linked = 0
        MIN = np.iinfo(np.int64).min
        for i in range(ids_np.size):
            me = int(ids_np[i])
            kind = "drop" if s[i] == DROPPED else "nokey" if s[i] == NOKEY else "key"
            if me >= loop:
                if me > loop:
                    link[i] = MIN + 1
                elif kind == "drop":
                    link[i] = MIN
                else:
                    link[i] = me
                    created += reads
                continue
            b = below(me)
            pos = me + b
            twice = b < len(rr) and rr[b] == me
            if pos >= limit:
                link[i] = MIN + 1
            elif kind == "drop":
                link[i] = MIN
            elif kind == "nokey":
                link[i] = me
                created += 1 + (1 if twice and pos + 1 < limit else 0)
            else:
                v = int(r[s[i]])
                if v < 0:
                    link[i] = v
                    linked += 1
                elif pos // cs == (v + below(v)) // cs:
                    link[i] = me
                    created += 1
                else:
                    link[i] = v
                    linked += 1
        return torch.from_numpy(link), torch.tensor([created, linked], dtype=torch.int64)


def make_corpus(seed, n, pool=4000, zipf=1.3, p_none=0.02, p_err=0.01, n_existing=300):
    """keys with Zipf duplicates, None cas_ids, I/O errors, existing Objects"""
    rng = np.random.default_rng(seed)
    pool_keys = rng.integers(0, 2**64, pool, dtype=np.uint64)
    keys = pool_keys[rng.zipf(zipf, n) % pool]
    has = (rng.random(n) > p_none).astype(np.uint8)
    status = np.where(rng.random(n) < p_err, 5, 0).astype(np.int32)
    existing = np.concatenate([pool_keys[rng.integers(0, pool, n_existing)],
                               rng.integers(0, 2**64, n_existing // 6, dtype=np.uint64)])
    return keys, has, status, existing


def shard(keys, has, status, existing, R, device="cpu", contiguous=True):
    """split the orphan list into R contiguous ranges (rank r holds ordinals
    [lo_r, hi_r)), existing Objects round-robin by DB index"""
    n = keys.size
    cuts = [n * r // R for r in range(R + 1)]
    out = []
    for r in range(R):
        lo, hi = cuts[r], cuts[r + 1]
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(device)
        out.append((t(keys[lo:hi].view(np.int64), None), t(has[lo:hi], None), t(status[lo:hi], None),
                    t(np.arange(lo, hi, dtype=np.int64), None)))
    ex = []
    for r in range(R):
        idx = np.arange(r, existing.size, R, dtype=np.int64)
        ex.append((torch.from_numpy(existing[idx].view(np.int64)).to(device), torch.from_numpy(idx).to(device)))
    return out, ex


def dedup_virtual_buckets(stages_for, shards, chunk_size, existing_shards, caps):
    """The bucket protocol of identifier_dedup_distributed (fixed-capacity
    owner buckets, equal-split exchanges, no host synchronisation inside) for
    R virtual ranks in one process. caps = (file bucket capacity, existing
    bucket capacity). Returns (per-rank links, created, linked, overflowed)."""
    R = len(shards)
    fcap, ecap = caps
    st = [stages_for(r) for r in range(R)]
    sends, slots, fcnts, over = [], [], [], 0
    for r, (k, h, s, ids) in enumerate(shards):
        send, slot, cnt, ovf = st[r].combine_buckets(k, h, s, ids, R, fcap)
        sends.append(send)
        slots.append(slot)
        fcnts.append(cnt.cpu().numpy())
        over |= int(ovf.cpu()[0])
    esends, ecnts = [], []
    for r in range(R):
        if existing_shards is not None and existing_shards[r][0].numel():
            ek, eids = existing_shards[r]
            es, _, ec, eo = st[r].combine_buckets(ek, None, None, eids, R, ecap, need_slot=False)
            over |= int(eo.cpu()[0])
        else:
            es = sends[r].new_zeros((R * ecap, 2))
            ec = np.zeros(R, np.int64)
        esends.append(es)
        ecnts.append(ec if isinstance(ec, np.ndarray) else ec.cpu().numpy())

    def xchg(bufs, cap):  # equal splits: destination d gets bucket d of every source, in source order
        return [torch.cat([bufs[s][d * cap:(d + 1) * cap] for s in range(R)]) for d in range(R)]

    dev = sends[0].device
    frecv, erecv = xchg(sends, fcap), xchg(esends, ecap)
    answers = []
    for d in range(R):
        fc = torch.tensor([int(fcnts[s][d]) for s in range(R)], dtype=torch.int64, device=dev)
        ec = torch.tensor([int(ecnts[s][d]) for s in range(R)], dtype=torch.int64, device=dev)
        answers.append(st[d].resolve_buckets(frecv[d], fcap, fc, erecv[d] if ecap else None, ecap, ec, R))
    back = xchg(answers, fcap)
    plan = virtual_plan(st, shards, chunk_size)
    links, created, linked = [], 0, 0
    for r, (k, h, s, ids) in enumerate(shards):
        link, cnt = st[r].apply(ids, slots[r], back[r], chunk_size, plan)
        links.append(link)
        c = cnt.cpu().tolist()
        created += int(c[0])
        linked += int(c[1])
    return links, created, linked, over
