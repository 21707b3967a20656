"""GPU parity of the device-resident big-message stream (sdcas_dev_stream_*,
the C4 path of file_checksum, core/src/object/validation/hash.rs:11-25):
messages delivered as 1 MiB-aligned segments in arbitrary order from HBM,
against the golden 4 GiB + 1 checksum (upstream BLAKE3 C) and the CPU oracle."""
import numpy as np
import pytest
import torch

from tests._oracle import content_key, golden

pytestmark = pytest.mark.gpu
MiB = 1 << 20


@pytest.fixture(scope="module")
def eng():
    from spacedrive_amd import Engine
    e = Engine()
    yield e
    e.close()


def _segments(rng, size, max_pieces=5):
    """random 1 MiB-aligned cut of [0, size) into segments"""
    segs, off = [], 0
    while off < size:
        take = int(rng.integers(1, max_pieces + 1)) * MiB
        take = min(take, size - off)
        segs.append((off, take))
        off += take
    return segs


def test_stream_synth_vs_oracle(eng, oracle):
    rng = np.random.default_rng(4)
    sizes = [MiB + 1, 3 * MiB + 17, 8 * MiB, 17 * MiB + 1025, 33 * MiB - 1]
    keys = [content_key(0x5D0004, 100 + i) for i in range(len(sizes))]
    segs = [(f, o, l) for f, s in enumerate(sizes) for o, l in _segments(rng, s)]
    rng.shuffle(segs)
    cap = sum((l + MiB - 1) // MiB * MiB for _, _, l in segs) + 4096
    blob = torch.empty(cap, dtype=torch.uint8, device="cuda")
    base = blob.data_ptr()
    boffs, used = [], 0
    for _, _, l in segs:
        boffs.append(used)
        used += (l + MiB - 1) // MiB * MiB
    t = lambda a: torch.from_numpy(np.array(a, np.uint64).view(np.int64)).cuda()
    s = torch.cuda.Stream()
    out = torch.zeros((len(sizes), 32), dtype=torch.uint8, device="cuda")
    args = [t([keys[f] for f, _, _ in segs]), t([o for _, o, _ in segs]), t([l for _, _, l in segs]), t(boffs)]
    torch.cuda.synchronize()  # inputs written before the side stream reads them
    eng.dev_synth_content(*(a.data_ptr() for a in args), len(segs), base, s.cuda_stream)
    eng.dev_stream_begin(sizes)
    # deliver in two calls, in shuffled order
    h = len(segs) // 2
    for part in (slice(0, h), slice(h, None)):
        sg = segs[part]
        eng.dev_stream_update([f for f, _, _ in sg], [o for _, o, _ in sg], [l for _, _, l in sg],
                              [base + b for b in boffs[part]], stream=s.cuda_stream)
    eng.dev_stream_finish(out.data_ptr(), s.cuda_stream)
    eng.dev_sync(s.cuda_stream)
    got = out.cpu().numpy()
    for i, (k, n) in enumerate(zip(keys, sizes)):
        assert bytes(got[i]).hex() == oracle.synth_checksum(k, n), n


def test_stream_sessions_back_to_back(oracle):
    """sessions enqueued without a host wait between them (stream_begin no
    longer synchronises; its descriptors and the node-list clear go up on the
    session's first stream call, the piece list is expanded on the device):
    three sessions of different shapes — the second smaller, the third larger
    than the first (its buffers grow) — alternating between two streams, then
    one sync; every digest exact"""
    from spacedrive_amd import Engine
    rng = np.random.default_rng(12)
    shapes = [[MiB + 1, 5 * MiB + 3, 9 * MiB], [2 * MiB], [3 * MiB + 17, MiB + 1025, 12 * MiB, 4 * MiB + 1, 7 * MiB]]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    with Engine() as e:
        runs = []
        for si, sizes in enumerate(shapes):
            keys = [content_key(0x5D0004, 300 + 10 * si + i) for i in range(len(sizes))]
            segs = [(f, o, l) for f, n in enumerate(sizes) for o, l in _segments(rng, n, 3)]
            rng.shuffle(segs)
            boffs, used = [], 0
            for _, _, l in segs:
                boffs.append(used)
                used += (l + MiB - 1) // MiB * MiB
            blob = torch.empty(used + 4096, dtype=torch.uint8, device="cuda")
            t = lambda a: torch.from_numpy(np.array(a, np.uint64).view(np.int64)).cuda()
            args = [t([keys[f] for f, _, _ in segs]), t([o for _, o, _ in segs]), t([l for _, _, l in segs]), t(boffs)]
            out = torch.zeros((len(sizes), 32), dtype=torch.uint8, device="cuda")
            runs.append((keys, sizes, segs, boffs, blob, args, out))
        torch.cuda.synchronize()
        for si, (keys, sizes, segs, boffs, blob, args, out) in enumerate(runs):
            st = streams[si % 2].cuda_stream
            base = blob.data_ptr()
            e.dev_synth_content(*(a.data_ptr() for a in args), len(segs), base, st)
            e.dev_stream_begin(sizes)
            for part in (slice(0, 1), slice(1, None)):
                sg = segs[part]
                e.dev_stream_update([f for f, _, _ in sg], [o for _, o, _ in sg], [l for _, _, l in sg],
                                    [base + b for b in boffs[part]], stream=st)
            e.dev_stream_finish(out.data_ptr(), st)
        for s in streams:
            e.dev_sync(s.cuda_stream)
        for keys, sizes, _, _, _, _, out in runs:
            got = out.cpu().numpy()
            for i, (k, n) in enumerate(zip(keys, sizes)):
                assert bytes(got[i]).hex() == oracle.synth_checksum(k, n), n
        # a session with no update at all still clears its node list: a
        # message none of whose pieces arrived finishes as the same garbage
        # every time (zeros in), never as the previous session's nodes
        out0 = torch.zeros((1, 32), dtype=torch.uint8, device="cuda")
        out1 = torch.zeros((1, 32), dtype=torch.uint8, device="cuda")
        e.dev_stream_begin([3 * MiB])
        e.dev_stream_finish(out0.data_ptr(), streams[0].cuda_stream)
        keys, sizes, segs, boffs, blob, args, out = runs[1]
        e.dev_stream_begin(sizes)
        e.dev_stream_update([f for f, _, _ in segs], [o for _, o, _ in segs], [l for _, _, l in segs],
                            [blob.data_ptr() + b for b in boffs], stream=streams[0].cuda_stream)
        e.dev_stream_finish(out.data_ptr(), streams[0].cuda_stream)
        e.dev_stream_begin([3 * MiB])
        e.dev_stream_finish(out1.data_ptr(), streams[0].cuda_stream)
        e.dev_sync(streams[0].cuda_stream)
        assert torch.equal(out0, out1)
        assert bytes(out.cpu().numpy()[0]).hex() == oracle.synth_checksum(keys[0], sizes[0])


@pytest.mark.parametrize("variant", [17, 19])
def test_stream_piece_boundaries_vs_oracle(oracle, variant):
    """every product piece kernel over files whose lengths sit at and around
    1 MiB-piece, 1 KiB-chunk and 64-byte-block boundaries (a last piece of
    exactly 1024 chunks with a partial last chunk among them: piece 19 must
    store its deferred node too), delivered as random 1 MiB-aligned segments
    in shuffled order over three update calls, against the oracle"""
    from spacedrive_amd import Engine
    rng = np.random.default_rng(70 + variant)
    deltas = [-1025, -1024, -1023, -65, -64, -1, 0, 1, 63, 64, 1023, 1024, 1025]
    sizes = sorted({int(k) * MiB + d for k in (2, 3, 5, 8) for d in deltas} |
                   {MiB + d for d in deltas if d > 0})
    sizes = [int(x) for x in rng.permutation(sizes)]
    keys = [content_key(0x5D0004, 1000 + 64 * variant + i) for i in range(len(sizes))]
    segs = [(f, o, l) for f, n in enumerate(sizes) for o, l in _segments(rng, n, 3)]
    rng.shuffle(segs)
    boffs, used = [], 0
    for _, _, l in segs:
        boffs.append(used)
        used += (l + MiB - 1) // MiB * MiB
    blob = torch.empty(used + 4096, dtype=torch.uint8, device="cuda")
    base = blob.data_ptr()
    t = lambda a: torch.from_numpy(np.array(a, np.uint64).view(np.int64)).cuda()
    out = torch.zeros((len(sizes), 32), dtype=torch.uint8, device="cuda")
    with Engine() as e:
        assert e.dev_set_piece_variant(variant)
        s = torch.cuda.Stream()
        args = [t([keys[f] for f, _, _ in segs]), t([o for _, o, _ in segs]), t([l for _, _, l in segs]), t(boffs)]
        torch.cuda.synchronize()
        e.dev_synth_content(*(a.data_ptr() for a in args), len(segs), base, s.cuda_stream)
        e.dev_stream_begin(sizes)
        cuts = [0, len(segs) // 3, 2 * len(segs) // 3, len(segs)]
        for a, b in zip(cuts[:-1], cuts[1:]):
            sg = segs[a:b]
            e.dev_stream_update([f for f, _, _ in sg], [o for _, o, _ in sg], [l for _, _, l in sg],
                                [base + x for x in boffs[a:b]], stream=s.cuda_stream)
        e.dev_stream_finish(out.data_ptr(), s.cuda_stream)
        e.dev_sync(s.cuda_stream)
    got = out.cpu().numpy()
    bad = [n for i, (k, n) in enumerate(zip(keys, sizes)) if bytes(got[i]).hex() != oracle.synth_checksum(k, n)]
    assert not bad, (variant, bad)


def test_stream_4gib_plus_1_golden(eng):
    c = [c for c in golden("checksums.json") if c["size"] == (4 << 30) + 1][0]
    n = c["size"]
    period = (np.arange(251 * 4096, dtype=np.uint64) % np.uint64(251)).astype(np.uint8)
    host = np.resize(period, n)
    dev = torch.empty(n + 4096, dtype=torch.uint8, device="cuda")
    dev[:n].copy_(torch.from_numpy(host))
    del host
    rng = np.random.default_rng(1)
    segs = _segments(rng, n, max_pieces=700)
    rng.shuffle(segs)
    out = torch.zeros((1, 32), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    torch.cuda.synchronize()
    eng.dev_stream_begin([n])
    eng.dev_stream_update([0] * len(segs), [o for o, _ in segs], [l for _, l in segs],
                          [dev.data_ptr() + o for o, _ in segs])
    eng.dev_stream_finish(out.data_ptr())
    eng.dev_sync()
    assert bytes(out.cpu().numpy()[0]).hex() == c["checksum"]


def test_stream_rejects_bad_segments(eng):
    from spacedrive_amd import _native as N
    with pytest.raises(N.SdcasError):
        eng.dev_stream_begin([MiB])  # small messages go through dev_hash_messages
    eng.dev_stream_begin([4 * MiB])
    buf = torch.empty(8 * MiB, dtype=torch.uint8, device="cuda")
    with pytest.raises(N.SdcasError):
        eng.dev_stream_update([0], [MiB // 2], [MiB], [buf.data_ptr()])  # not on a piece boundary
    with pytest.raises(N.SdcasError):
        eng.dev_stream_update([1], [0], [MiB], [buf.data_ptr()])  # no such message


def test_stream_over_4tib_golden(eng):
    """file_checksum of a 4 TiB + 1 MiB + 17 byte file: chunk counters reach
    2^32 + 1024, so the high counter word (v13) and a 2^22-piece root merge
    are exercised. The content repeats with a 1 MiB period, so every segment
    is the same resident 1 MiB buffer; the expected value is the committed
    fixture from upstream BLAKE3 C 1.8.2 (oracle/gen_golden_periodic.py)."""
    import json
    import os
    from tests._oracle import GOLDEN
    with open(os.path.join(GOLDEN, "checksums_periodic.json")) as f:
        doc = json.load(f)
    assert doc["period"] == MiB
    period = (np.arange(MiB, dtype=np.uint64) % np.uint64(251)).astype(np.uint8)
    dev = torch.zeros(MiB + 4096, dtype=torch.uint8, device="cuda")
    dev[:MiB].copy_(torch.from_numpy(period))
    torch.cuda.synchronize()
    for c in doc["cases"]:
        n = c["size"]
        q, r = divmod(n, MiB)
        offs = np.arange(q + (r > 0), dtype=np.uint64) * np.uint64(MiB)
        lens = np.full(offs.size, MiB, np.uint64)
        if r:
            lens[-1] = r
        out = torch.zeros((1, 32), dtype=torch.uint8, device="cuda")
        eng.dev_stream_begin([n])
        # two updates: the high-counter pieces arrive first
        h = offs.size - 3
        for part in (slice(h, None), slice(0, h)):
            k = offs[part].size
            eng.dev_stream_update(np.zeros(k, np.uint64), offs[part], lens[part],
                                  np.full(k, dev.data_ptr(), np.uint64))
        eng.dev_stream_finish(out.data_ptr())
        eng.dev_sync()
        assert bytes(out.cpu().numpy()[0]).hex() == c["checksum"], n


@pytest.mark.parametrize("variant", [17, 19])
def test_piece_variants_vs_oracle(oracle, variant):
    """every product piece kernel (17: one workgroup per piece, whole chunks
    through the full-chunk loop; 19: 17 with the full pieces' tree levels
    5-10 in k_piece_top, eight pieces per workgroup) over
    multi-window files whose windows hold many pieces and a ragged tail,
    against the oracle"""
    from spacedrive_amd import Engine
    rng = np.random.default_rng(40 + variant)
    sizes = [MiB + 1, 5 * MiB + 17, 16 * MiB, 9 * MiB + 4095, 2 * MiB - 1, 40 * MiB + 3, 3 * MiB - 1000]
    # contents differ per variant: a node a kernel failed to write must not
    # be found intact in memory an earlier case freed
    keys = [content_key(0x5D0004, 300 + 16 * variant + i) for i in range(len(sizes))]
    with Engine(staging_bytes=8 * MiB) as e:
        assert e.dev_set_piece_variant(variant)
        from tests._oracle import content
        blob, offs = [], []
        pos = 0
        for k, n in zip(keys, sizes):
            offs.append(pos)
            blob.append(content("synth", 0, n, k))
            pos += n
        host = np.concatenate(blob)
        out = e.hash_messages(host, np.array(offs, np.uint64), np.array(sizes, np.uint64))
    for i, (k, n) in enumerate(zip(keys, sizes)):
        assert bytes(out[i]).hex() == oracle.synth_checksum(k, n), (variant, n)


def test_checksums_progress_and_cancel(oracle, tmp_path):
    """a 1 GiB validator batch (eight 128 MiB files, 1 MiB-piece windows of
    16 MiB) reports progress window by window and is cancelled midway
    (job/mod.rs:862-960): files whose every piece was submitted keep exact
    digests and status 0, the rest get SDCAS_STATUS_CANCELLED, the call
    raises Cancelled; a second batch with the flag cleared completes"""
    import ctypes
    from spacedrive_amd import Engine
    from spacedrive_amd import _native as N
    from tests._oracle import content
    sizes = [128 * MiB] * 7 + [128 * MiB + 777]
    keys = [content_key(0x5D0004, 900 + i) for i in range(len(sizes))]
    paths = []
    for i, (k, n) in enumerate(zip(keys, sizes)):
        p = tmp_path / f"big{i}"
        p.write_bytes(content("synth", 0, n, k).tobytes())
        paths.append(str(p))
    flag = ctypes.c_int32(0)
    seen = []

    def progress(done, total):
        seen.append((done, total))
        if done >= 0.4 * total:
            flag.value = 1

    with Engine(staging_bytes=16 * MiB, io_threads=4, progress=progress, cancel=flag) as e:
        with pytest.raises(N.Cancelled) as ex:
            e.file_checksums(paths)
        out, st = ex.value.partial
        assert set(int(x) for x in st) <= {0, N.SDCAS_STATUS_CANCELLED}
        done_files = [i for i in range(len(paths)) if st[i] == 0]
        assert 0 < len(done_files) < len(paths), st
        for i in done_files:
            assert bytes(out[i]).hex() == oracle.synth_checksum(keys[i], sizes[i]), i
        assert len(seen) >= 8 and all(t == sum(sizes) for _, t in seen)
        assert all(a[0] <= b[0] for a, b in zip(seen, seen[1:]))
        # cleared flag: the same context completes the whole batch
        flag.value = 0
        seen.clear()
        e.set_progress(lambda d, t: seen.append((d, t)), flag)
        out, st = e.file_checksums(paths[:3])
        assert not st.any()
        for i in range(3):
            assert bytes(out[i]).hex() == oracle.synth_checksum(keys[i], sizes[i])
        assert seen[-1][0] == seen[-1][1] == sum(sizes[:3])


def test_cas_ids_cancel_per_slot(oracle, tmp_path):
    """sdcas_cas_ids over 3000 small files in 1 MiB staging slots, cancelled
    after about a third: completed files keep exact keys, the others are
    SDCAS_STATUS_CANCELLED; a flag set before the call cancels every file"""
    import ctypes
    from spacedrive_amd import Engine
    from spacedrive_amd import _native as N
    rng = np.random.default_rng(8)
    paths, sizes = [], []
    for i in range(3000):
        n = int(rng.integers(1, 60000))
        p = tmp_path / f"s{i}"
        p.write_bytes(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        paths.append(str(p))
        sizes.append(n)
    flag = ctypes.c_int32(0)

    def progress(done, total):
        if done >= total // 3:
            flag.value = 1

    with Engine(staging_bytes=1 * MiB, io_threads=4, progress=progress, cancel=flag) as e:
        with pytest.raises(N.Cancelled) as ex:
            e.generate_cas_ids(paths, sizes)
        keys, st = ex.value.partial
        ok = np.nonzero(st == 0)[0]
        assert 0 < ok.size < len(paths) and set(st.tolist()) <= {0, N.SDCAS_STATUS_CANCELLED}
        for i in ok[:: max(1, ok.size // 200)]:
            assert f"{int(keys[i]):016x}" == oracle.generate_cas_id(paths[i], sizes[i])
        with pytest.raises(N.Cancelled) as ex:
            e.generate_cas_ids(paths[:50], sizes[:50])  # still set: nothing is read
        assert (ex.value.partial[1] == N.SDCAS_STATUS_CANCELLED).all()


def test_message_calls_cancel(oracle):
    """sdcas_hash_messages over many staging slots, cancelled after about a
    third: the call returns SDCAS_E_CANCELLED (its outputs carry no per-item
    status, so Cancelled holds no partial results); with the flag cleared the
    same context hashes the batch exactly"""
    import ctypes
    from spacedrive_amd import Engine
    from spacedrive_amd import _native as N
    rng = np.random.default_rng(12)
    msgs = [rng.integers(0, 256, int(rng.integers(1, 100_000)), dtype=np.uint8).tobytes() for _ in range(600)]
    blob, offs, lens = Engine.pack(msgs)
    flag = ctypes.c_int32(0)

    def progress(done, total):
        if done >= total // 3:
            flag.value = 1

    with Engine(staging_bytes=1 * MiB, io_threads=4, progress=progress, cancel=flag) as e:
        with pytest.raises(N.Cancelled) as ex:
            e.hash_messages(blob, offs, lens)
        assert ex.value.partial is None
        with pytest.raises(N.Cancelled):
            e.cas_ids_from_messages(blob, offs, lens)
        flag.value = 0
        e.set_progress(None, flag)
        out = e.hash_messages(blob, offs, lens)
        for i in range(0, len(msgs), 37):
            assert bytes(out[i]).hex() == oracle.hash(msgs[i]), i


@pytest.mark.parametrize("direct", [False, True])
def test_checksums_parallel_pieces_and_direct_io(oracle, tmp_path, direct):
    """file_checksum of files over 1 MiB: a window's 1 MiB pieces are read by
    the I/O threads in parallel, with O_DIRECT when asked (page cache where
    the filesystem refuses it); digests exact, small files alongside"""
    from spacedrive_amd import Engine
    from tests._oracle import content
    sizes = [3 * MiB + 5, 40 * MiB + 1, 2 * MiB, 100 * MiB + 4097, 5000, MiB + 1]
    keys = [content_key(0x5D0004, 700 + i) for i in range(len(sizes))]
    paths = []
    for i, (k, n) in enumerate(zip(keys, sizes)):
        p = tmp_path / f"d{i}"
        p.write_bytes(content("synth", 0, n, k).tobytes())
        paths.append(str(p))
    with Engine(staging_bytes=16 * MiB, io_threads=6, direct_io=direct) as e:
        out, st = e.file_checksums(paths)
    assert not st.any(), st
    for i, (k, n) in enumerate(zip(keys, sizes)):
        assert bytes(out[i]).hex() == oracle.synth_checksum(k, n), n
