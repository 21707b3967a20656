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
