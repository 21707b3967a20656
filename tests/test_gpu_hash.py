"""GPU parity tests: the HIP path (through the C ABI) against the golden
fixtures (upstream BLAKE3 C, tests/golden) and the CPU oracle, bit-exact."""
import os

import numpy as np
import pytest

from tests._oracle import cas_windows, content, golden, spec_content, write_sparse_file

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from spacedrive_amd import Engine
    e = Engine(staging_bytes=64 << 20)
    yield e
    e.close()


def test_blake3_vectors(eng):
    cases = golden("blake3_vectors.json")
    msgs = [content("pattern251", 0, c["len"]).tobytes() for c in cases]
    out = eng.hash_messages(*eng.pack(msgs))
    for c, d in zip(cases, out):
        assert bytes(d).hex() == c["hash"], c["len"]


def test_blake3_vectors_one_by_one(eng):
    # every message alone in its batch: single-tile layouts
    for c in golden("blake3_vectors.json"):
        m = content("pattern251", 0, c["len"]).tobytes()
        assert bytes(eng.hash_messages(*eng.pack([m]))[0]).hex() == c["hash"], c["len"]


def test_cas_messages_golden(eng):
    cases = [c for c in golden("cas_ids.json")]
    msgs = []
    for c in cases:
        kind, key = spec_content(c["content"])
        parts = [c["size"].to_bytes(8, "little")] + [content(kind, o, n, key).tobytes()
                                                       for o, n in cas_windows(c["size"])]
        msgs.append(b"".join(parts))
    keys = eng.cas_ids_from_messages(*eng.pack(msgs))
    for c, k in zip(cases, keys):
        assert f"{int(k):016x}" == c["cas_id"], c


def test_generate_cas_id_files(eng, tmp_path):
    cases = golden("cas_ids.json")
    paths, sizes = [], []
    for c in cases:
        kind, key = spec_content(c["content"])
        p = tmp_path / f"f_{c['content'].replace(':', '_')}_{c['size']}"
        write_sparse_file(p, kind, key, c["size"], cas_windows(c["size"]))
        paths.append(str(p))
        sizes.append(c["size"])
    keys, st = eng.generate_cas_ids(paths, sizes)
    assert (st == 0).all()
    for c, k in zip(cases, keys):
        assert f"{int(k):016x}" == c["cas_id"], c
    # the single-file mirror of cas.rs:23
    assert eng.generate_cas_id(paths[3], sizes[3]) == cases[3]["cas_id"]


def test_generate_cas_id_files_direct_io(tmp_path):
    """SDCAS_OPT_DIRECT_IO on the cas_id path: every golden file (whole-file
    and sampled windows, sparse) read with O_DIRECT where the filesystem takes
    it — unaligned sample windows through the aligned bounce buffer — gives
    the same cas_ids; small checksums alongside, and a missing path keeps its
    errno"""
    import errno
    from spacedrive_amd import Engine
    cases = golden("cas_ids.json")
    paths, sizes = [], []
    for c in cases:
        kind, key = spec_content(c["content"])
        p = tmp_path / f"f_{c['content'].replace(':', '_')}_{c['size']}"
        write_sparse_file(p, kind, key, c["size"], cas_windows(c["size"]))
        paths.append(str(p))
        sizes.append(c["size"])
    with Engine(direct_io=True, staging_bytes=8 << 20) as e:
        keys, st = e.generate_cas_ids(paths + [str(tmp_path / "missing")], sizes + [10])
        assert st[-1] == errno.ENOENT
        assert (st[:-1] == 0).all()
        for c, k in zip(cases, keys):
            assert f"{int(k):016x}" == c["cas_id"], c
        small = [(p, n) for p, n in zip(paths, sizes) if n <= (1 << 20)]
        d_direct, s1 = e.file_checksums([p for p, _ in small])
    d_plain, s2 = eng_plain_checksums([p for p, _ in small])
    assert not s1.any() and not s2.any()
    assert (d_direct == d_plain).all()


def _fds_on(path):
    """this process's descriptors open on `path` (the directory itself)"""
    out = []
    for fd in os.listdir("/proc/self/fd"):
        try:
            if os.readlink(f"/proc/self/fd/{fd}") == str(path):
                out.append(fd)
        except OSError:
            pass
    return out


def test_no_directory_descriptor_outlives_a_path_call(tmp_path):
    """the readers open files relative to a cached directory descriptor
    (cas_io.cpp dir_of); once a path call returns, neither the pool threads nor
    the calling thread (big-file checksums open on it) may keep one — an idle
    engine must not hold a volume it just indexed busy"""
    from spacedrive_amd import Engine
    d = tmp_path / "vol"
    d.mkdir()
    small = []
    for i in range(200):
        p = d / f"s{i}"
        p.write_bytes(os.urandom(1000 + 517 * i))
        small.append(str(p))
    big = d / "big"
    big.write_bytes(os.urandom((3 << 20) + 5))
    with Engine(io_threads=8, staging_bytes=8 << 20) as e:
        keys, st = e.generate_cas_ids(small, [os.path.getsize(p) for p in small])
        assert not st.any()
        assert _fds_on(d) == []
        out, st = e.file_checksums(small[:50] + [str(big)])
        assert not st.any()
        assert _fds_on(d) == []
    assert _fds_on(d) == []


def test_file_metadata_matches_stat_then_cas_ids(eng, oracle, tmp_path):
    """sdcas_file_metadata (fs::metadata folded into the cas_id reads,
    mod.rs:48-96) against the two-step form — os.stat, then sdcas_cas_ids for
    the non-empty files — and the oracle: whole-file and sampled sizes, an
    empty file (no cas_id, no error), a missing path (ENOENT), a directory
    (flagged, no cas_id), every key exact"""
    import errno
    rng = np.random.default_rng(23)
    paths = []
    for i, size in enumerate([0, 1, 1000, 65536, 102400, 102401, 300_000, 5 << 20]
                             + [int(x) for x in rng.integers(1, 200_000, 300)]):
        p = tmp_path / f"m{i}"
        write_sparse_file(str(p), "synth", 1000 + i, size, cas_windows(size))
        paths.append(str(p))
    d = tmp_path / "adir"
    d.mkdir()
    paths += [str(tmp_path / "missing"), str(d)]
    sizes, keys, st, fl = eng.file_metadata(paths)
    # the same with the indexer's sizes as hints (the directory's and the
    # missing path's hints are 0)
    hinted = eng.file_metadata(paths, [os.path.getsize(p) if os.path.isfile(p) else 0 for p in paths])
    for a, b in zip((sizes, keys, st, fl), hinted):
        assert np.array_equal(a, b)
    assert st[-2] == errno.ENOENT and fl[-2] == 0
    assert st[-1] == 0 and fl[-1] == 2  # SDCAS_META_DIR
    real = paths[:-2]
    want_sz = [os.path.getsize(p) for p in real]
    assert sizes[:-2].tolist() == want_sz and not st[:-2].any()
    nonempty = [i for i, z in enumerate(want_sz) if z]
    assert all(fl[i] == 1 for i in nonempty) and all(fl[i] == 0 for i, z in enumerate(want_sz) if not z)
    k2, s2 = eng.generate_cas_ids([real[i] for i in nonempty], [want_sz[i] for i in nonempty])
    assert not s2.any() and np.array_equal(keys[nonempty], k2)
    for i in nonempty[::17]:
        assert f"{int(keys[i]):016x}" == oracle.generate_cas_id(real[i], want_sz[i]), i


def test_file_metadata_with_stale_size_hints(eng, oracle, tmp_path):
    """sdcas_file_metadata planned from the indexer's sizes when those are
    stale: files that grew or shrank since (across the 100 KiB branch of
    cas.rs too) are read again with room for their size now; every size,
    flag and key equals the hint-free call's and the oracle's"""
    rng = np.random.default_rng(31)
    paths, hints = [], []
    for i in range(400):
        size = int(rng.choice([0, 1, 5000, 99_000, 102_400, 102_401, 150_000, 3 << 20]))
        hint = int(rng.choice([size, 0, size + 1, max(0, size - 1), 50_000, 102_400, 102_401, 1 << 22]))
        p = tmp_path / f"h{i}"
        write_sparse_file(str(p), "synth", 5000 + i, size, cas_windows(size))
        paths.append(str(p))
        hints.append(hint)
    s0, k0, st0, f0 = eng.file_metadata(paths)
    s1, k1, st1, f1 = eng.file_metadata(paths, hints)
    assert not st0.any() and not st1.any()
    assert np.array_equal(s0, s1) and np.array_equal(f0, f1) and np.array_equal(k0, k1)
    for i in range(0, 400, 13):
        size = os.path.getsize(paths[i])
        assert s1[i] == size and f1[i] == (1 if size else 0)
        if size:
            assert f"{int(k1[i]):016x}" == oracle.generate_cas_id(paths[i], size), i


def eng_plain_checksums(paths):
    from spacedrive_amd import Engine
    with Engine() as e:
        return e.file_checksums(paths)


def test_file_checksums_golden(eng, tmp_path):
    cases = [c for c in golden("checksums.json") if c["size"] < (64 << 20)]
    paths = []
    for c in cases:
        kind, key = spec_content(c["content"])
        p = tmp_path / f"c_{c['content'].replace(':', '_')}_{c['size']}"
        p.write_bytes(content(kind, 0, c["size"], key).tobytes())
        paths.append(str(p))
    out, st = eng.file_checksums(paths)
    assert (st == 0).all()
    for c, d in zip(cases, out):
        assert bytes(d).hex() == c["checksum"], c
    assert eng.file_checksum(paths[0]) == cases[0]["checksum"]


def test_checksum_4gib_plus_1(eng):
    """unaligned multi-Mi-chunk tree (4096 full pieces + 1 tail byte) through
    the streamed big-message path, against upstream BLAKE3 C"""
    c = [c for c in golden("checksums.json") if c["size"] == (4 << 30) + 1][0]
    n = c["size"]
    period = np.arange(251 * 4096, dtype=np.uint64) % np.uint64(251)
    blob = np.resize(period.astype(np.uint8), n)
    out = eng.hash_messages(blob, np.array([0], np.uint64), np.array([n], np.uint64))
    assert bytes(out[0]).hex() == c["checksum"]


def test_errors_per_item(eng, tmp_path):
    import errno
    from spacedrive_amd import _native as N
    short = tmp_path / "short"
    short.write_bytes(b"x" * 20000)
    ok = tmp_path / "ok"
    ok.write_bytes(b"hello")
    keys, st = eng.generate_cas_ids([str(tmp_path / "missing"), str(short), str(ok)], [10, 200000, 5])
    assert st[0] == errno.ENOENT
    assert st[1] == N.SDCAS_STATUS_UNEXPECTED_EOF
    assert st[2] == 0
    with pytest.raises(OSError) as e:
        eng.generate_cas_id(str(short), 200000)
    assert "fill whole buffer" in str(e.value)
    d, st = eng.file_checksums([str(tmp_path), str(ok)])
    assert st[0] == errno.EISDIR and st[1] == 0


def test_file_grew_since_indexing(eng, oracle, tmp_path):
    """the indexer's size is stale: content comes from the file as it is now
    (cas.rs:29 fs::read), the prefix from `size`"""
    p = tmp_path / "grown"
    p.write_bytes(content("pattern251", 0, 70000).tobytes())
    assert eng.generate_cas_id(str(p), 5000) == oracle.generate_cas_id(str(p), 5000)
    p2 = tmp_path / "grown_past_100k"
    p2.write_bytes(content("pattern251", 0, 300000).tobytes())
    assert eng.generate_cas_id(str(p2), 100000) == oracle.generate_cas_id(str(p2), 100000)


def test_random_messages_vs_oracle(eng, oracle):
    rng = np.random.default_rng(1234)
    lens = np.concatenate([
        rng.integers(0, 4096, 300), rng.integers(0, 200_000, 200), rng.integers(900_000, 1_200_000, 6),
        np.array([0, 1, 1023, 1024, 1025, 1048576, 1048577, 2 * 1048576 + 5, 3 * 1048576])])
    rng.shuffle(lens)
    msgs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in lens]
    out = eng.hash_messages(*eng.pack(msgs))
    for m, d in zip(msgs, out):
        assert bytes(d).hex() == oracle.hash(m), len(m)


def test_tile_straddles_vs_oracle(eng, oracle):
    """message lengths chosen so that messages start at every offset inside a
    1024-slot tile and straddle tile boundaries at every tree level"""
    rng = np.random.default_rng(7)
    lens = []
    for c in [1, 2, 3, 5, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 101, 127, 128, 129, 255, 256,
              257, 511, 512, 513, 700, 1000, 1023, 1024]:
        lens += [c * 1024, c * 1024 - 1, c * 1024 + 1]
    lens = np.array(lens * 3)
    rng.shuffle(lens)
    msgs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in lens]
    out = eng.hash_messages(*eng.pack(msgs))
    for m, d in zip(msgs, out):
        assert bytes(d).hex() == oracle.hash(m), len(m)


@pytest.mark.parametrize("variant,finish", [(52, "quad"), (67, "quad"), (71, "quad"), (73, "quad"), (84, "quad"),
                                            (67, "lane"), (73, "lane"), (84, "lane")])
def test_tile_straddles_per_variant(oracle, variant, finish, monkeypatch):
    """the straddle corpus through each product leaf variant, in caller
    order (shape sort off) so messages straddle tiles at every level (71, 73
    and 84, the small-batch kernels — a lane / a quad of lanes per slot / a
    quad with four blocks in flight staged in LDS — selected
    explicitly: their 128-slot tiles for the whole batch, so messages of up to
    2049 chunks cross dozens of them), the crossing messages finished by
    k_finish_q (default) or k_finish_t (SDCAS_FINISH=lane)"""
    from spacedrive_amd import Engine
    if finish == "lane":
        monkeypatch.setenv("SDCAS_FINISH", "lane")
    rng = np.random.default_rng(70 + variant)
    lens = []
    for c in [1, 2, 3, 7, 8, 9, 16, 17, 31, 32, 33, 64, 65, 127, 128, 129, 255, 256, 257, 511, 512, 513, 1000,
              1023, 1024, 1025, 2049]:
        lens += [c * 1024, c * 1024 - 1, c * 1024 + 1]
    lens = np.array(lens * 2)
    rng.shuffle(lens)
    msgs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in lens]
    e = Engine(staging_bytes=64 << 20)
    try:
        assert e.dev_set_leaf_variant(variant)
        e.dev_set_sort(0)
        out = e.hash_messages(*e.pack(msgs))
    finally:
        e.close()
    bad = [i for i, (m, d) in enumerate(zip(msgs, out)) if bytes(d).hex() != oracle.hash(m)]
    assert not bad, [len(msgs[i]) for i in bad[:10]]


@pytest.mark.parametrize("variant", [52, 67, 71, 73, 84])
def test_many_short_multichunk_messages(oracle, variant):
    """C5-shaped batches — mostly 2..5-chunk messages, so tiles hold far more
    partial last chunks than a wave has lanes and the leaf kernel's block-count
    order is taken — next to runs of single-chunk messages and a few long
    ones; every digest against the oracle, for every product kernel (52:
    one tile per workgroup, the last-block-index loop, the first chunk kept
    from phase 1; 67, the default: 52 with the tail masks from a table; 71,
    73 and 84: the small-batch kernels, 128-slot tiles, a lane / a quad per
    slot / a quad with four blocks in flight staged in LDS)"""
    from spacedrive_amd import Engine
    rng = np.random.default_rng(55 + variant)
    lens = np.concatenate([rng.integers(1025, 5 * 1024 + 1, 12000), rng.integers(0, 1025, 3000),
                           rng.integers(5 * 1024, 200_000, 300), np.array([1024, 1025, 2048, 2049, 0])])
    rng.shuffle(lens)
    msgs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in lens]
    e = Engine(staging_bytes=64 << 20)
    try:
        assert e.dev_set_leaf_variant(variant)
        out = e.hash_messages(*e.pack(msgs))
    finally:
        e.close()
    bad = [i for i, (m, d) in enumerate(zip(msgs, out)) if bytes(d).hex() != oracle.hash(m)]
    assert not bad, [len(msgs[i]) for i in bad[:10]]


def test_diagnostic_variants_unreachable(eng, oracle):
    """the DIAGNOSTIC leaf variants (no memory reads / no compression / no
    tree: wrong digests) are not in the product library: selecting one is
    refused through the API, and the SDCAS_LEAF_VARIANT / SDCAS_PIECE_VARIANT
    environment overrides fall back to the default kernels — digests stay
    bit-exact"""
    import subprocess
    import sys
    for v in (4, 5, 6, 7, 26, 27, 28, 39, 40, 41, 1, 25, 29, 36, 43, 46, 47, 48, 49, 50, 51, 64, 65, 66, 68):
        assert not eng.dev_set_leaf_variant(v), v
    for v in (4, 6, 7, 11, 14, 15, 16, 18):
        assert not eng.dev_set_piece_variant(v), v
    code = (
        "import numpy as np, sys; sys.path.insert(0, %r)\n"
        "from spacedrive_amd import Engine\n"
        "from tests._oracle import load_oracle\n"
        "o = load_oracle(); rng = np.random.default_rng(3)\n"
        "msgs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in "
        "list(rng.integers(0, 300000, 200)) + [3 << 20, (1 << 20) + 1]]\n"
        "e = Engine(staging_bytes=16 << 20)\n"
        "out = e.hash_messages(*e.pack(msgs))\n"
        "bad = sum(bytes(d).hex() != o.hash(m) for m, d in zip(msgs, out))\n"
        "print('bad', bad); sys.exit(1 if bad else 0)\n") % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for env in ({"SDCAS_LEAF_VARIANT": "4"}, {"SDCAS_LEAF_VARIANT": "40", "SDCAS_PIECE_VARIANT": "7"}):
        r = subprocess.run([sys.executable, "-c", code], env={**os.environ, **env}, capture_output=True, text=True,
                           timeout=100)
        assert r.returncode == 0, (env, r.stdout[-500:], r.stderr[-2000:])


def test_device_api_synthetic_c2_sample(eng, oracle):
    """C2-shaped synthetic corpus generated in HBM, hashed by the device API;
    a random sample of files is re-derived by the CPU oracle"""
    import torch
    from tests._oracle import content_key
    n = 20000
    seed = 0x5D0002
    idx = np.arange(n, dtype=np.uint64)
    sizes = np.array([1024 + int(x) % (102400 - 1024 + 1) for x in _c2_raw(seed, idx)], np.uint64)
    keys = np.array([content_key(seed, i) for i in range(n)], np.uint64)
    lens = sizes + 8
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum((lens[:-1] + 15) // 16 * 16)
    total = int(offs[-1] + (lens[-1] + 15) // 16 * 16) + 64
    dev = torch.device("cuda:0")
    d_blob = torch.empty(total, dtype=torch.uint8, device=dev)
    t = lambda a: torch.from_numpy(a.view(np.int64)).to(dev)
    d_keys, d_sizes, d_offs, d_lens = t(keys), t(sizes), t(offs), t(lens)
    d_out = torch.zeros(n, dtype=torch.int64, device=dev)
    eng.dev_reserve(n, int(((lens + 1023) // 1024).sum()))
    eng.dev_synth_cas_messages(d_keys.data_ptr(), d_sizes.data_ptr(), d_offs.data_ptr(), n, d_blob.data_ptr())
    eng.dev_hash_messages(d_blob.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, 0, d_out.data_ptr())
    eng.dev_sync()
    got = d_out.cpu().numpy().view(np.uint64)
    rng = np.random.default_rng(3)
    for i in rng.choice(n, 300, replace=False):
        assert int(got[i]) == oracle.synth_cas_key(int(keys[i]), int(sizes[i])), i
    # the generated bytes themselves match the synthetic definition
    i = 17
    o = int(offs[i])
    assert bytes(d_blob[o:o + int(lens[i])].cpu().numpy()) == bytes(
        oracle.synth_cas_message(int(keys[i]), int(sizes[i])))


def test_small_and_big_batch_kernels(oracle):
    """the default leaf kernel is chosen by batch size: a device batch whose
    workspace holds at most 2^14 chunk slots runs the small-batch kernel
    (128-slot tiles, b3_batch.h kSmallSlots), a larger one the 1 MiB-tile
    kernel; the same C2-shaped corpus through both, every key against the
    oracle"""
    import torch
    from spacedrive_amd import Engine
    from tests._oracle import content_key
    n = 250
    seed = 0x5D0002
    idx = np.arange(n, dtype=np.uint64)
    sizes = np.array([1024 + int(x) % (102400 - 1024 + 1) for x in _c2_raw(seed, idx)], np.uint64)
    keys = np.array([content_key(seed, 7000 + i) for i in range(n)], np.uint64)
    lens = sizes + 8
    chunks = int(((lens + 1023) // 1024).sum())
    assert chunks + 3 * n + 2048 < (1 << 14)  # the small kernel's side of the threshold
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum((lens[:-1] + 15) // 16 * 16)
    total = int(offs[-1] + (lens[-1] + 15) // 16 * 16) + 64
    dev = torch.device("cuda:0")
    d_blob = torch.empty(total, dtype=torch.uint8, device=dev)
    t = lambda a: torch.from_numpy(a.view(np.int64)).to(dev)
    d_keys, d_sizes, d_offs, d_lens = t(keys), t(sizes), t(offs), t(lens)
    want = [oracle.synth_cas_key(int(keys[i]), int(sizes[i])) for i in range(n)]
    for reserve in (chunks, 4 * (1 << 14)):
        with Engine() as eng:
            d_out = torch.zeros(n, dtype=torch.int64, device=dev)
            eng.dev_reserve(n, reserve)
            eng.dev_synth_cas_messages(d_keys.data_ptr(), d_sizes.data_ptr(), d_offs.data_ptr(), n, d_blob.data_ptr())
            eng.dev_hash_messages(d_blob.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, 0, d_out.data_ptr())
            eng.dev_sync()
            got = d_out.cpu().numpy().view(np.uint64)
        bad = [i for i in range(n) if int(got[i]) != want[i]]
        assert not bad, (reserve, bad[:10])


def test_host_planned_small_batches(oracle, monkeypatch):
    """a staging-path batch of fewer than kSortMinMsgs messages for the small
    kernel is planned on the host (b3_batch.h BatchPlan: no scan, no
    k_tile_first, no k_finish_t when no message crosses a 128-slot tile):
    batches of 1-127 messages with empty, one-block, whole-chunk, 128-chunk
    and tile-crossing lengths give the oracle's digests, planned and with the
    plan turned off (SDCAS_PLAN_SMALL=0)"""
    from spacedrive_amd import Engine
    rng = np.random.default_rng(128)
    special = [0, 1, 63, 64, 65, 1023, 1024, 1025, 2048, 127 * 1024, 128 * 1024 - 1, 128 * 1024, 128 * 1024 + 1,
               129 * 1024 + 7, 300 * 1024 + 5]
    batches = [[L] for L in special]
    for n in (2, 3, 7, 40, 100, 127):
        batches.append([int(x) for x in rng.choice(special, n // 3)] +
                       [int(x) for x in rng.integers(0, 140 * 1024, n - n // 3)])
    for env in ("1", "0"):
        monkeypatch.setenv("SDCAS_PLAN_SMALL", env)
        with Engine(staging_bytes=16 << 20) as e:
            for lens in batches:
                msgs = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in lens]
                out = e.hash_messages(*e.pack(msgs))
                bad = [len(m) for m, d in zip(msgs, out) if bytes(d).hex() != oracle.hash(m)]
                assert not bad, (env, len(lens), bad[:10])


def _c2_raw(seed, idx):
    from tests._oracle import mix64
    with np.errstate(over="ignore"):
        x = np.uint64(seed) ^ np.uint64(0xC2C2C2C2) ^ (idx << np.uint64(20)) ^ (idx >> np.uint64(44))
        return mix64(x)


def test_dedup_vs_oracle(eng, oracle):
    rng = np.random.default_rng(99)
    n = 50000
    pool = rng.integers(0, 2**64, 8000, dtype=np.uint64)
    keys = pool[rng.zipf(1.3, n) % pool.size]
    has = (rng.random(n) > 0.02).astype(np.uint8)
    status = np.where(rng.random(n) < 0.01, 2, 0).astype(np.int32)
    existing = np.concatenate([pool[rng.integers(0, pool.size, 300)], rng.integers(0, 2**64, 50, dtype=np.uint64)])
    for cs in (100, 7, 1):
        want, wc, wl = oracle.identifier_dedup(keys, has, status, cs, existing)
        got, gc, gl = eng.identifier_dedup(keys, has, status, cs, existing)
        assert np.array_equal(want, got), cs
        assert (wc, wl) == (gc, gl)


def test_dedup_small_cases(eng):
    keys = np.array([10, 10, 11, 10, 12, 11, 99], np.uint64)
    has = np.array([1, 1, 1, 1, 1, 1, 0], np.uint8)
    out, created, linked = eng.identifier_dedup(keys, has, chunk_size=3)
    assert out.tolist() == [0, 1, 2, 0, 4, 2, 6] and created == 5 and linked == 2
    out, created, linked = eng.identifier_dedup(np.array([2**64 - 1, 2**64 - 1], np.uint64), [1, 1])
    assert out.tolist() == [0, 1] and created == 2
    out, created, linked = eng.identifier_dedup(np.zeros(0, np.uint64), np.zeros(0, np.uint8))
    assert out.size == 0 and created == 0


def test_pipelined_staging_many_batches(oracle, tmp_path):
    """tiny staging slots force dozens of double-buffered batches (host fills
    one pinned slot while the GPU hashes the other) on every host API"""
    from spacedrive_amd import Engine
    rng = np.random.default_rng(55)
    lens = np.concatenate([rng.integers(0, 300_000, 400), np.array([2 * 1048576 + 77, 1048577])])
    msgs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in lens]
    with Engine(staging_bytes=1 << 20, io_threads=4) as e:
        out = e.hash_messages(*e.pack(msgs))
        keys = e.cas_ids_from_messages(*e.pack(msgs))
        for m, d, k in zip(msgs, out, keys):
            want = oracle.hash(m)
            assert bytes(d).hex() == want, len(m)
            assert f"{int(k):016x}" == want[:16]
        paths, sizes = [], []
        for i, m in enumerate(msgs[:150]):
            p = tmp_path / f"f{i}"
            p.write_bytes(m)
            paths.append(str(p))
            sizes.append(len(m))
        ck, st = e.generate_cas_ids(paths, sizes)
        assert not st.any()
        for p, s, k in zip(paths, sizes, ck):
            assert f"{int(k):016x}" == oracle.generate_cas_id(p, s)
        d32, st = e.file_checksums(paths)
        assert not st.any()
        for m, d in zip(msgs[:150], d32):
            assert bytes(d).hex() == oracle.hash(m)


def test_pinned_caller_buffer_direct_dma(oracle):
    """messages in a pinned caller buffer (ascending, 16-byte aligned, with
    gaps) are DMA'd range by range into the device slots; the results equal
    the oracle's and the pageable path's, across many small slots; a pinned
    buffer with out-of-order offsets takes the staging copy"""
    import torch
    from spacedrive_amd import Engine
    rng = np.random.default_rng(77)
    lens = np.concatenate([rng.integers(0, 200_000, 300), np.array([1048577, 3 * 1048576 + 5, 0, 1])]).astype(np.uint64)
    gaps = rng.integers(0, 5, lens.size).astype(np.uint64) * np.uint64(16)
    offs = np.zeros(lens.size, np.uint64)
    pos = 0
    for i, L in enumerate(lens):
        pos += int(gaps[i])
        offs[i] = pos
        pos = (pos + int(L) + 15) // 16 * 16
    pinned = torch.empty(pos + 64, dtype=torch.uint8).pin_memory()
    host = pinned.numpy()
    host[:] = rng.integers(0, 256, host.size, dtype=np.uint8)
    want = [oracle.hash(host[int(o):int(o) + int(L)].tobytes()) for o, L in zip(offs, lens)]
    with Engine(staging_bytes=1 << 20, io_threads=4) as e:
        out = e.hash_messages(host, offs, lens)
        keys = e.cas_ids_from_messages(host, offs, lens)
        page = e.hash_messages(host.copy(), offs, lens)
        assert [bytes(d).hex() for d in out] == want
        assert [f"{int(k):016x}" for k in keys] == [w[:16] for w in want]
        assert np.array_equal(out, page)
        perm = rng.permutation(lens.size)
        out2 = e.hash_messages(host, offs[perm], lens[perm])
        assert [bytes(d).hex() for d in out2] == [want[i] for i in perm]


def test_concurrent_contexts_and_shared_context(oracle):
    """sd-core calls from several tokio workers: one context per thread runs
    concurrently; one context shared by threads serialises internally. Every
    result stays bit-exact."""
    import threading
    from spacedrive_amd import Engine
    rng = np.random.default_rng(99)
    batches = [[rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in rng.integers(0, 150_000, 60)]
               for _ in range(6)]
    want = [[oracle.hash(m) for m in b] for b in batches]
    got = [None] * len(batches)
    errs = []

    def work(i, e):
        try:
            got[i] = [bytes(d).hex() for d in e.hash_messages(*e.pack(batches[i]))]
        except Exception as x:  # surfaced below
            errs.append(repr(x))

    own = [Engine(staging_bytes=1 << 20, io_threads=2) for _ in range(3)]
    shared = Engine(staging_bytes=1 << 20, io_threads=2)
    try:
        th = [threading.Thread(target=work, args=(i, own[i] if i < 3 else shared)) for i in range(len(batches))]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
    finally:
        for e in own + [shared]:
            e.close()
    assert not errs, errs
    assert got == want


def test_mid_size_batches_cut_into_slots(oracle, tmp_path):
    """a call of a few slots' worth runs as several alternating slots (the
    reads of one overlap the GPU's work on the other): 500 files (~25 MB)
    through the default 256 MiB staging, every cas_id and checksum exact, a
    1000-byte message batch through the pinned-buffer path likewise"""
    from spacedrive_amd import Engine
    rng = np.random.default_rng(17)
    paths, sizes = [], []
    for i in range(500):
        n = int(rng.integers(1, 102400 + 1))
        p = tmp_path / f"m{i}"
        p.write_bytes(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        paths.append(str(p))
        sizes.append(n)
    with Engine() as e:
        keys, st = e.generate_cas_ids(paths, sizes)
        assert (st == 0).all()
        for i in range(len(paths)):
            assert f"{int(keys[i]):016x}" == oracle.generate_cas_id(paths[i], sizes[i]), i
        d32, st = e.file_checksums(paths[:300])
        assert (st == 0).all()
        for i in range(300):
            assert bytes(d32[i]).hex() == oracle.file_checksum(paths[i]), i
        msgs = [rng.integers(0, 256, int(rng.integers(0, 90000)), dtype=np.uint8).tobytes() for _ in range(600)]
        out = e.hash_messages(*e.pack(msgs))
        for m, d in zip(msgs, out):
            assert bytes(d).hex() == oracle.hash(m)


def test_small_calls_and_metadata_layouts(oracle):
    """the small-call launch path: single messages and batches under the
    shape-sort threshold (128) on the default 256 MiB staging (leaf and finish
    grids sized to the slot), one after another on one context; then 20 000
    messages of 0-100 bytes through 1 MiB staging, whose slots fill with more
    messages than the packed offsets + lengths copy holds (the two-copy
    layout) and end with a partial slot that packs"""
    from spacedrive_amd import Engine
    rng = np.random.default_rng(23)
    with Engine() as e:
        for n in (1, 1, 2, 3, 64, 127, 128, 129):
            msgs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes()
                    for L in rng.integers(0, 300_000 if n < 64 else 40_000, n)]
            out = e.hash_messages(*e.pack(msgs))
            for m, d in zip(msgs, out):
                assert bytes(d).hex() == oracle.hash(m), (n, len(m))
    msgs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in rng.integers(0, 101, 20_000)]
    with Engine(staging_bytes=1 << 20) as e:
        out = e.hash_messages(*e.pack(msgs))
    bad = [i for i, (m, d) in enumerate(zip(msgs, out)) if bytes(d).hex() != oracle.hash(m)]
    assert not bad, bad[:10]


@pytest.mark.parametrize("direct", ["1", "0"])
def test_small_path_calls_direct_results(oracle, tmp_path, monkeypatch, direct):
    """round 6: a small planned batch read into the slot goes up as ONE copy
    (its metadata behind its bytes) and the kernels write its cas keys or
    digests straight into the slot's pinned result words
    (SDCAS_SMALL_DIRECT, default on; 0: the device buffer and a download).
    Path calls of 1-20 files (whole-file and sampled, empty and missing ones
    among them), checksums of small files, and a 600-file call between them on
    the same context: every cas_id, checksum and status equals the oracle's"""
    from spacedrive_amd import Engine
    monkeypatch.setenv("SDCAS_SMALL_DIRECT", direct)
    rng = np.random.default_rng(84)
    paths, sizes = [], []
    for i in range(700):
        n = int(rng.choice([0, 1, 63, 1024, 1025, 102400, 102401, 300_000])) if i % 7 == 0 else \
            int(rng.integers(1, 140_000))
        p = tmp_path / f"s{i}"
        p.write_bytes(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        paths.append(str(p))
        sizes.append(n)
    paths[5] = str(tmp_path / "missing")

    def check(e, lo, hi):
        keys, st = e.generate_cas_ids(paths[lo:hi], sizes[lo:hi])
        for k, i in enumerate(range(lo, hi)):
            if i == 5:
                assert st[k] != 0
                continue
            assert st[k] == 0, (i, st[k])
            assert f"{int(keys[k]):016x}" == oracle.generate_cas_id(paths[i], sizes[i]), (direct, i, sizes[i])

    with Engine() as e:
        lo = 0
        for n in [1, 1, 2, 3, 5, 8, 13, 20, 1, 7]:
            check(e, lo, lo + n)
            lo += n
        check(e, 100, 700)  # a big call on the same context, then small ones again
        for n in [1, 4, 20]:
            check(e, lo, lo + n)
            lo += n
        for i in (0, 1, 2, 3):
            d32, st = e.file_checksums([paths[10 + i]])
            assert st[0] == 0 and bytes(d32[0]).hex() == oracle.file_checksum(paths[10 + i])
