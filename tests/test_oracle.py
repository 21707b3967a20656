"""CPU tests: the oracle against the golden vectors (upstream BLAKE3 C,
llvm_blake3 1.3.1 + 1.8.2) and SURVEY.md Appendix B; the dedup restatement
against hand-derived cases of core/src/object/file_identifier/mod.rs."""
import os

import numpy as np
import pytest

from tests._oracle import (cas_windows, content, content_key, golden, mix64, spec_content,
                           write_sparse_file)

APPENDIX_B = {0: "71e0a99173564931", 1: "9b779f74b305adc3", 1016: "c0de16cef5f85601",
              1017: "62fe3d833d2df619", 102400: "c66a52267c7e5ee9", 102401: "17f74805066119da",
              1048576: "5aefa86eb26df03d"}


def test_blake3_vectors(oracle):
    for c in golden("blake3_vectors.json"):
        data = content("pattern251", 0, c["len"])
        assert oracle.hash(data.tobytes()) == c["hash"], c["len"]


def test_cas_messages_match_golden(oracle):
    for c in golden("cas_ids.json"):
        if c["size"] > (1 << 22):
            continue
        kind, key = spec_content(c["content"])
        parts = [np.frombuffer(c["size"].to_bytes(8, "little"), np.uint8)]
        parts += [content(kind, o, n, key) for o, n in cas_windows(c["size"])]
        msg = np.concatenate(parts)
        assert msg.size == c["msg_len"]
        assert f"{oracle.cas_key_of_message(msg):016x}" == c["cas_id"]


def test_appendix_b(oracle):
    cases = {c["size"]: c["cas_id"] for c in golden("cas_ids.json") if c["content"] == "pattern251"}
    for size, want in APPENDIX_B.items():
        assert cases[size] == want


def test_generate_cas_id_real_files(oracle, tmp_path):
    """cas.rs:23-62 through real file I/O (sparse files for the big ones)"""
    for c in golden("cas_ids.json"):
        kind, key = spec_content(c["content"])
        p = tmp_path / f"f_{c['content'].replace(':', '_')}_{c['size']}"
        write_sparse_file(p, kind, key, c["size"], cas_windows(c["size"]))
        assert oracle.generate_cas_id(str(p), c["size"]) == c["cas_id"], c


def test_file_checksum_real_files(oracle, tmp_path):
    for c in golden("checksums.json"):
        if c["size"] > (8 << 20):
            continue
        kind, key = spec_content(c["content"])
        p = tmp_path / f"c_{c['size']}"
        p.write_bytes(content(kind, 0, c["size"], key).tobytes())
        assert oracle.file_checksum(str(p)) == c["checksum"], c


def test_synth_checksum(oracle):
    for c in golden("checksums.json"):
        if c["content"].startswith("synth") and c["size"] < (4 << 20):
            _, key = spec_content(c["content"])
            assert oracle.synth_checksum(key, c["size"]) == c["checksum"]


def test_synth_generator_spots():
    for c in golden("synth_spots.json"):
        assert content_key(c["seed"], c["cid"]) == c["key"]
        assert content("synth", c["off"], 16, c["key"]).tobytes().hex() == c["bytes"]


def test_synth_cas_key_matches_message(oracle):
    rng = np.random.default_rng(1)
    for size in [0, 1, 1016, 5000, 102400, 102401, 300000, 7 << 20]:
        key = int(rng.integers(0, 2**63))
        msg = oracle.synth_cas_message(key, size)
        parts = [np.frombuffer(size.to_bytes(8, "little"), np.uint8)]
        parts += [content("synth", o, n, key) for o, n in cas_windows(size)]
        assert np.array_equal(msg, np.concatenate(parts))
        assert oracle.synth_cas_key(key, size) == oracle.cas_key_of_message(msg)


def test_short_file_unexpected_eof(oracle, tmp_path):
    """a file that is shorter than the size the indexer recorded fails with
    UnexpectedEof in read_exact (cas.rs:36,43,56)"""
    p = tmp_path / "short"
    p.write_bytes(b"x" * 20000)
    with pytest.raises(OSError) as e:
        oracle.generate_cas_id(str(p), 200000)
    assert e.value.errno == 100001


def test_missing_file_errno(oracle, tmp_path):
    with pytest.raises(OSError) as e:
        oracle.generate_cas_id(str(tmp_path / "nope"), 10)
    assert e.value.errno == 2


# ---- dedup restatement (file_identifier/mod.rs:98-350) ----------------------

def test_dedup_semantics(oracle):
    # chunk size 3: chunk0 = files 0,1,2; chunk1 = 3,4,5; chunk2 = 6
    keys = np.array([10, 10, 11, 10, 12, 11, 99], np.uint64)
    has = np.array([1, 1, 1, 1, 1, 1, 0], np.uint8)
    out, created, linked = oracle.identifier_dedup(keys, has, chunk_size=3)
    # chunk0: 10 and 10 are intra-chunk duplicates -> two Objects (mod.rs:246-254)
    # chunk1: 10 links to the first Object with cas 10 (file 0); 11 links to file 2; 12 new
    # chunk2: None cas_id -> new Object
    assert out.tolist() == [0, 1, 2, 0, 4, 2, 6]
    assert created == 5 and linked == 2


def test_dedup_existing_and_errors(oracle):
    keys = np.array([5, 6, 5, 7], np.uint64)
    has = np.ones(4, np.uint8)
    status = np.array([0, 0, 0, 2], np.int32)
    out, created, linked = oracle.identifier_dedup(keys, has, status, chunk_size=100,
                                                   existing_keys=[6, 6, 9])
    # 6 links to the FIRST existing Object carrying it; file 3 failed -> dropped
    # same chunk: both 5s are new Objects
    assert out.tolist() == [0, -1, 2, np.iinfo(np.int64).min]
    assert created == 2 and linked == 1


MIN = np.iinfo(np.int64).min
DEFERRED = MIN + 1


def test_dedup_last_row_none_is_read_again(oracle):
    """file_identifier_job.rs:296-319 + mod.rs:401-405: the next step starts AT
    the previous step's last row (id >= cursor); a row with cas_id None keeps
    cas_id NULL, stays an orphan (file_identifier_job.rs:258-264) and, being
    the last row, is read again and gets a second Object (mod.rs:246-254)"""
    keys = np.array([10, 11, 0, 10, 12, 11, 13], np.uint64)
    has = np.array([1, 1, 0, 1, 1, 1, 1], np.uint8)
    out, created, linked, win = oracle.identifier_job(keys, has, chunk_size=3)
    # step 1: rows 0,1,2 (2 is None: new Object); step 2: rows 2,3,4 (2 again:
    # another Object; 3 links to 0; 4 new); step 3: rows 5,6 (5 links to 1)
    assert out.tolist() == [0, 1, 2, 0, 4, 1, 6]
    assert (created, linked) == (6, 2)
    assert win == {"steps": 3, "rows": 7, "rereads": 1}


def test_dedup_error_at_chunk_end_shifts_boundaries(oracle):
    """an errored last row shifts every later chunk: rows 4 and 5 (same
    cas_id) land in different steps, so 5 links to 4's Object instead of
    creating its own; the fixed 3-row chunks would give 6 Objects"""
    keys = np.array([1, 2, 0, 3, 4, 4, 6], np.uint64)
    has = np.ones(7, np.uint8)
    status = np.array([0, 0, 5, 0, 0, 0, 0], np.int32)
    out, created, linked, win = oracle.identifier_job(keys, has, status, chunk_size=3)
    assert out.tolist() == [0, 1, MIN, 3, 4, 4, 6]
    assert (created, linked) == (5, 1)
    assert win == {"steps": 3, "rows": 7, "rereads": 1}


def test_dedup_task_count_leaves_tail_for_next_job(oracle):
    """task_count = ceil(orphans / 100) is fixed at init (file_identifier_job.rs:146):
    a re-read costs a row of the budget, so the last row is not reached"""
    keys = np.array([1, 2, 0, 3, 4, 5], np.uint64)
    status = np.array([0, 0, 5, 0, 0, 0], np.int32)
    out, created, linked, win = oracle.identifier_job(keys, np.ones(6, np.uint8), status, chunk_size=3)
    assert out.tolist() == [0, 1, MIN, 3, 4, DEFERRED]
    assert (created, linked) == (4, 0)
    assert win == {"steps": 2, "rows": 5, "rereads": 1}


def test_dedup_window_of_a_longer_job(oracle):
    """a batch of the job (more orphans follow): a step that would reach past
    the batch is left to the next batch, whose cursor is row rows-1"""
    keys = np.array([1, 2, 0, 3, 4], np.uint64)
    has = np.array([1, 1, 0, 1, 1], np.uint8)
    out, created, linked, win = oracle.identifier_job(keys, has, chunk_size=3, max_steps=10, more=True)
    assert out.tolist() == [0, 1, 2, 3, 4] and (created, linked) == (6, 0)
    assert win == {"steps": 2, "rows": 5, "rereads": 1}
    out, created, linked, win = oracle.identifier_job(np.array([1, 2, 3, 4], np.uint64), np.ones(4, np.uint8),
                                                      chunk_size=3, max_steps=10, more=True)
    assert out.tolist() == [0, 1, 2, DEFERRED] and win == {"steps": 1, "rows": 3, "rereads": 0}
    # the budget caps a window too
    out, _, _, win = oracle.identifier_job(np.arange(9, dtype=np.uint64), np.ones(9, np.uint8), chunk_size=3,
                                           max_steps=2)
    assert out.tolist() == list(range(6)) + [DEFERRED] * 3 and win["steps"] == 2 and win["rows"] == 6


def test_dedup_batches_equal_the_100_row_job(oracle):
    """a job run in windows of 1000 rows, each window's next cursor from the
    oracle's `rows`, equals the job run 100 rows at a time over the same rows:
    the windows reproduce the 100-row chunks exactly (the re-read row is the
    next window's first row)"""
    rng = np.random.default_rng(3)
    n = 5000
    pool = rng.integers(0, 2**64, 600, dtype=np.uint64)
    keys = pool[rng.integers(0, 600, n)]
    has = (rng.random(n) > 0.05).astype(np.uint8)
    status = np.where(rng.random(n) < 0.05, 5, 0).astype(np.int32)
    # force stay-orphans onto many chunk ends
    has[99::100] = 0
    status[198::100] = 7
    whole, wc, wl, ww = oracle.identifier_job(keys, has, status, 100)
    assert ww["rereads"] >= 5
    for batch in (100, 300, 1000, 4096):
        link = np.full(n, DEFERRED, np.int64)
        start, steps_left, created, linked = 0, (n + 99) // 100, 0, 0
        obj_key, obj_row = [], []  # the library's Objects with a cas_id, DB (creation) order
        while steps_left and start < n:
            hi = min(n, start + batch)
            out, c, l, w = oracle.identifier_job(keys[start:hi], has[start:hi], status[start:hi], 100,
                                                 np.array(obj_key, np.uint64), max_steps=steps_left, more=hi < n)
            if w["steps"] == 0:
                break
            for i in range(int(w["rows"])):
                v = int(out[i])
                if v == DEFERRED:
                    continue
                link[start + i] = v + start if v >= 0 else (v if v == MIN else obj_row[-v - 1])
            for i in range(int(w["rows"])):
                if int(out[i]) == i and has[start + i] and status[start + i] == 0:
                    obj_key.append(keys[start + i])
                    obj_row.append(start + i)
            created += c
            linked += l
            steps_left -= int(w["steps"])
            start += int(w["rows"]) - 1  # the cursor row: read again if it is still an orphan
            if start < n and status[start] == 0 and has[start]:
                start += 1  # no longer an orphan: the next query skips it
        assert (created, linked) == (wc, wl), batch
        assert np.array_equal(link, whole), batch


def test_mix64_python_matches_header():
    # sds_mix64(0) reference value computed from the header's definition
    assert int(mix64(np.uint64(0))) == 0xE220A8397B1DCDAF


def test_cpu_bench_files_keys(oracle):
    """bench.py's CPU-baseline leg (oracle_cpu_bench_files) hashes the same
    cas messages / whole-file contents as the per-file oracle"""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from spacedrive_amd import synth as S
    sizes = np.array([0, 1, 1023, 1024, 1025, 102400, 102401, 300_000, 5 << 20], np.uint64)
    ckeys = np.array([S.content_key(S.SEED_C3, i) for i in range(sizes.size)], np.uint64)
    want = np.array([oracle.synth_cas_key(int(k), int(s)) for k, s in zip(ckeys, sizes)], np.uint64)
    base, par = bench.cpu_baseline_files(want, sizes, ckeys, 0, 2, "unit")
    assert par["mismatches"] == 0 and base["unit"] == "files/s"
    sel = sizes <= (1 << 20)
    want1 = np.array([int(oracle.synth_checksum(int(k), int(s))[:16], 16) for k, s in zip(ckeys[sel], sizes[sel])],
                     np.uint64)
    base, par = bench.cpu_baseline_files(want1, sizes[sel], ckeys[sel], 1, 2, "unit")
    assert par["mismatches"] == 0 and base["unit"] == "GB/s"


def test_periodic_checksum_matches_whole_hash(oracle):
    """oracle/periodic.c (the >= 4 TiB fixture's construction) equals the
    whole-message hash of materialised periodic messages, scalar and upstream"""
    period = content("pattern251", 0, 1 << 20)
    for plen in (1024, 8192, 1 << 20):
        p = period[:plen]
        for total in (plen + 1, 3 * plen + 17, 8 * plen, 13 * plen + plen // 2 + 1, (24 << 20) + 1025):
            want = oracle.hash(np.resize(p, total).tobytes())
            assert oracle.periodic_checksum(p, total, upstream=False) == want, (plen, total)
            assert oracle.periodic_checksum(p, total, upstream=True) == want, (plen, total)


def test_subtree_cv_high_counter(oracle):
    """chunk counters >= 2^32 (the high word v13): the scalar oracle's subtree
    CVs equal upstream BLAKE3 C 1.8.2's (llvm_blake3_compress_subtree_wide),
    and the high word changes the result"""
    p = content("pattern251", 0, 1 << 20)
    cvs = {}
    for c in (0, (1 << 32) - 1024, 1 << 32, (1 << 32) + 1024, (3 << 32) + (5 << 10), (1 << 52)):
        cvs[c] = oracle.subtree_cv(p, c, upstream=False)
        assert cvs[c] == oracle.subtree_cv(p, c, upstream=True), c
    assert cvs[0] != cvs[1 << 32]
    small = p[:4096]
    assert oracle.subtree_cv(small, 1 << 32, False) == oracle.subtree_cv(small, 1 << 32, True)


def test_periodic_golden_is_large():
    """the periodic fixture reaches chunk counters >= 2^32"""
    cases = golden("checksums_periodic.json")
    assert cases and all(c["size"] > (4 << 40) for c in cases)


def test_synth_cas_keys_mt_matches_per_file(oracle):
    """the multi-threaded checker of the -m gpu corpus tests equals the
    per-file scalar oracle, with upstream SIMD BLAKE3 and with the scalar
    restatement"""
    from spacedrive_amd import synth as S
    sizes, ckeys, _ = S.c3_files(0, 400)
    want = np.array([oracle.synth_cas_key(int(k), int(s)) for k, s in zip(ckeys, sizes)], np.uint64)
    for up in (True, False):
        got, _ = oracle.synth_cas_keys(ckeys, sizes, threads=3, upstream=up)
        assert np.array_equal(got, want)


def test_cpu_faithful_matches_generate_cas_id(oracle, tmp_path):
    """bench.py's reference-faithful CPU leg reads real files with cas.rs's
    pattern in 100-file steps: its keys and statuses equal the per-file oracle
    (whole files, sampled sparse files, a short file, a missing one), over
    several steps and with ragged last steps"""
    from tests._oracle import cas_windows, write_sparse_file
    rng = np.random.default_rng(5)
    sizes = [int(x) for x in rng.integers(0, 102400, 180)] + [102401, 5 << 20, 1 << 30, 0, 1]
    paths = []
    for i, s in enumerate(sizes):
        p = tmp_path / f"f{i}"
        write_sparse_file(p, "synth", 1000 + i, s, cas_windows(s))
        paths.append(str(p))
    short = tmp_path / "short"
    short.write_bytes(b"y" * 50000)
    paths += [str(short), str(tmp_path / "missing")]
    sizes += [300000, 10]
    for chunk in (100, 7):
        keys, st, secs, _ = oracle.cpu_faithful(paths, sizes, chunk=chunk, io_threads=4)
        assert secs > 0
        for i, (p, s) in enumerate(zip(paths, sizes)):
            try:
                want = oracle.generate_cas_id(p, s)
            except OSError as e:
                assert st[i] == e.errno, (i, st[i])
                continue
            assert st[i] == 0 and f"{int(keys[i]):016x}" == want, i
