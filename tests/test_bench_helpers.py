"""bench.py's pricing helpers (CPU): the compression count the VALU roofline
is priced on, the dedup's algorithmic bytes, the peaks, and the lookups of
the committed PMC traffic passes the lines carry (profiles/)."""
import numpy as np
import pytest

import bench


def _compressions_by_definition(L):
    # one compression per 64-byte block of each 1 KiB chunk (an empty message
    # still compresses one block), one per parent node: C - 1 for C chunks
    C = max(1, -(-L // 1024))
    blocks = sum(max(1, -(-min(1024, L - 1024 * c) // 64)) for c in range(C))
    return blocks + (C - 1)


def test_compressions_match_the_definition():
    lens = np.array([0, 1, 63, 64, 65, 1023, 1024, 1025, 2048, 2049, 57352, 102408, 1 << 20, (1 << 20) + 17])
    got = bench.compressions(lens)
    assert [int(x) for x in got] == [_compressions_by_definition(int(L)) for L in lens]


def test_dedup_bytes():
    assert bench.dedup_bytes(0) == 0
    assert bench.dedup_bytes(6_250_000) == 156_250_000  # the C5 share's 156.3 MB
    assert bench.dedup_bytes(10, 3) == 25 * 10 + 16 * 3


def test_peaks():
    # spec lane rate: 256 CUs x 4 SIMD x 32 lanes x 2.4 GHz; 680 lane-ops per compression
    assert bench.VALU_PEAK_OPS / bench.OPS_PER_COMPRESSION / 1e9 == pytest.approx(115.66, abs=0.01)
    # the ISA issue model: 77.4 G compressions/s at 2.4 GHz
    assert bench.VALU_PEAK_ISA / 1e9 == pytest.approx(77.4, abs=0.1)
    assert bench.HBM_PEAK_GBS == 8000.0


def test_committed_traffic_passes_are_found():
    """the C2 / C3 / C5 leaf lines find their PMC traffic files (the lines'
    `roofline.traffic`) under the default kernel's name, old or new, and the
    C3 / C5 dedup lines theirs (`dedup.roofline.traffic`)"""
    for w in ("c2", "c3", "c5"):
        t = bench.load_traffic(w, bench.DEFAULT_LEAF_KERNEL)
        assert t is not None, w
        assert t["hbm_bytes_per_launch"] > 0
    assert "k_leaf_tree<512, 279, 1, 1, 2, 2, 0, 1024u, 0>".startswith(bench.DEFAULT_LEAF_KERNEL)
    for w, n in (("c5", 6_250_000), ("c3", 1_250_000)):
        d = bench.load_dedup_traffic(w, n)
        assert d is not None, w


def test_c5_shares_keep_the_corpus_mix_at_any_size():
    """bench.c5_share: the full-size shares are the corpus' files 8i + r (the
    committed C5 lines' workload), and a small share still carries the
    corpus' duplicates — the Zipf head on every rank, links within a rank and
    across ranks"""
    from spacedrive_amd import synth as S
    n = 6_250_000
    for world, rank in ((1, 0), (8, 0), (8, 5)):
        got = bench.c5_share(rank, 1000, world) if world == 1 else None
        full = bench.c5_share(rank, n, world)
        assert np.array_equal(full[:1000], np.arange(1000) * 8 + (rank if world == 8 else 0))
        if got is not None:
            assert got[0] == 0 and np.all(np.diff(got) > 0)
    for world in (2, 8):
        cids = [S.c5_content_ids_at(bench.c5_share(r, 20_000, world).astype(np.uint64)) for r in range(world)]
        for c in cids:
            assert (c == 0).any()  # the Zipf head
            assert np.unique(c).size < c.size  # duplicates inside a rank
            first = (bench.c5_share(0, 20_000, world) < 20_000_000).mean()
            assert 0.35 < first < 0.45  # ~40 % first copies, as the corpus
        assert np.intersect1d(cids[0], cids[1]).size > 0  # duplicates across ranks
    # shares are disjoint and inside the corpus
    allf = np.concatenate([bench.c5_share(r, 20_000, 8) for r in range(8)])
    assert np.unique(allf).size == allf.size and allf.max() < bench.C5_CORPUS
