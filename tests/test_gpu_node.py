"""A node: one process driving several GPU contexts (sdcas_node_*,
spacedrive_amd.Node) — sd-core is one process (apps/server/src/main.rs:40,
job/manager.rs:32), so the multi-GPU paths must be reachable without a
process per GPU. On this one-GPU box the node is [0, 0] (up to eight
contexts, [0] * 8: the layout sd-core's one process would drive on an
8-GPU node, include/sdcas.h:395-427) on one device, the exchange as
device-to-device copies — the default between
distinct devices too (over xGMI); RCCL (ncclCommInitAll) is opt-in with
SDCAS_NODE_EXCHANGE=rccl and unmeasured here.
Everything against the oracle."""
import numpy as np
import pytest

from tests._dist_stages import make_corpus
from tests._oracle import cas_windows, content, content_key, write_sparse_file

pytestmark = pytest.mark.gpu
MiB = 1 << 20


@pytest.fixture(scope="module", params=[(0,), (0, 0), (0, 0, 0), (0,) * 8], ids=["node1", "node2", "node3", "node8"])
def node(request):
    from spacedrive_amd import Node
    n = Node(devices=request.param, staging_bytes=16 * MiB)
    assert n.size == len(request.param) and not n.uses_rccl
    yield n
    n.close()


def test_node_dedup_vs_oracle(node, oracle):
    """stays + plan on every context, records to their owner context, resolve,
    answers back: the links and counts of the job over these orphans"""
    for seed, p_none, p_err, cs in ((3, 0.02, 0.01, 100), (4, 0.2, 0.2, 100), (5, 0.05, 0.05, 7)):
        keys, has, status, existing = make_corpus(seed, 30000, pool=5000, p_none=p_none, p_err=p_err)
        want, wc, wl, ww = oracle.identifier_job(keys, has, status, cs, existing)
        got, gc, gl, gw = node.identifier_dedup_window(keys, has, status, cs, existing)
        assert np.array_equal(got, want), seed
        assert (gc, gl) == (wc, wl) and gw == ww, seed
    # a window of a longer job, and no existing Objects at all
    keys, has, status, existing = make_corpus(6, 12345, p_none=0.1, p_err=0.1)
    want, wc, wl, ww = oracle.identifier_job(keys, has, status, 100, (), 70, True)
    got, gc, gl, gw = node.identifier_dedup_window(keys, has, status, 100, (), 70, True)
    assert np.array_equal(got, want) and (gc, gl) == (wc, wl) and gw == ww
    # fewer files than contexts
    got, gc, gl, gw = node.identifier_dedup_window(keys[:1], has[:1], status[:1], 100, existing[:3])
    want, wc, wl, ww = oracle.identifier_job(keys[:1], has[:1], status[:1], 100, existing[:3])
    assert np.array_equal(got, want) and (gc, gl) == (wc, wl)


def test_node_dedup_waits_once_per_phase(node, oracle, monkeypatch, capfd):
    """every context's combine (files and existing Objects) is enqueued before
    the host reads any owner range: the trace shows ONE host wait for the
    owner ranges and one for the results, whatever the number of contexts"""
    keys, has, status, existing = make_corpus(11, 20000, pool=3000, p_none=0.05, p_err=0.05)
    capfd.readouterr()
    monkeypatch.setenv("SDCAS_NODE_TRACE", "1")
    got, gc, gl, gw = node.identifier_dedup_window(keys, has, status, 100, existing)
    monkeypatch.delenv("SDCAS_NODE_TRACE")
    err = capfd.readouterr().err
    waits = [ln for ln in err.splitlines() if ln.startswith("sdcas_node: host wait")]
    assert waits == [f"sdcas_node: host wait [owner ranges] over {node.size} ranks",
                     f"sdcas_node: host wait [results] over {node.size} ranks"], err
    want, wc, wl, ww = oracle.identifier_job(keys, has, status, 100, existing)
    assert np.array_equal(got, want) and (gc, gl) == (wc, wl) and gw == ww


def test_node_cas_ids_and_checksums(node, oracle, tmp_path):
    """files sharded over the contexts (contiguous ranges by cas-message bytes;
    checksums largest file first): every key and digest exact, errors in place"""
    rng = np.random.default_rng(9)
    paths, sizes = [], []
    for i in range(400):
        size = int(rng.choice([0, 1, 1017, 60_000, 102_400, 102_401, 3 * MiB + 7]))
        k = content_key(0x5D0003, 5000 + i)
        p = tmp_path / f"f{i}"
        write_sparse_file(str(p), "synth", k, size, cas_windows(size))
        paths.append(str(p))
        sizes.append(size)
    paths.append(str(tmp_path / "missing"))
    sizes.append(10)
    keys, st = node.generate_cas_ids(paths, sizes)
    assert st[-1] == 2 and not st[:-1].any()
    for i in range(0, 400, 7):
        assert f"{int(keys[i]):016x}" == oracle.generate_cas_id(paths[i], sizes[i]), i
    big = []
    for i, size in enumerate([2 * MiB + 3, 5000, 9 * MiB, 1, 0, MiB + 1]):
        p = tmp_path / f"c{i}"
        p.write_bytes(content("synth", 0, size, content_key(0x5D0004, i)).tobytes())
        big.append(str(p))
    out, st = node.file_checksums(big + [str(tmp_path / "missing")])
    assert st[-1] == 2 and not st[:-1].any()
    for i, p in enumerate(big):
        assert bytes(out[i]).hex() == oracle.file_checksum(p), p


def c5_share_keys(oracle, n, world=8):
    """real cas keys (upstream BLAKE3 C) of an even sample of the C5 corpus
    (bench.c5_share: the Zipf head and ~60 % duplicates at any size)"""
    import bench
    sizes, ckeys, _ = bench.files_of("c5", 0, n, world)
    keys, _ = oracle.synth_cas_keys(ckeys, sizes, threads=16)
    return keys, sizes


def test_node_dedup_c5_share_waits_per_phase(node, oracle, monkeypatch, capfd):
    """sdcas_node_dedup_window over a C5 share with the Zipf head (one
    content carries ~7 % of the files, so one owner context receives far more
    records than the others), existing Objects present: links and counts
    against the oracle, two host waits, and the per-phase wait times the
    trace reports (printed: gpurun logs keep them)"""
    keys, sizes = c5_share_keys(oracle, 160_000)
    rng = np.random.default_rng(41)
    has = (sizes != 0).astype(np.uint8)
    status = np.where(rng.random(keys.size) < 0.003, 5, 0).astype(np.int32)
    existing = np.concatenate([keys[rng.choice(keys.size, 2000, replace=False)],
                               rng.integers(0, 2**64, 400, dtype=np.uint64)])
    assert 1 - np.unique(keys).size / keys.size > 0.4  # the share duplicates as the corpus does
    want, wc, wl, ww = oracle.identifier_job(keys, has, status, 100, existing)
    for rep in range(2):  # the second call on warm buffers
        capfd.readouterr()
        monkeypatch.setenv("SDCAS_NODE_TRACE", "1")
        got, gc, gl, gw = node.identifier_dedup_window(keys, has, status, 100, existing)
        monkeypatch.delenv("SDCAS_NODE_TRACE")
        err = capfd.readouterr().err
        assert np.array_equal(got, want), rep
        assert (gc, gl) == (wc, wl) and gw == ww, rep
        waits = [ln for ln in err.splitlines() if ln.startswith("sdcas_node: host wait")]
        assert len(waits) == 2, err
        waited = [ln for ln in err.splitlines() if ln.startswith("sdcas_node: waited")]
        assert len(waited) == 2, err
        with capfd.disabled():
            print(f"\n[node{node.size} c5 share {keys.size} files, call {rep}] " + " | ".join(waited))
