"""bench.py's N > 1 plumbing on CPU: the max-over-ranks reduction that turns
per-rank timings into the job's time and the sum that totals the per-rank
parity samples (the driver launches bench.py with one rank per GPU; here
gloo, world 2 and 3, one process per rank)."""
import os
import socket
import tempfile

import pytest
import torch


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    import torch.distributed as dist

    import bench
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        got = bench.max_over_ranks(torch, dist, torch.device("cpu"), [1.0 + rank, 10.0 - rank, 0.5])
        tot = bench.sum_over_ranks(torch, dist, torch.device("cpu"), [2000 + rank, rank])
        with open(os.path.join(outdir, f"r{rank}.txt"), "w") as f:
            f.write(" ".join(repr(x) for x in got + tot))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_max_over_ranks_gloo(world):
    with tempfile.TemporaryDirectory() as d:
        torch.multiprocessing.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        for r in range(world):
            vals = [float(x) for x in open(os.path.join(d, f"r{r}.txt")).read().split()]
            assert vals == [float(world), 10.0, 0.5, float(2000 * world + world * (world - 1) // 2),
                            float(world * (world - 1) // 2)]


# --- `bench.py --gpus N` without a launcher: bench.py starts the ranks itself

def test_check_world():
    import bench
    assert bench.check_world(1, {}) is None
    assert bench.check_world(8, {}) == "spawn"
    assert bench.check_world(2, {"WORLD_SIZE": "2"}) is None
    assert "disagree" in bench.check_world(2, {"WORLD_SIZE": "1"})
    assert "disagree" in bench.check_world(1, {"WORLD_SIZE": "4"})
    assert "must be" in bench.check_world(0, {})


def test_gpus_world_mismatch_fails_loudly():
    """--gpus 2 under a launch of one rank exits non-zero before any GPU or
    torch work and prints nothing on stdout (no JSON line to misread)"""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode != 0
    assert r.stdout == ""
    assert "WORLD_SIZE=1" in r.stderr


_RANK_SCRIPT = r'''
import json, os, sys
import torch.distributed as dist
dist.init_process_group("gloo")
import torch
t = torch.tensor([int(os.environ["RANK"]) + 1])
dist.all_reduce(t)
if int(os.environ["RANK"]) == 0:
    print(json.dumps({"world": dist.get_world_size(), "sum": int(t), "argv": sys.argv[1:],
                      "local": [os.environ["LOCAL_RANK"]], "addr": os.environ["MASTER_ADDR"]}))
if os.environ.get("FAIL_RANK") == os.environ["RANK"]:
    sys.exit(3)
dist.destroy_process_group()
'''


@pytest.mark.parametrize("world", [2, 4])
def test_launch_ranks_spawns_a_world(world, tmp_path, capfd):
    """launch_ranks gives each child the torchrun environment: the children
    form one gloo world of `world` ranks over 127.0.0.1, see the parent's
    arguments, and only rank 0's line reaches stdout"""
    import bench
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT)
    rc = bench.launch_ranks(world, ["--gpus", str(world), "--steps", "1"], script=str(script))
    assert rc == 0
    # (gloo's own "[Gloo] Rank ..." banners also go to stdout here; bench.py
    # moves them to stderr in its ranks)
    out = [ln for ln in capfd.readouterr().out.splitlines() if ln.startswith("{")]
    assert len(out) == 1
    import json
    d = json.loads(out[0])
    assert d == {"world": world, "sum": world * (world + 1) // 2, "argv": ["--gpus", str(world), "--steps", "1"],
                 "local": ["0"], "addr": "127.0.0.1"}


def test_launch_ranks_reports_a_failed_rank(tmp_path, monkeypatch):
    import bench
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT)
    monkeypatch.setenv("FAIL_RANK", "1")
    assert bench.launch_ranks(2, [], script=str(script)) == 3
