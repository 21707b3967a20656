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
