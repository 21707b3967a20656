"""The host side of a small staging batch's slot plan (b3_batch.h BatchPlan,
sdcas::batch_plan_host in libsdcas.so; no GPU call), CPU suite: the C++ test
tests/cpp/test_batch_plan.cpp checks it against a slot-by-slot restatement of
the device scan + k_tile_first over edge and random batches of 1-127
messages, tiles of 128 and 1024 slots. The device side (the leaf kernel on a
host plan) is tests/test_gpu_hash.py::test_host_planned_small_batches."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")


def test_batch_plan_host():
    r = subprocess.run(["make", "-s", "-C", CPP, "build/test_batch_plan"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    r = subprocess.run([os.path.join(CPP, "build", "test_batch_plan")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ALL OK" in r.stdout, (r.stdout + r.stderr)[-4000:]
