#!/usr/bin/env python3
"""ORACLE — TEST INFRASTRUCTURE ONLY. Generates tests/golden/checksums_periodic.json:
file_checksum (core/src/object/validation/hash.rs:11-25) of files larger than
4 TiB, whose chunk counters need their high 32-bit word (BLAKE3 v13), a path
no whole-message fixture of gen_golden.py can reach here.

Content: byte i of the file is (i mod 2^20) mod 251, i.e. one 1 MiB period of
the official ``i % 251`` pattern repeated; every full period is a complete
level-10 subtree of the BLAKE3 tree whose chaining value is computed by the
upstream BLAKE3 C 1.8.2 (``llvm_blake3_compress_subtree_wide`` in ROCm's
libclang-cpp) at that period's chunk counter, and the subtree list is merged
by oracle/periodic.c with the crate's stack rule. tests/test_oracle.py pins
that construction against whole-message hashes of materialised periodic
messages and the scalar oracle's subtree CVs at counters around 2^32.

Run from the repo root after ``make -C oracle``: ``python oracle/gen_golden_periodic.py``
(about 10 minutes on 8 cores). Never runs on the GPU box.
"""
import ctypes
import json
import os
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "..", "tests", "golden")
MiB = 1 << 20
TiB = 1 << 40
SIZES = [4 * TiB + MiB + 17]


def main():
    L = ctypes.CDLL(os.path.join(HERE, "build", "liboracle.so"))
    L.oracle_periodic_checksum.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_void_p]
    assert L.oracle_periodic_upstream_available(), "llvm_blake3_compress_subtree_wide not found"
    period = (np.arange(MiB, dtype=np.uint64) % np.uint64(251)).astype(np.uint8)
    cases = []
    for n in SIZES:
        t = time.time()
        out = ctypes.create_string_buffer(32)
        rc = L.oracle_periodic_checksum(period.ctypes.data, MiB, n, os.cpu_count() or 1, 1, out)
        assert rc == 0, rc
        cases.append({"size": n, "checksum": out.raw.hex()})
        print(f"{n}: {out.raw.hex()} ({time.time() - t:.0f} s)", flush=True)
    doc = {
        "content": "byte i = (i mod 2^20) mod 251 (a 1 MiB period of the i % 251 pattern)",
        "period": MiB,
        "oracle": "upstream BLAKE3 C 1.8.2 llvm_blake3_compress_subtree_wide per period + oracle/periodic.c stack merge",
        "cases": cases,
    }
    with open(os.path.join(GOLDEN, "checksums_periodic.json"), "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
