#!/usr/bin/env python3
"""ORACLE — TEST INFRASTRUCTURE ONLY. Generates the committed golden fixtures
under tests/golden/ from an implementation that is independent of this repo:
the upstream BLAKE3 C library exported as ``llvm_blake3_*`` by two libraries
of this image (BLAKE3 1.3.1 in libLLVM-15, BLAKE3 1.8.2 in ROCm's
libclang-cpp). Every value is computed by BOTH builds and must agree.

The Rust reference cannot be built here (no cargo/rustc, crate ``blake3``
1.5.0 not vendored — SURVEY.md §8c), so the fixtures pin:

* ``blake3_vectors.json`` — BLAKE3 of the official ``i % 251`` input pattern
  at lengths exercising every block/chunk/tree boundary;
* ``cas_ids.json`` — cas_id of files of chosen sizes and contents, where the
  message is built by THIS script following core/src/object/cas.rs:23-62
  (le64(size) || whole file, or header / 4 samples at 8192 + k*jump / footer)
  and hashed by llvm_blake3;
* ``checksums.json`` — file_checksum (core/src/object/validation/hash.rs:11-25)
  = BLAKE3 of the full content, up to 4 GiB + 1 byte.

Contents are either the ``i % 251`` pattern or the synthetic stream of
include/sdcas_synth.h (re-implemented here in numpy). Run from the repo root:
``python oracle/gen_golden.py``. Never runs on the GPU box.
"""
import ctypes
import json
import os
import sys

import numpy as np

LIBS = {
    "1.8.2": "/opt/rocm-7.2.0/lib/llvm/lib/libclang-cpp.so.22.0git",
    "1.3.1": "/usr/lib/x86_64-linux-gnu/libLLVM-15.so.1",
}
HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "..", "tests", "golden")

# cas.rs:10-15
SAMPLE_COUNT = 4
SAMPLE_SIZE = 10240
HEADER_OR_FOOTER_SIZE = 8192
MINIMUM_FILE_SIZE = 102400

M64 = (1 << 64) - 1


class UpstreamBlake3:
    """ctypes view of llvm_blake3_hasher_{init,update,finalize} (no header is
    installed; the hasher struct is ~1.9 KB, 4 KB is allocated)."""

    def __init__(self, path):
        self.lib = ctypes.CDLL(path)
        self.lib.llvm_blake3_version.restype = ctypes.c_char_p
        self.version = self.lib.llvm_blake3_version().decode()
        self.lib.llvm_blake3_hasher_update.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        self.lib.llvm_blake3_hasher_finalize.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]

    def hasher(self):
        h = ctypes.create_string_buffer(4096)
        self.lib.llvm_blake3_hasher_init(h)
        return h

    def update(self, h, data):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        self.lib.llvm_blake3_hasher_update(h, data.ctypes.data, data.size)

    def finalize(self, h):
        out = ctypes.create_string_buffer(32)
        self.lib.llvm_blake3_hasher_finalize(h, out, 32)
        return out.raw.hex()


# ---- contents --------------------------------------------------------------

def mix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def content_key(seed, cid):
    with np.errstate(over="ignore"):
        return int(mix64(np.uint64(seed) ^ (np.uint64(cid) * np.uint64(0xD1B54A32D192ED03))))


def content(spec, off, n):
    """bytes [off, off+n) of a content stream"""
    if n <= 0:
        return np.zeros(0, np.uint8)
    if spec["kind"] == "pattern251":
        return (np.arange(off, off + n, dtype=np.uint64) % np.uint64(251)).astype(np.uint8)
    key = spec["key"]
    w0, w1 = off // 8, (off + n + 7) // 8
    with np.errstate(over="ignore"):
        words = mix64(np.uint64(key) + np.arange(w0, w1, dtype=np.uint64))
    b = words.view(np.uint8)
    s = off - 8 * w0
    return b[s:s + n].copy()


def cas_message_parts(spec, size):
    """cas.rs:23-62 message construction (file content == `size` bytes)"""
    parts = [np.frombuffer(int(size).to_bytes(8, "little"), dtype=np.uint8)]
    if size <= MINIMUM_FILE_SIZE:
        parts.append(content(spec, 0, size))
    else:
        parts.append(content(spec, 0, HEADER_OR_FOOTER_SIZE))
        jump = (size - HEADER_OR_FOOTER_SIZE * 2) // SAMPLE_COUNT
        for k in range(SAMPLE_COUNT):
            parts.append(content(spec, HEADER_OR_FOOTER_SIZE + k * jump, SAMPLE_SIZE))
        parts.append(content(spec, size - HEADER_OR_FOOTER_SIZE, HEADER_OR_FOOTER_SIZE))
    return parts


def hash_both(libs, feed):
    outs = {}
    for ver, lib in libs.items():
        h = lib.hasher()
        for part in feed():
            lib.update(h, part)
        outs[ver] = lib.finalize(h)
    vals = set(outs.values())
    assert len(vals) == 1, f"upstream builds disagree: {outs}"
    return vals.pop()


def stream(spec, size, step=64 << 20):
    def gen():
        off = 0
        while off < size:
            n = min(step, size - off)
            yield content(spec, off, n)
            off += n
        if size == 0:
            yield np.zeros(0, np.uint8)
    return gen


def main():
    libs = {v: UpstreamBlake3(p) for v, p in LIBS.items() if os.path.exists(p)}
    if len(libs) < 2:
        print("need both llvm_blake3 builds", file=sys.stderr)
        sys.exit(1)
    for v, lib in libs.items():
        assert lib.version == v, (v, lib.version)
    os.makedirs(GOLDEN, exist_ok=True)
    pat = {"kind": "pattern251"}

    # 1) BLAKE3 vectors over the official i%251 input
    lens = [0, 1, 2, 7, 8, 63, 64, 65, 127, 128, 129, 1023, 1024, 1025, 2048, 2049, 3072, 3073,
            4096, 4097, 5120, 5121, 6144, 6145, 7168, 7169, 8192, 8193, 16384, 31744, 57352,
            65536, 102408, 1048575, 1048576, 1048577]
    vec = [{"len": n, "hash": hash_both(libs, stream(pat, n))} for n in lens]
    with open(os.path.join(GOLDEN, "blake3_vectors.json"), "w") as f:
        json.dump({"input": "byte i = i % 251", "source": "llvm_blake3 1.3.1 + 1.8.2",
                   "cases": vec}, f, indent=1)

    # 2) cas_ids
    sizes = [0, 1, 63, 64, 65, 1015, 1016, 1017, 1023, 1024, 1025, 2040, 2041, 65536, 102399,
             102400, 102401, 102402, 102403, 114688, 1048576, 1048577, (1 << 30) + 3]
    cases = []
    for spec_name, spec in [("pattern251", pat),
                            ("synth:0x5D0001:7", {"kind": "synth", "key": content_key(0x5D0001, 7)})]:
        for s in sizes:
            parts = cas_message_parts(spec, s)
            msg_len = int(sum(p.size for p in parts))
            h = hash_both(libs, lambda parts=parts: iter(parts))
            cases.append({"content": spec_name, "size": s, "msg_len": msg_len, "cas_id": h[:16],
                          "digest": h})
    with open(os.path.join(GOLDEN, "cas_ids.json"), "w") as f:
        json.dump({"message": "cas.rs:23-62 construction, hashed by llvm_blake3 1.3.1 + 1.8.2",
                   "cases": cases}, f, indent=1)

    # 3) checksums (full content)
    MiB = 1 << 20
    csizes = [0, 1, 1023, 1024, 1025, MiB - 1, MiB, MiB + 1, 3 * MiB + 17]
    big = [(4 << 30) + 1]
    cks = []
    for spec_name, spec in [("pattern251", pat),
                            ("synth:0x5D0004:3", {"kind": "synth", "key": content_key(0x5D0004, 3)})]:
        for s in csizes + (big if spec_name == "pattern251" else []):
            cks.append({"content": spec_name, "size": s, "checksum": hash_both(libs, stream(spec, s))})
    with open(os.path.join(GOLDEN, "checksums.json"), "w") as f:
        json.dump({"message": "full file content (hash.rs:11-25), llvm_blake3 1.3.1 + 1.8.2",
                   "cases": cks}, f, indent=1)

    # 4) synthetic-stream spot values (pins include/sdcas_synth.h's generator)
    spots = []
    for seed, cid, off in [(0x5D0002, 0, 0), (0x5D0002, 1, 13), (0x5D0003, 999, 4097),
                           (0x5D0004, 12345, (3 << 30) + 5)]:
        k = content_key(seed, cid)
        spots.append({"seed": seed, "cid": cid, "off": off, "key": k,
                      "bytes": content({"kind": "synth", "key": k}, off, 16).tobytes().hex()})
    with open(os.path.join(GOLDEN, "synth_spots.json"), "w") as f:
        json.dump({"cases": spots}, f, indent=1)
    print("wrote", GOLDEN)


if __name__ == "__main__":
    main()
