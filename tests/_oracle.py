"""ctypes loader for the CPU oracle (oracle/build/liboracle.so).

Test infrastructure only: the oracle is the checker, never the thing measured
or shipped. Builds the library with `make -C oracle` when it is missing and a
compiler is present (both here and on the GPU box, which has the same image).
"""
import ctypes
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
LIB = os.path.join(ROOT, "oracle", "build", "liboracle.so")

_u64p = ctypes.POINTER(ctypes.c_uint64)


LINK_DROPPED = np.iinfo(np.int64).min
LINK_DEFERRED = LINK_DROPPED + 1


class JobWindow(ctypes.Structure):
    """oracle_job_window (oracle/oracle.h), the layout of sdcas_job_window"""
    _fields_ = [("max_steps", ctypes.c_uint64), ("more", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("steps", ctypes.c_uint64), ("rows", ctypes.c_uint64), ("rereads", ctypes.c_uint64)]


class Oracle:
    def __init__(self, lib):
        self.lib = lib
        L = lib
        L.b3ref_hash.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.oracle_generate_cas_id.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
        L.oracle_generate_cas_id.restype = ctypes.c_int
        L.oracle_file_checksum.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_file_checksum.restype = ctypes.c_int
        L.oracle_cas_key_of_message.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_cas_key_of_message.restype = ctypes.c_uint64
        L.oracle_synth_cas_key.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_synth_cas_key.restype = ctypes.c_uint64
        L.oracle_synth_checksum.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_synth_cas_message.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_synth_cas_message.restype = ctypes.c_size_t
        L.oracle_identifier_dedup.argtypes = [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_identifier_dedup.restype = ctypes.c_int64
        L.oracle_identifier_job.argtypes = [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p,
                                            ctypes.POINTER(JobWindow), ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_identifier_job.restype = ctypes.c_int64
        L.oracle_subtree_cv.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int,
                                        ctypes.c_void_p]
        L.oracle_periodic_checksum.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_void_p]
        L.oracle_synth_cas_keys_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_void_p]
        L.oracle_synth_cas_keys_mt.restype = ctypes.c_int
        L.oracle_cpu_faithful.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int),
                                          ctypes.c_char_p]
        L.oracle_cpu_faithful.restype = ctypes.c_int

    def hash(self, data: bytes) -> str:
        buf = np.frombuffer(bytes(data), dtype=np.uint8)
        out = ctypes.create_string_buffer(32)
        self.lib.b3ref_hash(buf.ctypes.data if buf.size else None, buf.size, out)
        return out.raw.hex()

    def generate_cas_id(self, path, size):
        out = ctypes.create_string_buffer(17)
        st = self.lib.oracle_generate_cas_id(os.fsencode(path), size, out)
        if st:
            raise OSError(st, f"oracle generate_cas_id status {st}")
        return out.value.decode()

    def file_checksum(self, path):
        out = ctypes.create_string_buffer(65)
        st = self.lib.oracle_file_checksum(os.fsencode(path), out)
        if st:
            raise OSError(st, f"oracle file_checksum status {st}")
        return out.value.decode()

    def cas_key_of_message(self, msg: np.ndarray) -> int:
        msg = np.ascontiguousarray(msg, dtype=np.uint8)
        return int(self.lib.oracle_cas_key_of_message(msg.ctypes.data if msg.size else None, msg.size))

    def synth_cas_key(self, content_key, size):
        return int(self.lib.oracle_synth_cas_key(content_key, size))

    def synth_cas_message(self, content_key, size):
        n = size + 8 if size <= 102400 else 57352
        out = np.zeros(n, np.uint8)
        self.lib.oracle_synth_cas_message(content_key, size, out.ctypes.data)
        return out

    def synth_checksum(self, content_key, size):
        out = ctypes.create_string_buffer(32)
        self.lib.oracle_synth_checksum(content_key, size, out)
        return out.raw.hex()

    def subtree_cv(self, data: np.ndarray, counter: int, upstream: bool) -> bytes:
        """CV of the complete subtree `data` (2^k chunks) starting at chunk `counter`"""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        out = ctypes.create_string_buffer(32)
        rc = self.lib.oracle_subtree_cv(data.ctypes.data, data.size, counter, int(upstream), out)
        assert rc == 0, rc
        return out.raw

    def periodic_checksum(self, period: np.ndarray, total: int, upstream: bool, threads: int = 4) -> str:
        """BLAKE3 of `total` bytes of `period` (2^k chunks) repeated (oracle/periodic.c)"""
        period = np.ascontiguousarray(period, dtype=np.uint8)
        out = ctypes.create_string_buffer(32)
        rc = self.lib.oracle_periodic_checksum(period.ctypes.data, period.size, total, threads, int(upstream), out)
        assert rc == 0, rc
        return out.raw.hex()

    def synth_cas_keys(self, content_keys, sizes, threads=16, upstream=True):
        """every cas key of synthetic files (content key, size), multi-threaded
        -> (keys uint64[n], hasher) with hasher 'upstream' (BLAKE3 C SIMD) or 'scalar'"""
        ck = np.ascontiguousarray(content_keys, dtype=np.uint64)
        sz = np.ascontiguousarray(sizes, dtype=np.uint64)
        out = np.zeros(ck.size, np.uint64)
        up = self.lib.oracle_synth_cas_keys_mt(ck.ctypes.data, sz.ctypes.data, ck.size, threads, int(upstream),
                                               out.ctypes.data)
        return out, ("upstream" if up else "scalar")

    def cpu_faithful(self, paths, sizes, chunk=100, io_threads=16, upstream=True):
        """the identifier job's CPU shape over real files (oracle/cpu_bench.c
        oracle_cpu_faithful) -> (keys, status, seconds, hasher)"""
        n = len(paths)
        parr = (ctypes.c_char_p * max(n, 1))(*[os.fsencode(p) for p in paths])
        sz = np.ascontiguousarray(sizes, dtype=np.uint64)
        keys = np.zeros(n, np.uint64)
        st = np.zeros(n, np.int32)
        secs = ctypes.c_double(0)
        kind = ctypes.c_int(0)
        ver = ctypes.create_string_buffer(32)
        rc = self.lib.oracle_cpu_faithful(parr, sz.ctypes.data, n, chunk, io_threads, int(upstream), keys.ctypes.data,
                                          st.ctypes.data, ctypes.byref(secs), ctypes.byref(kind), ver)
        assert rc == 0, rc
        hasher = f"upstream BLAKE3 C {ver.value.decode()} SIMD" if kind.value else "scalar BLAKE3 restatement"
        return keys, st, secs.value, hasher

    def identifier_dedup(self, keys, has_key, status=None, chunk_size=100, existing_keys=()):
        """the file identifier job over these orphans -> (link, created, linked)"""
        link, created, linked, _ = self.identifier_job(keys, has_key, status, chunk_size, existing_keys)
        return link, created, linked

    def identifier_job(self, keys, has_key, status=None, chunk_size=100, existing_keys=(), max_steps=0,
                       more=False):
        """oracle_identifier_job -> (link, created, linked, window dict)"""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        n = keys.size
        has_key = np.ascontiguousarray(has_key, dtype=np.uint8)
        st = None if status is None else np.ascontiguousarray(status, dtype=np.int32)
        ex = np.ascontiguousarray(existing_keys, dtype=np.uint64)
        out = np.zeros(n, np.int64)
        linked = ctypes.c_int64(0)
        win = JobWindow(max_steps, int(bool(more)), 0, 0, 0, 0)
        created = self.lib.oracle_identifier_job(
            n, keys.ctypes.data, has_key.ctypes.data, None if st is None else st.ctypes.data,
            chunk_size, ex.size, ex.ctypes.data if ex.size else None, ctypes.byref(win), out.ctypes.data,
            ctypes.byref(linked))
        return out, int(created), int(linked.value), {"steps": win.steps, "rows": win.rows, "rereads": win.rereads}


def build_oracle():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


def load_oracle():
    if not os.path.exists(LIB):
        build_oracle()
    return Oracle(ctypes.CDLL(LIB))


def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)["cases"]


# ---- python restatement of include/sdcas_synth.h (for fixture building) ----

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


def content(kind, off, n, key=0):
    if n <= 0:
        return np.zeros(0, np.uint8)
    if kind == "pattern251":
        return (np.arange(off, off + n, dtype=np.uint64) % np.uint64(251)).astype(np.uint8)
    w0, w1 = off // 8, (off + n + 7) // 8
    with np.errstate(over="ignore"):
        words = mix64(np.uint64(key) + np.arange(w0, w1, dtype=np.uint64))
    b = words.view(np.uint8)
    s = off - 8 * w0
    return b[s:s + n].copy()


def spec_content(spec_name):
    """'pattern251' or 'synth:<seed>:<cid>' -> (kind, key)"""
    if spec_name == "pattern251":
        return "pattern251", 0
    _, seed, cid = spec_name.split(":")
    return "synth", content_key(int(seed, 16), int(cid))


def write_sparse_file(path, kind, key, size, windows):
    """Create a file of `size` bytes whose content is correct on `windows`
    (list of (off, n)); the rest is a hole. Enough for cas_id, which only
    reads the sampled windows of large files."""
    with open(path, "wb") as f:
        f.truncate(size)
        for off, n in windows:
            f.seek(off)
            f.write(content(kind, off, n, key).tobytes())


def cas_windows(size):
    """byte windows of a file that cas.rs:23-62 reads"""
    if size <= 102400:
        return [(0, size)]
    jump = (size - 16384) // 4
    w = [(0, 8192)] + [(8192 + k * jump, 10240) for k in range(4)] + [(size - 8192, 8192)]
    return w
