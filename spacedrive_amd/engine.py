"""Host-side mirror of sd-core's content-identification interface over the
libsdcas.so C ABI.

The reference functions keep their names, argument meaning and error
behaviour:

* ``generate_cas_id(path, size) -> str`` — core/src/object/cas.rs:23-62
  (16 lowercase hex chars; io errors raise ``OSError``; a file shorter than
  the windows ``size`` implies raises ``OSError(UnexpectedEof, "failed to
  fill whole buffer")`` like tokio's read_exact);
* ``file_checksum(path) -> str`` — core/src/object/validation/hash.rs:11-25
  (64 lowercase hex chars);
* ``identifier_dedup(...)`` — the cas_id -> Object link of
  core/src/object/file_identifier/mod.rs:98-350 in canonical form.

The batch forms (``generate_cas_ids``, ``file_checksums``,
``hash_messages``) are what the identifier/validator jobs would call once per
chunk instead of per file. Everything runs on the GPU; there is no CPU path.
"""
import ctypes
import itertools
import os
import sys

import numpy as np

from . import _native as N



_STREAM_TOKENS = itertools.count(1)  # sdcas_dev_bind_stream tokens: unique per process

def _cpaths(paths):
    """(buffer, pointers) for a `const char* const*` argument: the paths
    NUL-terminated in ONE bytes buffer and a uint64 array of their addresses
    (one numpy pass instead of a ctypes object per path — the per-path form
    cost more than the library's reads of 200 K files). Keep `buffer` alive
    for the call."""
    n = len(paths)
    if n == 0:
        return None, np.zeros(1, np.uint64)
    try:  # the common case, a list of str: one join, one encode
        enc = ("\0".join(paths) + "\0").encode(sys.getfilesystemencoding(), "surrogateescape")
    except TypeError:  # bytes or os.PathLike items
        enc = b"\0".join(os.fsencode(p) for p in paths) + b"\0"
    buf = np.frombuffer(enc, np.uint8)
    ends = np.flatnonzero(buf == 0)
    if len(ends) != n:
        raise ValueError("a path contains a NUL byte")
    ptrs = np.empty(n, np.uint64)
    ptrs[0] = 0
    ptrs[1:] = ends[:-1] + 1
    ptrs += np.uint64(buf.ctypes.data)
    return buf, ptrs


def _arr(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def _ptr(a):
    return a.ctypes.data if a is not None and a.size else None


def key_to_hex(key: int) -> str:
    return f"{int(key):016x}"


def digest_to_hex(d) -> str:
    return bytes(np.asarray(d, dtype=np.uint8)).hex()


def io_error(status: int, path=None) -> OSError:
    if status == N.SDCAS_STATUS_UNEXPECTED_EOF:
        e = OSError(status, "failed to fill whole buffer")
    else:
        e = OSError(status, os.strerror(status) if status < 4096 else f"status {status}")
    if path is not None:
        e.filename = str(path)
    return e


class Engine:
    """One libsdcas context bound to one GPU.

    progress: optional callable(done_bytes, total_bytes), called on the
    calling thread after every staging slot of a path call (the job's
    progress report, job/worker.rs:458-480). cancel: optional
    ``ctypes.c_int32`` the caller may set nonzero from any thread to stop a
    path call (job/mod.rs:862-960); the call then raises ``Cancelled`` whose
    ``partial`` holds the completed items. direct_io: the path calls
    (generate_cas_ids, file_checksums) read with O_DIRECT (cold storage).
    """

    def __init__(self, device: int = 0, io_threads: int = 0, staging_bytes: int = 0, progress=None, cancel=None,
                 direct_io=False):
        self.L = N.load()
        self._cb = self._progress_fn(progress)
        self._cancel = cancel
        opts = N.Options(device, io_threads, N.SDCAS_OPT_DIRECT_IO if direct_io else 0, staging_bytes, self._cb,
                         None, ctypes.pointer(cancel) if cancel is not None else None)
        ctx = ctypes.c_void_p()
        rc = self.L.sdcas_init(ctypes.byref(opts), ctypes.byref(ctx))
        if rc != N.SDCAS_OK:
            raise N.SdcasError(rc, "sdcas_init failed (no HIP device?)")
        self.ctx = ctx

    @staticmethod
    def _progress_fn(progress):
        if progress is None:
            return N.PROGRESS_FN()
        return N.PROGRESS_FN(lambda _user, done, total: progress(int(done), int(total)))

    def set_progress(self, progress=None, cancel=None):
        """re-bind the progress callable and cancel flag (sdcas_set_progress)"""
        cb = self._progress_fn(progress)
        self._check(self.L.sdcas_set_progress(self.ctx, cb, None,
                                              ctypes.pointer(cancel) if cancel is not None else None),
                    "sdcas_set_progress")
        self._cb, self._cancel = cb, cancel

    # -- lifetime -------------------------------------------------------------
    def close(self):
        if getattr(self, "ctx", None):
            self.L.sdcas_destroy(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what, partial=None):
        if rc != N.SDCAS_OK:
            msg = self.L.sdcas_last_error(self.ctx).decode(errors="replace")
            if rc == N.SDCAS_E_CANCELLED:
                raise N.Cancelled(f"{what}: {msg}", partial)
            raise N.SdcasError(rc, f"{what}: {msg}")

    # -- reference functions, batched ------------------------------------------
    def generate_cas_ids(self, paths, sizes):
        """cas.rs:23-62 for many files -> (keys uint64[n], status int32[n])"""
        n = len(paths)
        buf, parr = _cpaths(paths)
        sizes = _arr(sizes, np.uint64)
        keys = np.zeros(n, np.uint64)
        st = np.zeros(n, np.int32)
        self._check(self.L.sdcas_cas_ids(self.ctx, _ptr(parr), _ptr(sizes), n, _ptr(keys), _ptr(st)),
                    "sdcas_cas_ids", (keys, st))
        del buf
        return keys, st

    def file_metadata(self, paths, size_hints=None):
        """FileMetadata::new's fs::metadata + generate_cas_id (mod.rs:48-96) for
        many files, the length from fstat of the read descriptor
        (sdcas_file_metadata; size_hints: the indexer's sizes, which only plan
        the staging) -> (sizes uint64[n], keys uint64[n], status int32[n],
        flags uint8[n]: SDCAS_META_HAS_CAS_ID | SDCAS_META_DIR)"""
        n = len(paths)
        buf, parr = _cpaths(paths)
        hints = _arr(size_hints, np.uint64) if size_hints is not None else None
        sizes = np.zeros(n, np.uint64)
        keys = np.zeros(n, np.uint64)
        st = np.zeros(n, np.int32)
        fl = np.zeros(n, np.uint8)
        self._check(self.L.sdcas_file_metadata(self.ctx, _ptr(parr), _ptr(hints) if hints is not None else None, n,
                                               _ptr(sizes), _ptr(keys), _ptr(st), _ptr(fl)),
                    "sdcas_file_metadata", (sizes, keys, st, fl))
        del buf
        return sizes, keys, st, fl

    def file_checksums(self, paths):
        """hash.rs:11-25 for many files -> (digests uint8[n, 32], status int32[n])"""
        n = len(paths)
        buf, parr = _cpaths(paths)
        out = np.zeros((n, 32), np.uint8)
        st = np.zeros(n, np.int32)
        self._check(self.L.sdcas_checksums(self.ctx, _ptr(parr), n, _ptr(out), _ptr(st)), "sdcas_checksums",
                    (out, st))
        del buf
        return out, st

    def generate_cas_id(self, path, size) -> str:
        keys, st = self.generate_cas_ids([path], [size])
        if st[0]:
            raise io_error(int(st[0]), path)
        return key_to_hex(keys[0])

    def file_checksum(self, path) -> str:
        out, st = self.file_checksums([path])
        if st[0]:
            raise io_error(int(st[0]), path)
        return digest_to_hex(out[0])

    # -- pre-assembled messages ---------------------------------------------------
    @staticmethod
    def pack(messages):
        """list of bytes-like -> (blob, offsets, lens)"""
        lens = np.array([len(m) for m in messages], np.uint64)
        offs = np.zeros(len(messages), np.uint64)
        if len(messages):
            offs[1:] = np.cumsum(lens[:-1])
        blob = np.frombuffer(b"".join(bytes(m) for m in messages), np.uint8) if len(messages) else \
            np.zeros(0, np.uint8)
        return blob, offs, lens

    def hash_messages(self, blob, offsets, lens):
        blob = _arr(blob, np.uint8)
        offsets, lens = _arr(offsets, np.uint64), _arr(lens, np.uint64)
        n = lens.size
        out = np.zeros((n, 32), np.uint8)
        self._check(self.L.sdcas_hash_messages(self.ctx, _ptr(blob) or 1, _ptr(offsets), _ptr(lens), n,
                                               _ptr(out)), "sdcas_hash_messages")
        return out

    def cas_ids_from_messages(self, blob, offsets, lens):
        blob = _arr(blob, np.uint8)
        offsets, lens = _arr(offsets, np.uint64), _arr(lens, np.uint64)
        n = lens.size
        keys = np.zeros(n, np.uint64)
        self._check(self.L.sdcas_cas_ids_from_messages(self.ctx, _ptr(blob) or 1, _ptr(offsets),
                                                       _ptr(lens), n, _ptr(keys)),
                    "sdcas_cas_ids_from_messages")
        return keys

    # -- dedup ------------------------------------------------------------------------
    def identifier_dedup(self, keys, has_key, status=None, chunk_size=100, existing_keys=()):
        """the file identifier job's group-by over these orphans (sdcas_dedup)
        -> (link int64[n], created, linked)"""
        link, created, linked, _ = self.identifier_dedup_window(keys, has_key, status, chunk_size, existing_keys)
        return link, created, linked

    def identifier_dedup_window(self, keys, has_key, status=None, chunk_size=100, existing_keys=(), max_steps=0,
                                more=False):
        """sdcas_dedup_window: the job's steps over one batch of its orphans
        -> (link, created, linked, {"steps", "rows", "rereads"})"""
        keys = _arr(keys, np.uint64)
        n = keys.size
        has_key = _arr(has_key, np.uint8)
        st = None if status is None else _arr(status, np.int32)
        ex = _arr(existing_keys, np.uint64)
        out = np.zeros(n, np.int64)
        created, linked = ctypes.c_int64(0), ctypes.c_int64(0)
        win = N.JobWindow(int(max_steps), int(bool(more)), 0, 0, 0, 0)
        self._check(self.L.sdcas_dedup_window(self.ctx, _ptr(keys), _ptr(has_key), _ptr(st), n, chunk_size,
                                              _ptr(ex), ex.size, ctypes.byref(win), _ptr(out), ctypes.byref(created),
                                              ctypes.byref(linked)), "sdcas_dedup_window")
        return out, created.value, linked.value, {"steps": win.steps, "rows": win.rows, "rereads": win.rereads}

    # -- device-resident (pointers are ints: device addresses, e.g. tensor.data_ptr())
    def dev_reserve(self, max_msgs, max_chunks):
        self._check(self.L.sdcas_dev_reserve(self.ctx, int(max_msgs), int(max_chunks)), "dev_reserve")

    def dev_hash_messages(self, blob, offs, lens, n, out32=0, keys=0, stream=0):
        self._check(self.L.sdcas_dev_hash_messages(self.ctx, blob, offs, lens, int(n), out32 or None,
                                                   keys or None, stream or None), "dev_hash_messages")

    def dev_sync(self, stream=0):
        self._check(self.L.sdcas_dev_sync(self.ctx, stream or None), "dev_sync")

    def dev_bind_stream(self, stream, token=None):
        """name `stream`'s identity (sdcas_dev_bind_stream): consecutive
        device calls on it skip the scratch fence's event wait. token None:
        a fresh one (never reused in this process); 0: unbind"""
        if token is None:
            token = next(_STREAM_TOKENS)
        self._check(self.L.sdcas_dev_bind_stream(self.ctx, stream or None, int(token)), "dev_bind_stream")
        return token

    def dev_synth_cas_messages(self, keys, sizes, offs, n, blob, stream=0):
        self._check(self.L.sdcas_dev_synth_cas_messages(self.ctx, keys, sizes, offs, int(n), blob,
                                                        stream or None), "synth")

    def dev_synth_content(self, keys, starts, lens, offs, n, blob, stream=0):
        self._check(self.L.sdcas_dev_synth_content(self.ctx, keys, starts, lens, offs, int(n), blob,
                                                   stream or None), "synth")

    def dev_dedup(self, keys, has_key, status, n, chunk_size, out_link, counts, stream=0):
        self._check(self.L.sdcas_dev_dedup(self.ctx, keys, has_key, status or None, int(n), chunk_size,
                                           out_link, counts or None, stream or None), "dev_dedup")

    def dev_stream_begin(self, lens):
        """device-resident big-message session (sdcas_dev_stream_*): lens > 1 MiB each"""
        lens = _arr(lens, np.uint64)
        self._check(self.L.sdcas_dev_stream_begin(self.ctx, _ptr(lens), lens.size), "dev_stream_begin")

    def dev_stream_update(self, files, msg_offs, lens, dev_addrs, stream=0):
        f, o, l, a = (_arr(x, np.uint64) for x in (files, msg_offs, lens, dev_addrs))
        self._check(self.L.sdcas_dev_stream_update(self.ctx, f.size, _ptr(f), _ptr(o), _ptr(l), _ptr(a),
                                                   stream or None), "dev_stream_update")

    def dev_stream_node_bytes(self):
        return int(self.L.sdcas_dev_stream_node_bytes(self.ctx))

    def dev_stream_export(self, dst, nbytes, stream=0):
        self._check(self.L.sdcas_dev_stream_export(self.ctx, dst, int(nbytes), stream or None), "dev_stream_export")

    def dev_stream_import(self, src, nbytes, stream=0):
        self._check(self.L.sdcas_dev_stream_import(self.ctx, src, int(nbytes), stream or None), "dev_stream_import")

    def dev_stream_finish(self, out32, stream=0):
        self._check(self.L.sdcas_dev_stream_finish(self.ctx, out32, stream or None), "dev_stream_finish")

    def dev_profile(self, enable=True):
        self._check(self.L.sdcas_dev_profile(self.ctx, 1 if enable else 0), "dev_profile")

    def dev_set_leaf_variant(self, v):
        """tuning knob: leaf/tree kernel variant (-1 = default); False (and the
        selection unchanged) for a variant this build does not hold"""
        return self.L.sdcas_dev_set_leaf_variant(self.ctx, int(v)) == N.SDCAS_OK

    def dev_set_piece_variant(self, v):
        """tuning knob: 1 MiB-piece kernel variant of the checksum path (-1 = default)"""
        return self.L.sdcas_dev_set_piece_variant(self.ctx, int(v)) == N.SDCAS_OK

    def dev_set_sort(self, enable):
        """tuning knob: length-sorted slot order (default on); results identical"""
        self._check(self.L.sdcas_dev_set_sort(self.ctx, 1 if enable else 0), "dev_set_sort")

    def dev_kernel_ms(self):
        a, b = ctypes.c_float(0), ctypes.c_float(0)
        self._check(self.L.sdcas_dev_last_kernel_ms(self.ctx, ctypes.byref(a), ctypes.byref(b)), "ms")
        return a.value, b.value


_default = None


def default_engine() -> Engine:
    global _default
    if _default is None:
        _default = Engine()
    return _default


def generate_cas_id(path, size) -> str:
    """core/src/object/cas.rs:23 — `pub async fn generate_cas_id(path, size) -> Result<String>`"""
    return default_engine().generate_cas_id(path, size)


def file_checksum(path) -> str:
    """core/src/object/validation/hash.rs:11 — `pub async fn file_checksum(path) -> Result<String>`"""
    return default_engine().file_checksum(path)


__all__ = ["Engine", "generate_cas_id", "file_checksum", "key_to_hex", "digest_to_hex", "io_error",
           "default_engine"]


class Node:
    """sdcas_node: one process driving several GPUs (one context per entry of
    `devices`; a device may repeat). The batch calls shard over the contexts
    and the dedup's exchange runs in this process (RCCL between distinct
    devices, device copies otherwise)."""

    def __init__(self, devices=(0,), io_threads: int = 0, staging_bytes: int = 0, direct_io=False, progress=None,
                 cancel=None):
        self.L = N.load()
        self._cb = Engine._progress_fn(progress)
        self._cancel = cancel
        opts = N.Options(-1, io_threads, N.SDCAS_OPT_DIRECT_IO if direct_io else 0, staging_bytes, self._cb,
                         None, ctypes.pointer(cancel) if cancel is not None else None)
        devs = (ctypes.c_int32 * len(devices))(*devices)
        node = ctypes.c_void_p()
        rc = self.L.sdcas_node_init(devs, len(devices), ctypes.byref(opts), ctypes.byref(node))
        if rc != N.SDCAS_OK:
            raise N.SdcasError(rc, "sdcas_node_init failed")
        self.node = node

    @property
    def size(self):
        return int(self.L.sdcas_node_size(self.node))

    @property
    def uses_rccl(self):
        return bool(self.L.sdcas_node_uses_rccl(self.node))

    def close(self):
        if getattr(self, "node", None):
            self.L.sdcas_node_destroy(self.node)
            self.node = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what, partial=None):
        if rc != N.SDCAS_OK:
            msg = self.L.sdcas_node_last_error(self.node).decode(errors="replace")
            if rc == N.SDCAS_E_CANCELLED:
                raise N.Cancelled(f"{what}: {msg}", partial)
            raise N.SdcasError(rc, f"{what}: {msg}")

    def generate_cas_ids(self, paths, sizes):
        n = len(paths)
        buf, parr = _cpaths(paths)
        sizes = _arr(sizes, np.uint64)
        keys = np.zeros(n, np.uint64)
        st = np.zeros(n, np.int32)
        self._check(self.L.sdcas_node_cas_ids(self.node, _ptr(parr), _ptr(sizes), n, _ptr(keys), _ptr(st)),
                    "sdcas_node_cas_ids", (keys, st))
        del buf
        return keys, st

    def file_checksums(self, paths):
        n = len(paths)
        buf, parr = _cpaths(paths)
        out = np.zeros((n, 32), np.uint8)
        st = np.zeros(n, np.int32)
        self._check(self.L.sdcas_node_checksums(self.node, _ptr(parr), n, _ptr(out), _ptr(st)),
                    "sdcas_node_checksums", (out, st))
        del buf
        return out, st

    def identifier_dedup_window(self, keys, has_key, status=None, chunk_size=100, existing_keys=(), max_steps=0,
                                more=False):
        keys = _arr(keys, np.uint64)
        n = keys.size
        has_key = _arr(has_key, np.uint8)
        st = None if status is None else _arr(status, np.int32)
        ex = _arr(existing_keys, np.uint64)
        out = np.zeros(n, np.int64)
        created, linked = ctypes.c_int64(0), ctypes.c_int64(0)
        win = N.JobWindow(int(max_steps), int(bool(more)), 0, 0, 0, 0)
        self._check(self.L.sdcas_node_dedup_window(self.node, _ptr(keys), _ptr(has_key), _ptr(st), n, chunk_size,
                                                   _ptr(ex), ex.size, ctypes.byref(win), _ptr(out),
                                                   ctypes.byref(created), ctypes.byref(linked)),
                    "sdcas_node_dedup_window")
        return out, created.value, linked.value, {"steps": win.steps, "rows": win.rows, "rereads": win.rereads}

    def identifier_dedup(self, keys, has_key, status=None, chunk_size=100, existing_keys=()):
        link, c, l, _ = self.identifier_dedup_window(keys, has_key, status, chunk_size, existing_keys)
        return link, c, l
