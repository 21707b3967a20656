"""ctypes binding of libsdcas.so (include/sdcas.h, include/sdcas_bench.h).

The library is the product: every hash and every dedup result comes from its
HIP kernels. Importing this module without the built library, or calling it
without a GPU, raises — there is no CPU fallback.

`use_ablation_library()` (tools/ab_leaf.py only) binds libsdcas_ablate.so
instead: the same sources built with every A/B kernel variant, including
diagnostic ones that produce wrong digests. Nothing in the package calls it.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsdcas.so")
ABLATION_LIB_PATH = os.path.join(_HERE, "libsdcas_ablate.so")

SDCAS_OK = 0
SDCAS_E_NO_DEVICE = -1
SDCAS_E_INVALID = -2
SDCAS_E_OOM = -3
SDCAS_E_HIP = -4
SDCAS_E_CAPACITY = -5
SDCAS_E_CANCELLED = -6
SDCAS_STATUS_UNEXPECTED_EOF = 100001
SDCAS_STATUS_CANCELLED = 125
SDCAS_MAX_BATCH = 0x7FFFFFFF
SDCAS_OPT_DIRECT_IO = 1
SDCAS_ABI_VERSION = 6
SDCAS_META_HAS_CAS_ID = 1
SDCAS_META_DIR = 2
SDCAS_LINK_DROPPED = -(1 << 63)
SDCAS_LINK_DEFERRED = SDCAS_LINK_DROPPED + 1
SDCAS_PLAN_HEADER_WORDS = 12

# every entry point include/sdcas.h and include/sdcas_bench.h declare
ABI_SYMBOLS = [
    "sdcas_version", "sdcas_abi_version", "sdcas_init", "sdcas_destroy", "sdcas_last_error", "sdcas_cas_ids",
    "sdcas_file_metadata",
    "sdcas_checksums", "sdcas_hash_messages", "sdcas_cas_ids_from_messages", "sdcas_dev_reserve",
    "sdcas_dev_hash_messages", "sdcas_dev_sync", "sdcas_dev_bind_stream", "sdcas_dedup", "sdcas_dedup_window", "sdcas_job_plan",
    "sdcas_key_to_hex",
    "sdcas_digest_to_hex", "sdcas_cas_message_len", "sdcas_dev_dedup_combine", "sdcas_dev_dedup_combine_async",
    "sdcas_dev_dedup_resolve",
    "sdcas_dev_dedup_apply", "sdcas_dev_dedup_local", "sdcas_dev_dedup_combine_buckets",
    "sdcas_dev_dedup_resolve_buckets", "sdcas_dev_dedup_stays", "sdcas_dev_dedup_plan", "sdcas_dev_stream_begin", "sdcas_dev_stream_update",
    "sdcas_dev_stream_finish", "sdcas_dev_stream_node_bytes", "sdcas_dev_stream_export", "sdcas_dev_stream_import",
    "sdcas_set_progress", "sdcas_node_init", "sdcas_node_destroy", "sdcas_node_last_error", "sdcas_node_size",
    "sdcas_node_uses_rccl", "sdcas_node_set_progress", "sdcas_node_cas_ids", "sdcas_node_checksums",
    "sdcas_node_dedup_window",
    # bench / test plumbing
    "sdcas_dev_synth_cas_messages", "sdcas_dev_synth_content", "sdcas_dev_dedup", "sdcas_dev_profile",
    "sdcas_dev_last_kernel_ms", "sdcas_dev_set_leaf_variant", "sdcas_dev_set_piece_variant", "sdcas_dev_set_sort",
]


class SdcasError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"sdcas error {code}: {msg}")
        self.code = code


class Cancelled(SdcasError):
    """SDCAS_E_CANCELLED: the call stopped at the cancel flag. `partial` holds
    what the call returns normally (results and per-item status); items with
    status SDCAS_STATUS_CANCELLED were not completed, the others are final."""

    def __init__(self, msg, partial=None):
        super().__init__(SDCAS_E_CANCELLED, msg)
        self.partial = partial


# void (*)(void* user, uint64_t done, uint64_t total)
PROGRESS_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64)


class Options(ctypes.Structure):
    """sdcas_options; struct_size is set to this layout's size"""
    _fields_ = [("struct_size", ctypes.c_uint32), ("device", ctypes.c_int32), ("io_threads", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("staging_bytes", ctypes.c_uint64),
                ("progress", PROGRESS_FN),
                ("progress_user", ctypes.c_void_p), ("cancel", ctypes.POINTER(ctypes.c_int32))]

    def __init__(self, *a, **k):
        super().__init__(ctypes.sizeof(Options), *a, **k)


class JobWindow(ctypes.Structure):
    """sdcas_job_window"""
    _fields_ = [("max_steps", ctypes.c_uint64), ("more", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("steps", ctypes.c_uint64), ("rows", ctypes.c_uint64), ("rereads", ctypes.c_uint64)]


_lib = None
_lib_path = LIB_PATH


def use_ablation_library():
    """Bind libsdcas_ablate.so (A/B tools only; see the module docstring).
    Must be called before the first load()."""
    global _lib_path
    if _lib is not None and _lib_path != ABLATION_LIB_PATH:
        raise RuntimeError("libsdcas.so is already loaded in this process")
    _lib_path = ABLATION_LIB_PATH

_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_u64 = ctypes.c_uint64


def load():
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: PyTorch-ROCm bundles its own
    # libamdhip64.so.7 / libhsa-runtime64.so.1 (same SONAMEs as /opt/rocm's).
    # If torch is importable it is loaded FIRST so that the dynamic linker
    # binds libsdcas.so to torch's already-loaded runtime instead of opening
    # a second HSA runtime on the same GPU (which leaves torch with "No HIP
    # GPUs are available"). Without torch, /opt/rocm's runtime is used.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(_lib_path):
        raise ImportError(f"{_lib_path} is not built: run `make -C spacedrive_amd/csrc` "
                          "(or __graft_entry__.build()) — there is no CPU fallback")
    L = ctypes.CDLL(_lib_path)
    L.sdcas_version.restype = ctypes.c_char_p
    L.sdcas_abi_version.restype = ctypes.c_int
    if L.sdcas_abi_version() != SDCAS_ABI_VERSION:
        raise ImportError(f"{_lib_path} has C ABI {L.sdcas_abi_version()}, this binding {SDCAS_ABI_VERSION}: rebuild")
    L.sdcas_init.argtypes = [ctypes.POINTER(Options), ctypes.POINTER(_vp)]
    L.sdcas_destroy.argtypes = [_vp]
    L.sdcas_last_error.argtypes = [_vp]
    L.sdcas_last_error.restype = ctypes.c_char_p
    L.sdcas_cas_ids.argtypes = [_vp, _vp, _vp, _sz, _vp, _vp]
    L.sdcas_file_metadata.argtypes = [_vp, _vp, _vp, _sz, _vp, _vp, _vp, _vp]
    L.sdcas_checksums.argtypes = [_vp, _vp, _sz, _vp, _vp]
    L.sdcas_hash_messages.argtypes = [_vp, _vp, _vp, _vp, _sz, _vp]
    L.sdcas_cas_ids_from_messages.argtypes = [_vp, _vp, _vp, _vp, _sz, _vp]
    L.sdcas_dev_reserve.argtypes = [_vp, _sz, _u64]
    L.sdcas_dev_hash_messages.argtypes = [_vp, _vp, _vp, _vp, _sz, _vp, _vp, _vp]
    L.sdcas_dev_sync.argtypes = [_vp, _vp]
    L.sdcas_dev_bind_stream.argtypes = [_vp, _vp, ctypes.c_uint64]
    L.sdcas_dedup.argtypes = [_vp, _vp, _vp, _vp, _sz, _sz, _vp, _sz, _vp, _vp, _vp]
    L.sdcas_job_plan.argtypes = [_vp, _vp, _sz, _sz, ctypes.POINTER(JobWindow), _vp, _vp]
    L.sdcas_dedup_window.argtypes = [_vp, _vp, _vp, _vp, _sz, _sz, _vp, _sz, ctypes.POINTER(JobWindow), _vp, _vp,
                                     _vp]
    L.sdcas_key_to_hex.argtypes = [_u64, ctypes.c_char_p]
    L.sdcas_digest_to_hex.argtypes = [_vp, ctypes.c_char_p]
    L.sdcas_cas_message_len.argtypes = [_u64]
    L.sdcas_cas_message_len.restype = _u64
    L.sdcas_dev_synth_cas_messages.argtypes = [_vp, _vp, _vp, _vp, _sz, _vp, _vp]
    L.sdcas_dev_synth_content.argtypes = [_vp, _vp, _vp, _vp, _vp, _sz, _vp, _vp]
    L.sdcas_dev_dedup.argtypes = [_vp, _vp, _vp, _vp, _sz, _sz, _vp, _vp, _vp]
    L.sdcas_dev_profile.argtypes = [_vp, ctypes.c_int]
    L.sdcas_dev_last_kernel_ms.argtypes = [_vp, ctypes.POINTER(ctypes.c_float),
                                           ctypes.POINTER(ctypes.c_float)]
    L.sdcas_dev_set_leaf_variant.argtypes = [_vp, ctypes.c_int]
    L.sdcas_dev_set_piece_variant.argtypes = [_vp, ctypes.c_int]
    L.sdcas_dev_set_sort.argtypes = [_vp, ctypes.c_int]
    L.sdcas_set_progress.argtypes = [_vp, PROGRESS_FN, _vp, ctypes.POINTER(ctypes.c_int32)]
    L.sdcas_dev_dedup_combine_buckets.argtypes = [_vp, _vp, _vp, _vp, _vp, _sz, ctypes.c_uint32, _sz, _vp, _vp,
                                                  _vp, _vp, _vp]
    L.sdcas_dev_dedup_resolve_buckets.argtypes = [_vp, _vp, _sz, _vp, _vp, _sz, _vp, ctypes.c_uint32, _vp, _vp]
    L.sdcas_dev_dedup_combine.argtypes = [_vp, _vp, _vp, _vp, _vp, _sz, ctypes.c_uint32, _vp, _vp, _vp, _vp]
    L.sdcas_dev_dedup_combine_async.argtypes = [_vp, _vp, _vp, _vp, _vp, _sz, ctypes.c_uint32, _vp, _vp, _vp, _vp]
    L.sdcas_dev_dedup_resolve.argtypes = [_vp, _vp, _sz, _vp, _sz, _vp, _vp]
    L.sdcas_dev_dedup_apply.argtypes = [_vp, _vp, _vp, _sz, _vp, _sz, _vp, _vp, _vp, _vp]
    L.sdcas_dev_dedup_local.argtypes = [_vp, _vp, _vp, _vp, _vp, _sz, _vp, _vp, _sz, _sz, _u64, _u64,
                                        ctypes.c_uint32, _vp, _vp, _vp, _vp]
    L.sdcas_dev_dedup_stays.argtypes = [_vp, _vp, _vp, _vp, _sz, _sz, _vp, _vp, _vp]
    L.sdcas_dev_dedup_plan.argtypes = [_vp, _vp, _sz, _u64, _sz, _u64, ctypes.c_uint32, _vp, _vp]
    L.sdcas_dev_stream_begin.argtypes = [_vp, _vp, _sz]
    L.sdcas_dev_stream_update.argtypes = [_vp, _sz, _vp, _vp, _vp, _vp, _vp]
    L.sdcas_dev_stream_finish.argtypes = [_vp, _vp, _vp]
    L.sdcas_dev_stream_node_bytes.argtypes = [_vp]
    L.sdcas_dev_stream_node_bytes.restype = _sz
    L.sdcas_dev_stream_export.argtypes = [_vp, _vp, _sz, _vp]
    L.sdcas_dev_stream_import.argtypes = [_vp, _vp, _sz, _vp]
    L.sdcas_node_init.argtypes = [_vp, _sz, ctypes.POINTER(Options), ctypes.POINTER(_vp)]
    L.sdcas_node_destroy.argtypes = [_vp]
    L.sdcas_node_last_error.argtypes = [_vp]
    L.sdcas_node_last_error.restype = ctypes.c_char_p
    L.sdcas_node_size.argtypes = [_vp]
    L.sdcas_node_size.restype = _sz
    L.sdcas_node_uses_rccl.argtypes = [_vp]
    L.sdcas_node_set_progress.argtypes = [_vp, PROGRESS_FN, _vp, ctypes.POINTER(ctypes.c_int32)]
    L.sdcas_node_cas_ids.argtypes = [_vp, _vp, _vp, _sz, _vp, _vp]
    L.sdcas_node_checksums.argtypes = [_vp, _vp, _sz, _vp, _vp]
    L.sdcas_node_dedup_window.argtypes = [_vp, _vp, _vp, _vp, _sz, _sz, _vp, _sz, ctypes.POINTER(JobWindow), _vp,
                                          _vp, _vp]
    _lib = L
    return L
