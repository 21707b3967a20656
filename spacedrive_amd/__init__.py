"""spacedrive_amd — MI355X-native content identification for Spacedrive sd-core.

Hot path: generate_cas_id (core/src/object/cas.rs:23-62),
file_checksum (core/src/object/validation/hash.rs:11-25) and the cas_id ->
Object dedup of core/src/object/file_identifier/mod.rs:98-350, executed by the
HIP kernels of libsdcas.so (spacedrive_amd/csrc) through the C ABI of
include/sdcas.h.
"""
from .engine import (Engine, Node, default_engine, digest_to_hex, file_checksum, generate_cas_id, io_error,
                     key_to_hex)

__all__ = ["Engine", "Node", "default_engine", "digest_to_hex", "file_checksum", "generate_cas_id", "io_error",
           "key_to_hex"]
