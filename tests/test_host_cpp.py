"""The C++ host mirror of sd-core's interface (include/sdcore.hpp,
spacedrive_amd/host/sdcore.cpp) through its test program tests/cpp/test_sdcore:
generate_cas_id / file_checksum (single and batched) against the oracle, per-file
errors (ENOENT, UnexpectedEof), FileMetadata::new, the file identifier job at
batch 100 (the reference's CHUNK_SIZE) and 1000 against the oracle's chunked
dedup, and the object validator job."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "build", "test_sdcore")


def _build():
    if not os.path.exists(BIN):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], check=True)
    return BIN


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is present (the gpu test covers this box)")
def test_engine_open_fails_loudly_without_gpu():
    r = subprocess.run([_build(), "--no-gpu"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "LibraryError" in r.stdout


def test_host_library_links_the_c_abi():
    lib = os.path.join(ROOT, "spacedrive_amd", "libsdcore.so")
    out = subprocess.run(["ldd", lib], capture_output=True, text=True).stdout
    assert "libsdcas.so" in out and "not found" not in out.split("libsdcas.so")[1].split("\n")[0]
    syms = subprocess.run(["nm", "-DC", "--defined-only", lib], capture_output=True, text=True).stdout
    for name in ("sdcore::generate_cas_id", "sdcore::file_checksum", "sdcore::identifier_job_step",
                 "sdcore::run_file_identifier_job", "sdcore::run_object_validator_job",
                 "sdcore::file_metadata_batch", "sdcore::Engine::open", "sdcore::object_kind_of",
                 "sdcore::resolve_conflicting_kind", "sdcore::extension_kinds"):
        assert name in syms, name


def test_db_side_sqlite_vs_memory():
    """the DB side of the identifier join: SqliteLibrary
    queries and a simulated identifier job equal MemoryLibrary's, with and
    without the cas_id index (CPU only; tests/cpp/test_sdcore_db.cpp)"""
    db_bin = os.path.join(ROOT, "tests", "cpp", "build", "test_sdcore_db")
    if not os.path.exists(db_bin):
        _build()
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], check=True)
    r = subprocess.run([db_bin], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_host_mirror_on_gpu():
    r = subprocess.run([_build()], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout + r.stderr
