"""CPU tests of the boundary: libsdcas.so loads and exports every entry point
include/*.h declares (no compute calls — there is no GPU here)."""
import os
import re
import subprocess

import pytest

from spacedrive_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = set()
    for h in ("sdcas.h", "sdcas_bench.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(sdcas_\w+)\s*\(", src))
    return names


def test_header_and_binding_agree():
    assert declared_symbols() == set(N.ABI_SYMBOLS)


def test_library_exports_every_declared_symbol():
    L = N.load()
    for s in declared_symbols():
        assert hasattr(L, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (sdcas_\w+)", out))
    assert declared_symbols() <= exported


def test_library_has_no_undefined_own_symbols():
    """a kernel declared with one signature and defined with another links as
    two overloads, the declared one undefined: the library then fails to load
    on the GPU box (round 6, k_solo_insert_idx) — catch it here"""
    out = subprocess.run(["nm", "-u", "-C", N.LIB_PATH], capture_output=True, text=True).stdout
    own = [ln for ln in out.splitlines() if "sdcas" in ln]
    assert own == [], own


def test_library_is_gfx950():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", N.LIB_PATH], capture_output=True,
                         text=True)
    blob = open(N.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_pure_helpers_without_gpu():
    import ctypes
    L = N.load()
    buf = ctypes.create_string_buffer(17)
    L.sdcas_key_to_hex(0x71E0A99173564931, buf)
    assert buf.value == b"71e0a99173564931"
    assert L.sdcas_cas_message_len(0) == 8
    assert L.sdcas_cas_message_len(102400) == 102408
    assert L.sdcas_cas_message_len(102401) == 57352
    d = bytes(range(32))
    out = ctypes.create_string_buffer(65)
    L.sdcas_digest_to_hex(d, out)
    assert out.value.decode() == d.hex()


def test_init_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from spacedrive_amd import Engine
    with pytest.raises(N.SdcasError):
        Engine()


def _kernel_stubs(path):
    out = subprocess.run(["nm", "-C", path], capture_output=True, text=True).stdout
    return sorted(set(re.findall(r"sdcas::__device_stub__(k_\w+(?:<[^>]*>)?)", out)))


def test_product_library_holds_only_product_kernels():
    """libsdcas.so carries only the product kernels — leaf 67 (default), 52
    and the small-batch kernels 84 (default since round 6, a quad of lanes
    per slot with four blocks in flight staged in LDS), 73 (a quad of lanes
    per slot) and 71, piece 19 (default: k_piece_l4 + k_piece_top) and 17, all bit-exact
    and GPU-tested — and no ablation or DIAGNOSTIC variant (those produce
    wrong digests and live only in libsdcas_ablate.so)"""
    stubs = _kernel_stubs(N.LIB_PATH)
    leaf = [s for s in stubs if s.startswith("k_leaf")]
    assert leaf == ["k_leaf_tree<128, 79, 1, 1, 2, 2, 0, 128u, 0, 0>",
                    "k_leaf_tree<512, 209, 1, 1, 2, 2, 0, 1024u, 0, 0>",
                    "k_leaf_tree<512, 279, 1, 1, 2, 2, 0, 1024u, 0, 0>",
                    "k_leaf_tree<512, 79, 1, 0, 2, 0, 0, 128u, 1, 0>",
                    "k_leaf_tree<512, 79, 1, 0, 2, 0, 0, 128u, 3, 0>"], leaf
    finish = [s for s in stubs if s.startswith("k_finish")]
    assert finish == ["k_finish_q<1024u>", "k_finish_q<128u>", "k_finish_t<1024u>", "k_finish_t<128u>"], finish
    assert not [s for s in stubs if "slim" in s or "quad" in s]
    pieces = [s for s in stubs if s.startswith("k_piece")]
    assert sorted(pieces) == ["k_piece_l4<259, 6>", "k_piece_top<259>", "k_piece_tree<259, 6, 1, 0, 10>"], pieces


def test_product_library_has_no_cub():
    """round 5: the last hipCUB / rocPRIM uses left the product library — the
    exact combine goes through the compact table (two emit passes), the
    gathered stays list is sorted by one workgroup or read back from a
    bitmap (dist_dedup.hip); only the ablation library's quad-layout scan
    keeps hipCUB"""
    out = subprocess.run(["nm", "-C", N.LIB_PATH], capture_output=True, text=True).stdout
    assert out and not re.search(r"hipcub|rocprim|\bcub::", out)


def test_ablation_build_is_separate():
    """the A/B library is a different file that no product module names"""
    assert N.ABLATION_LIB_PATH != N.LIB_PATH
    pkg = os.path.join(ROOT, "spacedrive_amd")
    for f in os.listdir(pkg):
        if f.endswith(".py") and f != "_native.py":
            assert "ablat" not in open(os.path.join(pkg, f)).read(), f


def test_quad_message_schedules_are_blake3s():
    """the quad compressions' message schedules in csrc/b3_device.h — the
    seven B3_QROUND lists of compress_quad and the table make_quad_words
    builds kQuadWord from (the small-batch kernel 84 reads each lane's 28
    words by it) — are BLAKE3's: round r applies the message permutation r
    times (Appendix A of SURVEY.md)"""
    src = open(os.path.join(ROOT, "spacedrive_amd", "csrc", "b3_device.h")).read()
    perm = [2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8]
    want, s = [], list(range(16))
    for _ in range(7):
        want.append(s)
        s = [s[p] for p in perm]
    qround = [[int(x) for x in m.split(",")]
              for m in re.findall(r"^\s*B3_QROUND\(([\d,\s]+)\);", src, re.M)]
    assert qround == want
    body = src[src.index("constexpr QuadWords make_quad_words()"):]
    body = body[:body.index("QuadWords t{}")]
    table = [[int(x) for x in row.split(",")] for row in re.findall(r"\{([\d,\s]+)\}", body)]
    assert table == want
