"""The Rust FFI a maintainer adds to sd-core against the C
header it binds (include/sdcas.h): every `extern "C"` function exists in the
header with the same parameter count, pointer parameters where the header has
pointers, the same return kind; `SdcasOptions` has the fields of
`sdcas_options` in order with the same widths; the constants agree. The
binding cannot be compiled here (no Rust toolchain), so this is what keeps the
text and the header from drifting apart."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rust_block():
    md = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"## 2\. Rust FFI module.*?```rust\n(.*?)```", md, flags=re.S)
    assert m, "INTEGRATION.md §2 has no rust block"
    return m.group(1)


def _header():
    src = open(os.path.join(ROOT, "include", "sdcas.h")).read()
    return re.sub(r"/\*.*?\*/", "", src, flags=re.S)


def _split_params(s):
    s = s.strip()
    if not s or s == "void":
        return []
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([<":
            depth += 1
        elif ch in ")]>":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def c_prototypes():
    protos = {}
    for ret, name, params in re.findall(r"([\w\s\*]+?)\b(sdcas_\w+)\s*\(([^;{]*?)\)\s*;", _header(), flags=re.S):
        protos[name] = (ret.strip(), _split_params(" ".join(params.split())))
    return protos


def rust_externs():
    blk = re.search(r'extern "C" \{(.*?)\n\}', _rust_block(), flags=re.S).group(1)
    fns = {}
    for name, params, ret in re.findall(r"fn (sdcas_\w+)\((.*?)\)\s*(?:->\s*([^;]+))?;", blk, flags=re.S):
        fns[name] = ([p.split(":", 1)[1].strip() for p in _split_params(" ".join(params.split()))],
                     (ret or "").strip())
    return fns


def _c_is_pointer(p):
    return "*" in p or "[" in p


def _rust_is_pointer(t):
    return t.startswith("*") or t == "SdcasProgressFn"  # a nullable C function pointer


def test_every_binding_is_declared_with_the_same_shape():
    C = c_prototypes()
    R = rust_externs()
    assert R, "no extern fns found"
    for name, (rparams, rret) in R.items():
        assert name in C, f"{name} bound in INTEGRATION.md but not declared in sdcas.h"
        cret, cparams = C[name]
        assert len(rparams) == len(cparams), (name, rparams, cparams)
        for rp, cp in zip(rparams, cparams):
            assert _rust_is_pointer(rp) == _c_is_pointer(cp) or "sdcas_progress_fn" in cp, (name, rp, cp)
            if "size_t" in cp and not _c_is_pointer(cp):
                assert rp == "usize", (name, rp, cp)
            if "uint64_t" in cp and not _c_is_pointer(cp):
                assert rp == "u64", (name, rp, cp)
        if cret == "void":
            assert rret == "", name
        elif cret == "int":
            assert rret == "c_int", name
        elif "char" in cret:
            assert rret == "*const c_char", name


def test_the_batch_entry_points_are_bound():
    """the three calls that replace sd-core's per-file hot path"""
    assert {"sdcas_init", "sdcas_destroy", "sdcas_cas_ids", "sdcas_checksums", "sdcas_dedup",
            "sdcas_set_progress", "sdcas_last_error"} <= set(rust_externs())


def test_options_struct_layout_agrees():
    rs = re.search(r"pub struct SdcasOptions \{(.*?)\}", _rust_block(), flags=re.S).group(1)
    rfields = re.findall(r"pub (\w+): ([^,]+),", rs)
    cs = re.search(r"typedef struct sdcas_options \{(.*?)\} sdcas_options;", _header(), flags=re.S).group(1)
    cfields = [(m[-1], " ".join(m[:-1])) for m in
               (re.findall(r"[\w\*]+", decl.replace("*", " * ")) for decl in cs.split(";") if decl.strip())]
    assert [f for f, _ in rfields] == [f for f, _ in cfields], (rfields, cfields)
    width = {"i32": "int32_t", "u32": "uint32_t", "u64": "uint64_t"}
    for (rf, rt), (cf, ct) in zip(rfields, cfields):
        rt = rt.strip()
        if rt in width:
            assert ct.split()[-1] == width[rt], (rf, rt, ct)
        else:
            assert "*" in ct or "fn" in ct, (rf, rt, ct)


def test_constants_agree():
    rust = _rust_block()
    hdr = _header()
    for name in ("SDCAS_E_CANCELLED", "SDCAS_STATUS_UNEXPECTED_EOF", "SDCAS_STATUS_CANCELLED", "SDCAS_OPT_DIRECT_IO"):
        rv = re.search(rf"pub const {name}: \w+ = (-?\d+);", rust)
        cv = re.search(rf"#define {name}\s+\(?(-?\d+)\)?", hdr)
        assert rv and cv, name
        assert int(rv.group(1)) == int(cv.group(1)), name
