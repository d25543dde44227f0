"""CPU: rust/maxio-ec-sys/src/lib.rs (the extern "C" block MaxIO would bind,
INTEGRATION.md §2) stays mechanically consistent with include/maxio_ec.h:
every declared function appears on both sides with the same arity and the
same argument / return widths (int = c_int, size_t = usize, pointers as
pointers with matching const-ness of the pointee), every #[repr(C)] struct
has the C struct's fields in order with the same types, and every MXEC_*
constant has the same value.  No Rust toolchain here, so this parse is the
check; it fails as soon as either side drifts.  Replaces the reference call
sites filesystem.rs:1062, :1084 and chunk_reader.rs:157."""
from __future__ import annotations

import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "maxio_ec.h")
RUST = os.path.join(ROOT, "rust", "maxio-ec-sys", "src", "lib.rs")

C_SCALAR = {"int": "i32", "float": "f32", "int32_t": "i32", "uint32_t": "u32", "uint64_t": "u64", "int64_t": "i64",
            "size_t": "usize", "uint8_t": "u8", "char": "i8", "void": "void"}
R_SCALAR = {"c_int": "i32", "i32": "i32", "u32": "u32", "u64": "u64", "i64": "i64", "usize": "usize",
            "u8": "u8", "c_char": "i8", "c_void": "void"}
STRUCTS = {"mxec_ctx": "MxecCtx", "mxec_reader": "MxecReader", "mxec_ticket": "MxecTicket",
           "mxec_chunk_info": "MxecChunkInfo", "mxec_object": "MxecObject", "mxec_body_sums": "MxecBodySums",
           "mxec_frames_job": "MxecFramesJob", "mxec_multipart_part": "MxecMultipartPart"}


# ---- C side -----------------------------------------------------------------

def _c_clean(text: str) -> str:
    t = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return re.sub(r"//[^\n]*", "", t)


def _c_type(ty: str) -> str:
    """'const uint8_t* const*' -> 'ptr(const ptr(const u8))' (innermost pointee last)."""
    toks = ty.replace("*", " * ").split()
    i, base_const = 0, False
    if toks[i] == "const":
        base_const, i = True, 1
    base = toks[i]
    i += 1
    ptr_consts = []
    while i < len(toks):
        if toks[i] == "*":
            ptr_consts.append(False)
        elif toks[i] == "const":
            ptr_consts[-1] = True
        else:
            raise AssertionError(f"unparsed C type {ty!r}")
        i += 1
    r = STRUCTS.get(base) or C_SCALAR[base]
    consts = [base_const] + ptr_consts[:-1]
    for c in consts[: len(ptr_consts)]:
        r = f"ptr({'const ' if c else ''}{r})"
    return r


def _c_param(p: str):
    p = " ".join(p.split())
    if p in ("void", ""):
        return None
    m = re.match(r"(const\s+)?(\w+)\s*\(\*\s*(\w+)\)\[(\d+)\]$", p)
    if m:
        c, base, _, n = m.groups()
        return f"ptr({'const ' if c else ''}[{C_SCALAR[base]};{n}])"
    m = re.match(r"(const\s+)?(\w+)\s+(\w+)\[(\d+)\]$", p)
    if m:  # array parameter decays to a pointer
        c, base, _, _n = m.groups()
        return f"ptr({'const ' if c else ''}{C_SCALAR[base]})"
    m = re.match(r"(.*?)(\w+)$", p)
    return _c_type(m.group(1).strip())


def c_functions() -> dict:
    t = _c_clean(open(HEADER).read())
    t = "\n".join(l for l in t.splitlines() if not l.strip().startswith("#"))
    t = re.sub(r"typedef\s+struct\s+\w+\s*\{.*?\}\s*\w+\s*;", "", t, flags=re.S)
    t = re.sub(r"typedef\s+struct\s+\w+\s+\w+\s*;", "", t)
    t = t.replace('extern "C" {', "").replace("}", "")
    out = {}
    for ret, name, params in re.findall(r"([A-Za-z_][\w\s\*]*?)\b(mxec_\w+)\s*\(([^;{]*?)\)\s*;", t, flags=re.S):
        ret = " ".join(ret.split())
        out[name] = ([q for q in (_c_param(x) for x in params.split(",")) if q], _c_type(ret))
    return out


def c_structs() -> dict:
    t = _c_clean(open(HEADER).read())
    out = {}
    for body, name in re.findall(r"typedef\s+struct\s+\w+\s*\{(.*?)\}\s*(\w+)\s*;", t, flags=re.S):
        fields = []
        for decl in body.split(";"):
            decl = " ".join(decl.split())
            if not decl:
                continue
            m = re.match(r"(.*?)(\w+)\s*(?:\[(\d+)\])?$", decl)
            ty, fname, n = m.group(1).strip(), m.group(2), m.group(3)
            fields.append((fname, f"[{C_SCALAR[ty]};{n}]" if n else _c_type(ty)))
        out[STRUCTS[name]] = fields
    return out


def c_constants() -> dict:
    out = {}
    for name, val in re.findall(r"#define\s+(MXEC_\w+)\s+\(?(-?(?:0x)?[0-9a-fA-F]+)u?\)?", open(HEADER).read()):
        out[name] = int(val, 0)
    return out


# ---- Rust side --------------------------------------------------------------

def _r_type(ty: str) -> str:
    ty = ty.strip()
    if ty.startswith("*const ") or ty.startswith("*mut "):
        const = ty.startswith("*const ")
        inner = _r_type(ty.split(" ", 1)[1])
        return f"ptr({'const ' if const else ''}{inner})"
    m = re.match(r"\[(\w+);\s*(\d+)\]$", ty)
    if m:
        return f"[{R_SCALAR[m.group(1)]};{m.group(2)}]"
    return R_SCALAR.get(ty) or ty


def rust_functions() -> dict:
    src = open(RUST).read()
    block = re.search(r'extern "C" \{(.*?)\n\}', src, flags=re.S).group(1)
    out = {}
    for name, params, ret in re.findall(r"pub fn (mxec_\w+)\((.*?)\)\s*(?:->\s*([^;]+))?;", block, flags=re.S):
        ps = [p.split(":", 1)[1] for p in (x.strip() for x in params.split(",")) if p]
        out[name] = ([_r_type(p) for p in ps], _r_type(ret) if ret else "void")
    return out


def rust_structs() -> dict:
    src = open(RUST).read()
    out = {}
    for name, body in re.findall(r"#\[repr\(C\)\][^\n]*\n(?:#\[[^\n]*\]\n)*pub struct (\w+) \{(.*?)\}", src, flags=re.S):
        fields = []
        for line in body.split(","):
            line = line.strip()
            if not line or line.startswith("_p"):
                continue
            fname, ty = line.replace("pub ", "", 1).split(":", 1)
            fields.append((fname.strip(), _r_type(ty)))
        out[name] = fields
    return out


def rust_constants() -> dict:
    src = open(RUST).read()
    return {n: int(v, 0) for n, v in re.findall(r"pub const (MXEC_\w+): \w+ = (-?(?:0x)?[0-9a-fA-F]+);", src)}


# ---- tests ------------------------------------------------------------------

def test_every_header_function_bound_with_same_signature():
    c, r = c_functions(), rust_functions()
    assert len(c) >= 50
    assert sorted(c) == sorted(r), (sorted(set(c) - set(r)), sorted(set(r) - set(c)))
    for name, (cp, cr) in c.items():
        rp, rr = r[name]
        assert len(cp) == len(rp), f"{name}: arity C {len(cp)} vs Rust {len(rp)}"
        for i, (a, b) in enumerate(zip(cp, rp)):
            assert a == b, f"{name} argument {i}: C {a} vs Rust {b}"
        assert cr == rr, f"{name} return: C {cr} vs Rust {rr}"


def test_structs_match_field_by_field():
    c, r = c_structs(), rust_structs()
    for name, fields in c.items():
        assert name in r, name
        assert fields == r[name], f"{name}: C {fields} vs Rust {r[name]}"
    for opaque in ("MxecCtx", "MxecReader", "MxecTicket"):
        assert r[opaque] == [], opaque


def test_constants_match():
    c, r = c_constants(), rust_constants()
    assert sorted(c) == sorted(r), (sorted(set(c) - set(r)), sorted(set(r) - set(c)))
    for k, v in c.items():
        assert r[k] == v, k


def test_parser_catches_drift(tmp_path, monkeypatch):
    """The check is not vacuous: a Rust block with a narrowed argument or a
    missing symbol fails it."""
    import tests.test_rust_ffi as me  # noqa: F401  (same module, patched paths below)

    src = open(RUST).read()
    bad = tmp_path / "lib.rs"
    bad.write_text(src.replace("shard_size: usize, data: *const *const u8", "shard_size: u32, data: *const *const u8", 1))
    monkeypatch.setattr(me, "RUST", str(bad))
    c, r = me.c_functions(), me.rust_functions()
    assert c["mxec_encode"] != r["mxec_encode"]
    bad.write_text(src.replace("    pub fn mxec_ticket_poll(t: *mut MxecTicket) -> c_int;\n", ""))
    assert "mxec_ticket_poll" not in me.rust_functions()
