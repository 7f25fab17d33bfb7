"""CPU test: the Rust binding (rust/sd-hip-cas/src/lib.rs) declares the C ABI exactly as
include/sd_hip_cas.h does — every function, with matching return and argument types.
Cargo is not available in this image, so this parse is the guard that keeps the crate a
faithful binding (and the ctypes table too: same argument counts)."""
import os
import re

from spacedrive_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

C_TO_RUST = {
    "void": "()", "int": "c_int", "size_t": "usize", "uint64_t": "u64", "uint32_t": "u32",
    "int32_t": "i32", "int64_t": "i64", "uint8_t": "u8", "char": "c_char", "sd_cas_ctx": "sd_cas_ctx",
    "sd_cas_multi": "sd_cas_multi",
}


def c_type_to_rust(t: str) -> str:
    """Normalised C parameter type -> the Rust FFI type it must be declared as."""
    t = " ".join(t.split())
    arr = re.match(r"^(const\s+)?(\w+)\s+\w+\[\d+\]$", t)  # `char out[17]` -> pointer
    if arr:
        return ("*const " if arr.group(1) else "*mut ") + rust_base(arr.group(2))
    t = re.sub(r"\s+\w+$", "", t) if not t.endswith("*") else t  # drop the parameter name
    stars = []
    # parse from the right: each '*' optionally preceded by 'const' (that qualifies the
    # pointer itself, which Rust does not express) — the pointee's const goes to its '*'
    m = re.match(r"^(const\s+)?(\w+)\s*(.*)$", t)
    base_const, base, rest = bool(m.group(1)), m.group(2), m.group(3)
    tokens = re.findall(r"\*|const", rest)
    # pointee constness for each level: level 1 = base_const; level k+1 = 'const' before '*' k+1
    levels = []
    pending_const = base_const
    for tok in tokens:
        if tok == "const":
            pending_const = True
        else:
            levels.append(pending_const)
            pending_const = False
    out = rust_base(base)
    for const in levels:
        out = ("*const " if const else "*mut ") + out
        stars.append(const)
    return out


def rust_base(b: str) -> str:
    return "c_void" if b == "void" else C_TO_RUST[b]


def header_prototypes():
    text = open(os.path.join(ROOT, "include", "sd_hip_cas.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = "\n".join(ln for ln in text.splitlines() if not ln.lstrip().startswith("#"))
    protos = {}
    for ret, name, args in re.findall(r"([A-Za-z_][\w\s\*]*?)\b(sd_cas_\w+)\s*\(([^)]*)\)\s*;", text):
        ret = " ".join(ret.split())
        params = [] if args.strip() in ("", "void") else [a.strip() for a in args.split(",")]
        protos[name] = (c_ret_to_rust(ret), [c_type_to_rust(p) for p in params])
    return protos


def c_ret_to_rust(ret: str) -> str:
    if ret == "void":
        return "()"
    return c_type_to_rust(ret + " x") if not ret.endswith("*") else c_type_to_rust(ret)


def rust_prototypes():
    text = open(os.path.join(ROOT, "rust", "sd-hip-cas", "src", "lib.rs")).read()
    block = text[text.index('extern "C" {'):]
    block = block[:block.index("\n}\n")]
    protos = {}
    for name, args, ret in re.findall(r"fn\s+(sd_cas_\w+)\s*\(([^)]*)\)\s*(?:->\s*([^;]+))?;", block, flags=re.S):
        params = [a.strip() for a in args.split(",") if a.strip()]
        types = [" ".join(p.split(":", 1)[1].split()) for p in params]
        protos[name] = ((ret or "()").strip(), types)
    return protos


def test_rust_extern_block_matches_header():
    h = header_prototypes()
    r = rust_prototypes()
    assert len(h) > 40
    assert sorted(h) == sorted(r), (set(h) ^ set(r))
    bad = {n: (h[n], r[n]) for n in h if h[n] != r[n]}
    assert not bad, bad


def test_ctypes_table_arity_matches_header():
    h = header_prototypes()
    table = {n: args for n, _, args in _native.SIGNATURES}
    assert sorted(table) == sorted(h)
    bad = {n: (len(table[n]), len(h[n][1])) for n in h if len(table[n]) != len(h[n][1])}
    assert not bad, bad


def test_type_mapping_examples():
    assert c_type_to_rust("const uint8_t* const* bufs") == "*const *const u8"
    assert c_type_to_rust("uint64_t* const* d_rep") == "*const *mut u64"
    assert c_type_to_rust("sd_cas_ctx** out") == "*mut *mut sd_cas_ctx"
    assert c_type_to_rust("char out[17]") == "*mut c_char"
    assert c_type_to_rust("const void* h") == "*const c_void"
    assert c_type_to_rust("size_t n") == "usize"


def test_rust_constants_match_header():
    """Every `pub const SD_CAS_*` of the crate equals the header's #define of that name."""
    hdr = open(os.path.join(ROOT, "include", "sd_hip_cas.h")).read()
    rs = open(os.path.join(ROOT, "rust", "sd-hip-cas", "src", "lib.rs")).read()

    def cint(v: str) -> int:
        return int(v.replace("_", "").rstrip("uUlL"), 0)
    defines = {m.group(1): m.group(2) for m in re.finditer(r"#define\s+(SD_CAS_\w+)\s+(\S+)", hdr)}
    consts = re.findall(r"pub const (SD_CAS_\w+):\s*\w+\s*=\s*([0-9xXa-fA-F_]+);", rs)
    assert len(consts) >= 8
    for name, val in consts:
        assert name in defines, name
        assert cint(defines[name]) == cint(val), (name, defines[name], val)
