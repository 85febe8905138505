"""CPU: the Julia drop-in (julia/RBL_hip.jl) against the C-ABI it binds (include/rbl_hip.h).

Julia is not installed here, so the binding cannot run; this test catches drift
between the two files instead.  Every `ccall((:rbl_..., librbl_hip), Ret, (T1, ...), a1, ...)`
in the .jl file must name a function the header declares, with the same number of arguments
and argument / return types that map onto the header's C types (Cint = int, Int64 = int64_t,
Ptr{Float64} = double*, Ptr{Cvoid} = an opaque handle, Ref{Ptr{Cvoid}} = a handle out-pointer,
...), and pass as many values as the type tuple names.  It also checks that the file defines
the reference's entry point `RBL_gpu(A::Union{SparseMatrixCSC{DOUBLE},Matrix{DOUBLE}}, k::Int64,
b::Int64)` (Julia/RBL_gpu.jl:205) and drives the loop with rbl_step_async / rbl_fetch.
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JL = os.path.join(ROOT, "julia", "RBL_hip.jl")
HDR = os.path.join(ROOT, "include", "rbl_hip.h")

# Julia type -> the set of C spellings it may bind (after whitespace normalisation)
JULIA_TO_C = {
    "Cint": {"int"},
    "Int64": {"int64_t"},
    "UInt64": {"uint64_t"},
    "Cdouble": {"double"},
    "Float64": {"double"},
    "Ptr{Cvoid}": {"rbl_ctx*", "const rbl_ctx*", "rbl_group*"},
    "Ref{Ptr{Cvoid}}": {"rbl_ctx**", "rbl_group**"},
    "Ptr{Float64}": {"double*", "const double*"},
    "Ptr{Int64}": {"int64_t*", "const int64_t*"},
    "Ptr{Int32}": {"int32_t*", "const int32_t*"},
    "Ptr{Cint}": {"int*", "const int*"},
    "Ptr{UInt8}": {"uint8_t*", "const uint8_t*", "uint8_t[128]", "const uint8_t[128]"},
    "Cstring": {"const char*", "char*"},
}


def _strip_c_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _ctype(decl):
    """'const double* S' -> 'const double*'; 'uint8_t unique_id[128]' -> 'uint8_t[128]'."""
    decl = " ".join(decl.split())
    arr = re.search(r"(\[\d+\])$", decl)
    if arr:
        decl = decl[: arr.start()]
    decl = decl.replace(" *", "*").replace("* ", "*")
    m = re.match(r"^(.*?[\s*])([A-Za-z_]\w*)$", decl)
    t = (m.group(1) if m else decl).strip()
    return t.replace(" *", "*") + (arr.group(1) if arr else "")


def header_prototypes():
    text = _strip_c_comments(open(HDR).read())
    protos = {}
    for m in re.finditer(r"\b(int|const char\s*\*)\s*(rbl_\w+)\s*\(([^;]*?)\)\s*;", text, re.S):
        ret = m.group(1).replace(" ", "")
        ret = "const char*" if "char" in ret else ret
        args = m.group(3).strip()
        params = [] if args in ("", "void") else [_ctype(a) for a in args.split(",")]
        protos[m.group(2)] = (ret, params)
    return protos


def _split_top(s):
    """Split s on commas not nested in (), {}, []."""
    out, depth, cur = [], 0, []
    for ch in s:
        if ch in "({[":
            depth += 1
        elif ch in ")}]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append("".join(cur).strip())
            cur = []
        else:
            cur.append(ch)
    if "".join(cur).strip():
        out.append("".join(cur).strip())
    return out


def julia_ccalls():
    src = open(JL).read()
    src = "\n".join(line.split("#", 1)[0] if not line.lstrip().startswith("#") else ""
                    for line in src.splitlines())
    calls = []
    for m in re.finditer(r"ccall\(", src):
        i, depth = m.end(), 1
        while depth:
            depth += {"(": 1, ")": -1}.get(src[i], 0)
            i += 1
        calls.append(_split_top(src[m.end(): i - 1]))
    return calls


def test_every_ccall_matches_the_header():
    protos = header_prototypes()
    assert "rbl_step_async" in protos and "rbl_create" in protos
    calls = julia_ccalls()
    assert len(calls) >= 20
    seen = set()
    for parts in calls:
        target, ret, types = parts[0], parts[1], parts[2]
        args = parts[3:]
        name = re.match(r"\(:(\w+),\s*librbl_hip\)", target).group(1)
        assert name in protos, f"{name}: not declared in rbl_hip.h"
        cret, cparams = protos[name]
        assert cret in JULIA_TO_C[ret], (name, ret, cret)
        jtypes = [] if types.strip() == "()" else _split_top(types.strip()[1:-1])
        assert len(jtypes) == len(cparams), (name, jtypes, cparams)
        assert len(args) == len(jtypes), (name, "values passed", args, jtypes)
        for jt, ct in zip(jtypes, cparams):
            assert ct in JULIA_TO_C[jt], (name, jt, ct)
        seen.add(name)
    for needed in ("rbl_create", "rbl_set_matrix_csc", "rbl_set_matrix_dense", "rbl_set_option",
                   "rbl_start", "rbl_step_async", "rbl_fetch", "rbl_ritz", "rbl_timers",
                   "rbl_stage_name", "rbl_num_stages", "rbl_synchronize", "rbl_free",
                   "rbl_last_error"):
        assert needed in seen, needed


def test_defines_reference_entry_point():
    src = open(JL).read()
    assert re.search(r"^function RBL_gpu\(A::Union\{SparseMatrixCSC\{DOUBLE\},Matrix\{DOUBLE\}\},"
                     r"\s*k::Int64,\s*b::Int64\)", src, re.M)
    # the stage labels of RBL_gpu.jl:152-219 come from the library (rbl_stage_name)
    import ctypes  # noqa: F401  (names only: no library load here)
    hdr = open(HDR).read()
    for label in ("AQ", "3-term", "qr", "part reorth", "loc reorth", "Ritz vectors"):
        assert f'"{label}"' in hdr
    assert "@timeit timer \"eig\"" in src


def test_header_parser_sees_every_exported_symbol():
    """The parser above is only as good as its coverage: every rbl_* symbol the header names in
    a prototype is parsed (compare with a plain scan of the names)."""
    text = _strip_c_comments(open(HDR).read())
    names = set(re.findall(r"\b(rbl_\w+)\s*\(", text))
    assert names == set(header_prototypes())
