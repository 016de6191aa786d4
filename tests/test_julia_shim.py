"""The Julia drop-in (julia/TCIGPU.jl) against the C ABI it binds (include/tci_hip.h).

Julia is not installed in this image, so the shim is UNVERIFIED AT RUNTIME. What can be checked
mechanically is checked here (CPU suite): every `ccall((:tci_*, libtci), Ret, (types...), args...)`
names a symbol the header declares (and the built library exports, when it is there), passes as
many arguments as its type tuple lists, and the tuple matches the C prototype parameter by
parameter -- pointer-ness, and for scalars and typed pointers the element width and kind
(Int32 <-> int32_t / int, Int64 <-> int64_t, Float64 <-> double, ...). The host callback's
@cfunction signature is checked against `tci_host_fn` the same way. Reference of the plugin
interface: /root/reference/src/cachedtensortrain.jl:31, docs/src/index.md:174-243.
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "julia", "TCIGPU.jl")
HEADER = os.path.join(ROOT, "include", "tci_hip.h")

# C scalar / pointee types -> (kind, bytes)
C_SCALARS = {"int": ("i", 4), "int32_t": ("i", 4), "int64_t": ("i", 8), "uint64_t": ("u", 8),
             "double": ("f", 8), "float": ("f", 4), "char": ("i", 1), "unsigned char": ("u", 1),
             "uint8_t": ("u", 1), "void": ("v", 0)}
# Julia types -> (kind, bytes)
JL_SCALARS = {"Cint": ("i", 4), "Int32": ("i", 4), "Int64": ("i", 8), "UInt64": ("u", 8),
              "Float64": ("f", 8), "Float32": ("f", 4), "UInt8": ("u", 1), "Cvoid": ("v", 0),
              "ComplexF64": ("f", 8)}  # ComplexF64 arrays are interleaved doubles (tci_*_c128_*)
OPAQUE = {"tci_ctx", "tci_func", "tci_comm", "tci_cache", "tci_tci2"}
FNPTR = {"tci_exchange_fn", "tci_host_fn"}


def _split_top(s):
    """split s at top-level commas (parentheses / braces / brackets balanced)"""
    out, depth, cur = [], 0, []
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append("".join(cur).strip())
            cur = []
        else:
            cur.append(ch)
    if "".join(cur).strip():
        out.append("".join(cur).strip())
    return out


def _balanced(s, i):
    """index just past the parenthesis that closes the one at s[i]"""
    depth = 0
    for j in range(i, len(s)):
        if s[j] == "(":
            depth += 1
        elif s[j] == ")":
            depth -= 1
            if depth == 0:
                return j + 1
    raise ValueError("unbalanced")


def _c_param(p):
    """C parameter declaration -> ('ptr', pointee kind/width or None) or ('val', kind, width)"""
    p = re.sub(r"\bconst\b", " ", p)
    p = " ".join(p.split())
    nstars = p.count("*")
    base = p.replace("*", " ").split()
    # drop the parameter name (the last word, when there are two or more)
    words = base[:-1] if len(base) > 1 else base
    t = " ".join(words)
    if t in FNPTR:
        return ("ptr", None)
    if nstars == 0:
        assert t in C_SCALARS, t
        return ("val",) + C_SCALARS[t]
    if nstars > 1 or t in OPAQUE or t == "void":
        return ("ptr", None)  # handles, out-handles, void*: any pointer
    return ("ptr", C_SCALARS[t])


def _jl_type(t):
    t = t.strip()
    m = re.fullmatch(r"(Ptr|Ref)\{(.+)\}", t)
    if m:
        inner = m.group(2).strip()
        if inner.startswith("Ptr{") or inner in ("Cvoid", "Any"):
            return ("ptr", None)
        return ("ptr", JL_SCALARS[inner])
    if t in ("Any", "Cstring"):
        return ("ptr", None)
    return ("val",) + JL_SCALARS[t]


def header_prototypes():
    s = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    protos = {}
    for rt, name, args in re.findall(r"\b((?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?)\s*(tci_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;",
                                     s, flags=re.S):
        a = " ".join(args.split())
        params = [] if a in ("", "void") else [_c_param(x) for x in _split_top(a)]
        protos[name] = (rt.strip(), params)
    for name, args in re.findall(r"typedef\s+int\s*\(\*\s*(tci_[a-z_]+)\)\s*\(([^;]*?)\)\s*;", s, flags=re.S):
        protos[name] = ("int", [_c_param(x) for x in _split_top(" ".join(args.split()))])
    return protos


def shim_ccalls():
    src = open(SHIM).read()
    src = re.sub(r"#.*", "", src)  # comments
    calls = []
    for mt in re.finditer(r"\bccall\(", src):
        i = mt.end() - 1
        body = src[i + 1:_balanced(src, i) - 1]
        parts = _split_top(body)
        m = re.fullmatch(r"\(\s*:(tci_[a-z0-9_]+)\s*,\s*libtci\s*\)", parts[0])
        assert m, parts[0]
        tup = parts[2].strip()
        assert tup.startswith("(") and tup.endswith(")"), tup
        types = [t for t in _split_top(tup[1:-1]) if t]
        calls.append((m.group(1), parts[1].strip(), types, parts[3:]))
    cfuns = []
    for mt in re.finditer(r"@cfunction\(", src):
        i = mt.end() - 1
        parts = _split_top(src[i + 1:_balanced(src, i) - 1])
        tup = parts[2].strip()
        cfuns.append((parts[0].strip(), parts[1].strip(), [t for t in _split_top(tup[1:-1]) if t]))
    return calls, cfuns


def test_shim_exists_and_is_a_module():
    src = open(SHIM).read()
    assert src.count("module TCIGPU") == 1 and src.rstrip().endswith("end # module")
    assert "unverified at runtime" in src
    # the reference's plugin points the shim specialises (tensorci2.jl:825, :599)
    assert "function TCI.updatepivots!(" in src and "function TCI.setsitetensor!(" in src
    assert "<: TCI.BatchEvaluator{Float64}" in src


def test_every_ccall_matches_the_header():
    protos = header_prototypes()
    calls, _ = shim_ccalls()
    assert len(calls) >= 30, len(calls)
    for name, ret, types, args in calls:
        assert name in protos, f"{name}: not declared in include/tci_hip.h"
        cret, params = protos[name]
        want_ret = {"int": "Cint", "const char*": "Cstring", "void*": "Ptr{Cvoid}"}[cret.replace(" *", "*")]
        assert ret == want_ret, (name, ret, cret)
        assert len(types) == len(params), (name, "type tuple", len(types), "C params", len(params))
        assert len(args) == len(types), (name, "arguments", len(args), "types", len(types))
        for i, (jt, cp) in enumerate(zip(types, params)):
            jp = _jl_type(jt)
            assert jp[0] == cp[0], (name, i, jt, cp)
            if jp[0] == "val":
                assert jp[1:] == cp[1:] or (jp[1] in "iu" and cp[1] in "iu" and jp[2] == cp[2]), (name, i, jt, cp)
            elif jp[1] is not None and cp[1] is not None:
                assert jp[1][1] == cp[1][1], (name, i, jt, cp)  # pointee width


def test_host_callback_matches_tci_host_fn():
    protos = header_prototypes()
    _, cfuns = shim_ccalls()
    assert cfuns, "the host batch callback"
    for fn, ret, types in cfuns:
        assert ret == "Cint"
        params = protos["tci_host_fn"][1]
        assert len(types) == len(params), (fn, len(types), len(params))
        for i, (jt, cp) in enumerate(zip(types, params)):
            jp = _jl_type(jt)
            assert jp[0] == cp[0] and (jp[0] == "ptr" or jp[1:] == cp[1:]), (fn, i, jt, cp)


def test_bound_symbols_are_exported():
    """every symbol the shim binds is exported by the built library (skipped when not built)"""
    lib = os.path.join(ROOT, "tensorcrossinterpolation.jl_amd", "lib", "libtci_hip.so")
    if not os.path.exists(lib):
        pytest.skip("libtci_hip.so not built")
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    calls, _ = shim_ccalls()
    missing = sorted({c[0] for c in calls} - exported)
    assert not missing, missing


def test_coverage_of_the_hot_path_entries():
    """the entries a TCI2 sweep goes through are all bound"""
    names = {c[0] for c in shim_ccalls()[0]}
    for need in ("tci_ctx_create", "tci_func_create", "tci_func_create_host", "tci_batcheval_h",
                 "tci_update_pivots_h", "tci_sitetensor_h", "tci_rrlu_h", "tci_rrlu_c128_h", "tci_luci_h",
                 "tci_tci2_sweep2site", "tci_tci2_sweep1site", "tci_rrlu_sharded_d", "tci_comm_create",
                 "tci_batcheval_da", "tci_rrlu_copy_d", "tci_schur_update_d"):
        assert need in names, need
