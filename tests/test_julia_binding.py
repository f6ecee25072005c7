"""Static checks of the Julia binding (julia/MPGPU.jl) against include/mpgpu.h.

Julia is not installed here, so the binding cannot run; these tests parse it instead:
  * every `struct` that mirrors a C parameter struct has the C fields, in order, with matching types
    (Int32 <-> int32_t, Float64 <-> double, UInt64 <-> uint64_t, NTuple{n,Float64} <-> double[n]);
  * every `ccall((:mp_*, libmpgpu), R, (T...), ...)` names a declared function and its return type and
    argument type tuple match the C prototype class by class (pointer / int32 / int64 / size_t / double),
    with the right struct behind each `Ref{...}`;
  * every declared entry point has at least one ccall (the INTEGRATION.md stubs).
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "mpgpu.h")
JL = os.path.join(ROOT, "julia", "MPGPU.jl")

JL_STRUCT = {"MppiParams": "mp_mppi_params", "MppiLoopParams": "mp_mppi_loop_params",
             "IlqrParams": "mp_ilqr_params", "HaParams": "mp_ha_params", "TrackParams": "mp_track_params"}


def header_text():
    return re.sub(r"/\*.*?\*/", "", open(HDR).read(), flags=re.S)


def c_structs():
    """{name: [(field, ctype, count)]} for every typedef struct of the header."""
    out = {}
    for body, name in re.findall(r"typedef struct \w+ \{(.*?)\} (\w+);", header_text(), flags=re.S):
        fields = []
        for decl in body.split(";"):
            decl = " ".join(decl.split())
            if not decl:
                continue
            m = re.match(r"(u?int\d+_t|double|int) (.*)", decl)
            assert m, decl
            for part in m.group(2).split(","):
                part = part.strip()
                a = re.match(r"(\w+)(?:\[(\w+)\])?$", part)
                n = a.group(2)
                cnt = 1 if n is None else {"MP_NX": 7, "MP_NU": 2}.get(n, None) or int(n)
                fields.append((a.group(1), m.group(1), cnt))
        out[name] = fields
    return out


def jl_structs():
    src = open(JL).read()
    out = {}
    for name, body in re.findall(r"^struct (\w+)\s*(?:#[^\n]*)?\n(.*?)^end", src, flags=re.S | re.M):
        fields = []
        for line in body.splitlines():
            line = line.split("#")[0].strip()
            if not line:
                continue
            m = re.match(r"(\w+)::(.+)$", line)
            assert m, line
            fields.append((m.group(1), m.group(2).strip()))
        out[name] = fields
    return out


def jl_type_matches(jt, ctype, cnt):
    scalar = {"int32_t": "Int32", "int": "Int32", "double": "Float64", "uint64_t": "UInt64", "int64_t": "Int64"}[ctype]
    if cnt == 1:
        return jt == scalar
    return jt == f"NTuple{{{cnt},{scalar}}}"


def test_julia_structs_match_c_layout():
    cs, js = c_structs(), jl_structs()
    for jname, cname in JL_STRUCT.items():
        assert jname in js, jname
        cf, jf = cs[cname], js[jname]
        assert [f for f, _, _ in cf] == [f for f, _ in jf], (jname, [f for f, _, _ in cf], [f for f, _ in jf])
        for (f, ct, n), (_, jt) in zip(cf, jf):
            assert jl_type_matches(jt, ct, n), (jname, f, ct, n, jt)


def c_prototypes():
    """{fn: (ret_class, [arg classes], [struct or None per arg])}."""
    out = {}
    for ret, name, args in re.findall(r"\n\s*(int|const char\s*\*|void\s*\*)\s*(mp_\w+)\((.*?)\);", header_text(),
                                      flags=re.S):
        cls, structs = [], []
        a = " ".join(args.split())
        parts = [] if a in ("", "void") else [x.strip() for x in a.split(",")]
        for x in parts:
            sm = re.search(r"\b(mp_\w+_params)\b", x)
            structs.append(sm.group(1) if sm else None)
            if "*" in x:
                cls.append("ptr")
            elif re.match(r"(const )?(int32_t|int) ", x):
                cls.append("i32")
            elif re.match(r"(const )?int64_t ", x):
                cls.append("i64")
            elif re.match(r"(const )?size_t ", x):
                cls.append("size")
            elif re.match(r"(const )?double ", x):
                cls.append("f64")
            else:
                raise AssertionError(x)
        out[name] = ("int" if ret == "int" else "ptr", cls, structs)
    return out


def _balanced(src, i):
    """Text of the parenthesised group starting at src[i] == '('."""
    assert src[i] == "("
    d = 0
    for j in range(i, len(src)):
        d += {"(": 1, ")": -1}.get(src[j], 0)
        if d == 0:
            return src[i + 1:j]
    raise AssertionError("unbalanced")


def _split_top(s):
    out, d, cur = [], 0, ""
    for ch in s:
        if ch in "({[":
            d += 1
        elif ch in ")}]":
            d -= 1
        if ch == "," and d == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def jl_ccalls():
    src = open(JL).read()
    calls = []
    for m in re.finditer(r"ccall\(\(:(mp_\w+), libmpgpu\),\s*(\w+),\s*", src):
        i = m.end()
        types = _split_top(_balanced(src, i))
        calls.append((m.group(1), m.group(2), types))
    return calls


def jl_class(t):
    if t.startswith(("Ptr{", "Ref{")) or t == "Cstring":
        return "ptr"
    return {"Int32": "i32", "Cint": "i32", "Int64": "i64", "Csize_t": "size", "Float64": "f64", "Cdouble": "f64"}[t]


def test_julia_ccalls_match_prototypes():
    protos = c_prototypes()
    calls = jl_ccalls()
    assert len(calls) >= 20
    rev = {v: k for k, v in JL_STRUCT.items()}
    for name, ret, types in calls:
        assert name in protos, f"{name} is not declared in mpgpu.h"
        pret, pcls, pstructs = protos[name]
        assert {"Cint": "int", "Cstring": "ptr", "Ptr": "ptr"}.get(ret, ret) == pret, (name, ret)
        assert [jl_class(t) for t in types] == pcls, (name, types, pcls)
        for t, st in zip(types, pstructs):
            if st is not None:
                assert t == f"Ref{{{rev[st]}}}", (name, t, st)


def test_every_entry_point_has_a_julia_stub():
    protos = c_prototypes()
    bound = {n for n, _, _ in jl_ccalls()}
    # diagnostics and timing hooks are for the Python test/bench harness, not the planner surface
    harness_only = {"mp_math_eval", "mp_ctx_kernel_timing", "mp_ctx_kernel_ms", "mp_ctx_stream", "mp_ctx_trim",
                    "mp_ctx_set_workspace_limit", "mp_ctx_synchronize", "mp_mppi_plan_dev", "mp_ilqr_backward_dev",
                    "mp_ilqr_forward_dev", "mp_ilqr_solve_dev", "mp_version", "mp_comm_allgather_dev"}
    missing = sorted(set(protos) - bound - harness_only)
    assert not missing, missing
