"""The Julia binding (symbolicregression.jl_amd/julia/SRHip.jl) against the C ABI.

Julia is not installed in this image, so SRHip.jl cannot run here. This CPU
test checks what can be checked statically: every `ccall((:srhip_*, libsrhip),
R, (A...), args...)` names a function that include/srhip.h declares and
libsrhip.so exports, passes as many arguments as the prototype has, and uses
Julia types that match the C parameter types (Int32 <-> int32_t, Int64 <->
int64_t, Ptr/Ref/Cstring <-> pointers); the constants it defines equal the
header's; every SRHIP_LOSS_* code is reachable from a loss type
(LossFunctions.jl's distance losses, src/Options.jl:429-431)."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
JL = ROOT / "symbolicregression.jl_amd" / "julia" / "SRHip.jl"
HDR = ROOT / "include" / "srhip.h"
LIB = ROOT / "symbolicregression.jl_amd" / "lib" / "libsrhip.so"


def _split_top(s):
    """Split on commas at nesting depth 0 (braces, parentheses, brackets)."""
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "({[":
            depth += 1
        elif ch in ")}]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def _matching(s, i):
    """Index of the parenthesis closing the one at s[i]."""
    depth = 0
    for j in range(i, len(s)):
        if s[j] == "(":
            depth += 1
        elif s[j] == ")":
            depth -= 1
            if depth == 0:
                return j
    raise ValueError("unbalanced")


def julia_ccalls():
    src = "\n".join(ln.split("#")[0] for ln in JL.read_text().splitlines())  # drop comments
    calls = []
    for m in re.finditer(r"ccall\(", src):
        start = m.end() - 1
        body = src[start + 1:_matching(src, start)]
        parts = _split_top(body)
        sym = re.match(r"\(:(\w+),\s*libsrhip\)", parts[0])
        assert sym, f"ccall without (:symbol, libsrhip): {parts[0]}"
        ret = parts[1]
        tup = parts[2]
        assert tup.startswith("(") and tup.endswith(")"), tup
        argtypes = _split_top(tup[1:-1])
        calls.append((sym.group(1), ret, argtypes, parts[3:]))
    return calls


def header_prototypes():
    txt = re.sub(r"/\*.*?\*/", "", HDR.read_text(), flags=re.S)
    protos = {}
    for m in re.finditer(r"^([\w\s\*]+?)\s*\b(srhip_\w+)\s*\(([^)]*)\)\s*;", txt, re.M):
        ret, name, params = m.group(1).strip(), m.group(2), m.group(3).strip()
        plist = [] if params in ("", "void") else [p.strip() for p in params.split(",")]
        protos[name] = (ret, plist)
    return protos


def _c_kind(param):
    p = re.sub(r"\b(const|struct)\b", "", param).strip()
    if "*" in p:
        return "ptr"
    ty = p.split()[0]
    return {"int32_t": "i32", "int64_t": "i64", "double": "f64", "uint8_t": "u8", "uint32_t": "u32"}[ty]


def _jl_kind(t):
    t = t.strip()
    if t.startswith(("Ptr{", "Ref{")) or t == "Cstring":
        return "ptr"
    return {"Int32": "i32", "Int64": "i64", "Float64": "f64", "UInt8": "u8", "UInt32": "u32", "Cint": "i32"}[t]


def test_every_ccall_matches_the_header():
    protos = header_prototypes()
    calls = julia_ccalls()
    assert len(calls) >= 12
    seen = set()
    for name, ret, argtypes, args in calls:
        assert name in protos, f"{name} is not declared in include/srhip.h"
        cret, cparams = protos[name]
        seen.add(name)
        assert len(argtypes) == len(cparams), f"{name}: {len(argtypes)} Julia argument types, {len(cparams)} in C"
        assert len(args) == len(argtypes), f"{name}: {len(args)} arguments for {len(argtypes)} types"
        for jt, cp in zip(argtypes, cparams):
            assert _jl_kind(jt) == _c_kind(cp), f"{name}: Julia {jt} vs C {cp}"
        if "char" in cret:
            assert ret == "Cstring", name
        else:
            assert ret == "Int32" and cret == "int32_t", f"{name}: returns {ret} / {cret}"
    # the entry points the shim of INTEGRATION.md §3 needs are all bound
    for need in ("srhip_eval_loss_batch_ctx", "srhip_eval_tree_array", "srhip_eval_grad_tree_array",
                 "srhip_eval_loss_grad", "srhip_program_create_ex", "srhip_program_set_constants",
                 "srhip_dataset_create", "srhip_op_lookup", "srhip_open", "srhip_device_count"):
        assert need in seen, need


def test_ccall_symbols_are_exported():
    if not LIB.exists():
        pytest.skip("libsrhip.so not built")
    lib = ctypes.CDLL(str(LIB))
    for name, *_ in julia_ccalls():
        assert hasattr(lib, name), f"libsrhip.so does not export {name}"


def test_constants_and_loss_table_match_the_header():
    hdr = HDR.read_text()
    src = JL.read_text()
    defs = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define SRHIP_(\w+)\s+\(?(-?\d+)\)?", hdr)}
    # scalar constants: const NAME = Int32(v)
    for name, val in re.findall(r"const (SRHIP_\w+) = Int32\((-?\d+)\)", src):
        assert defs[name[len("SRHIP_"):]] == int(val), name
    # tuple-assigned LOSS_* constants
    losses = {}
    for lhs, rhs in re.findall(r"const ((?:LOSS_\w+,?\s*)+)=\s*((?:Int32\(\d+\),?\s*)+)", src):
        names = [x.strip() for x in lhs.split(",") if x.strip()]
        vals = [int(v) for v in re.findall(r"Int32\((\d+)\)", rhs)]
        losses.update(zip(names, vals))
    hdr_losses = {k: v for k, v in defs.items() if k.startswith("LOSS_")}
    assert losses == hdr_losses
    # every loss code has a loss_code method
    mapped = set(re.findall(r"loss_code\([^)]*\)(?: where \{P\})? = \((LOSS_\w+),", src))
    for a, b in re.findall(r"loss_code\([^)]*\)(?: where \{P\})? = \(P isa Integer \? (LOSS_\w+) : (LOSS_\w+),", src):
        mapped |= {a, b}  # LPDistLoss{P}: Int P → LPINT, else LP
    assert mapped == set(hdr_losses), set(hdr_losses) ^ mapped
    # node kinds and the X layout
    kinds = re.search(r"const NODE_CONST, NODE_FEATURE, NODE_UNARY, NODE_BINARY = (.*)", src).group(1)
    assert [int(v) for v in re.findall(r"UInt8\((\d)\)", kinds)] == [
        defs["NODE_CONST"], defs["NODE_FEATURE"], defs["NODE_UNARY"], defs["NODE_BINARY"]]
    assert int(re.search(r"const X_JULIA = Int32\((\d)\)", src).group(1)) == defs["X_JULIA"]


def test_binding_exposes_the_shim_api():
    src = JL.read_text()
    for fn in ("enabled", "eval_loss_batch", "eval_tree_array", "eval_grad_tree_array", "eval_loss_grad_batch",
               "set_constants!", "flatten"):
        assert re.search(rf"^function {re.escape(fn)}\(|^{re.escape(fn)}\(.*\) =", src, re.M), fn
    # the shared device-dataset table is only touched under the lock, keyed by
    # (dataset, device); batch scoring creates its program in the calling
    # thread's context (srhip_eval_loss_batch_ctx), so threads run concurrently
    # on one shared dataset
    body = re.search(r"function device_dataset\(.*?\nend", src, re.S).group(0)
    assert re.search(r"lock\(CTX_LOCK\) do", body) and "DEVICE_DATASETS" in body and "device)" in body
    ev = re.search(r"function eval_loss_batch\(.*?\nend", src, re.S).group(0)
    assert "srhip_eval_loss_batch_ctx" in ev and "context(device)" in ev
    grad = re.search(r"function eval_loss_grad_batch\(.*?\nend", src, re.S).group(0)
    assert "device_dataset(dataset, p.device)" in grad
    assert re.search(r"rc == SRHIP_ERR_INVALID && throw\(ArgumentError", src)


BATCHED = ROOT / "symbolicregression.jl_amd" / "julia" / "BatchedCallers.jl"
REFERENCE_SRC = Path("/root/reference/src")


def test_batched_callers_use_existing_functions():
    """BatchedCallers.jl (the Julia-side candidate batching of SURVEY.md §8 f1)
    imports the reference's own mutation / scoring functions and calls the
    SRHip binding; every imported name must be defined in the reference
    (checked when its sources are present, i.e. in the build container) and
    every SRHip.* it uses must exist in SRHip.jl."""
    src = BATCHED.read_text()
    code = "\n".join(ln.split("#")[0] for ln in src.splitlines())
    imported = []
    for m in re.finditer(r"import \.\.(\w+):\s*((?:[\w!]+\s*,\s*)*[\w!]+)", code):
        imported += [n.strip() for n in m.group(2).split(",")]
    assert {"next_generation"} .isdisjoint(imported)  # it is split, not called
    for need in ("mutate_constant", "mutate_operator", "append_random_op", "prepend_random_op", "insert_random_op",
                 "delete_random_op", "check_constraints", "score_func", "loss_to_score", "optimize_constants",
                 "best_of_sample", "crossover_trees"):
        assert need in imported, need
    srhip_jl = JL.read_text()
    for call in set(re.findall(r"SRHip\.([\w!]+)", code)):
        c = re.escape(call)
        assert re.search(rf"(function {c}\(|struct {c}\b|^{c}\()", srhip_jl, re.M), f"SRHip.{call} missing"
    for fn in ("population_batched", "finalize_scores_batched", "reg_evol_cycle_batched", "propose", "accept",
               "reg_evol_cycle_lockstep", "s_r_cycle_lockstep", "crossover_children"):
        assert re.search(rf"^function {fn}\(", code, re.M), fn
    if REFERENCE_SRC.exists():
        defs = "\n".join(p.read_text() for p in REFERENCE_SRC.glob("*.jl"))
        dyn = {"Node", "copy_node", "count_constants", "count_depth", "simplify_tree", "combine_operators"}
        for name in imported:
            if name in dyn or name in ("Options", "Dataset", "RecordType", "RunningSearchStatistics", "PopMember",
                                       "Population"):
                continue  # DynamicExpressions (not vendored) or types
            assert re.search(rf"(function {re.escape(name)}\(|^{re.escape(name)}\(.*\) =)", defs, re.M), \
                f"{name} is not defined in the reference"


def test_device_datasets_are_weak_and_freed():
    """the device copies of a Dataset are held weakly
    (WeakKeyDict keyed by the mutable Dataset) and freed by a finaliser that
    calls srhip_dataset_destroy, or at once by release_dataset!."""
    src = JL.read_text()
    assert re.search(r"const DEVICE_DATASETS = WeakKeyDict\{Dataset,", src)
    assert re.search(r"mutable struct DeviceCopy", src)
    body = re.search(r"function device_dataset\(.*?\nend", src, re.S).group(0)
    assert "finalizer(free!, d)" in body
    free = re.search(r"function free!\(d::DeviceCopy\).*?\nend", src, re.S).group(0)
    assert "destroy_dataset(d.h)" in free and "d.h = C_NULL" in free
    assert re.search(r"^function release_dataset!\(", src, re.M)
    # the reference's Dataset is a mutable struct (a WeakKeyDict needs one)
    if REFERENCE_SRC.exists():
        assert re.search(r"mutable struct Dataset\{", (REFERENCE_SRC / "Dataset.jl").read_text())


def test_eval_tree_array_reuses_an_uploaded_dataset():
    """a Dataset's device copy is reused only when the caller
    passes the Dataset itself, with the Dataset and its DeviceCopy rooted
    (GC.@preserve) across the ccall; a bare X is uploaded for the call (it may
    have changed) and freed."""
    src = JL.read_text()
    assert "uploaded_dataset_of" not in src
    mats = re.findall(r"function eval_tree_array_batch\(.*?\nend", src, re.S)
    assert len(mats) == 2
    by_x = next(b for b in mats if "X::AbstractMatrix" in b.split("\n")[0])
    by_ds = next(b for b in mats if "dataset::Dataset" in b.split("\n")[0])
    assert "upload(X" in by_x and "destroy_dataset(ds)" in by_x
    assert "device_dataset(dataset, device)" in by_ds and "GC.@preserve dataset dcopy" in by_ds
    one = re.search(r"function eval_tree_array\(.*?\nend", src, re.S).group(0)
    assert "eval_tree_array_batch(" in one and "upload(" not in one


def test_constopt_struct_matches_the_header():
    """SRHip.ConstOptOptions mirrors srhip_constopt_options field by field."""
    hdr = re.sub(r"/\*.*?\*/", "", HDR.read_text(), flags=re.S)
    cstruct = re.search(r"typedef struct srhip_constopt_options \{(.*?)\}", hdr, re.S).group(1)
    cfields = [re.match(r"\s*(.*?)\s*(\w+)$", f.strip()).groups() for f in cstruct.split(";") if f.strip()]
    jl = re.search(r"struct ConstOptOptions.*?\n(.*?)\nend", JL.read_text(), re.S).group(1)
    jfields = [ln.split("#")[0].strip().split("::") for ln in jl.splitlines() if "::" in ln]
    assert [n for _, n in cfields] == [n for n, _ in jfields]
    kinds = {"int32_t": "Int32", "const double*": "Ptr{Float64}", "uint64_t": "UInt64"}
    assert [kinds[t] for t, _ in cfields] == [t for _, t in jfields]


def test_batched_optimiser_is_used_by_the_callers():
    """optimize_and_simplify_population (SingleIteration.jl:63-82)
    and the :optimize mutation go through SRHip.optimize_constants_batch!
    (srhip_optimize_constants_batch), not the per-member CPU optimiser."""
    src = JL.read_text()
    body = re.search(r"function optimize_constants_batch!\(.*?\nend", src, re.S).group(0)
    assert "srhip_optimize_constants_batch" in body and "randn(T, nc)" in body
    assert "options.optimizer_options.iterations" in body and "set_constants(trees[i]" in body
    code = "\n".join(ln.split("#")[0] for ln in BATCHED.read_text().splitlines())
    oc = re.search(r"function optimize_constants_batched\(.*?\nend", code, re.S).group(0)
    assert "SRHip.optimize_constants_batch!(" in oc
    pop = re.search(r"function optimize_and_simplify_population_batched\(.*?\nend", code, re.S).group(0)
    assert "optimize_constants_batched(" in pop and "finalize_scores_batched(" in pop
    prop = re.search(r"function propose\(.*?\nend", code, re.S).group(0)
    assert "optimize_constants(" not in prop  # deferred to one batched call per cycle
    cyc = re.search(r"function reg_evol_cycle_batched\(.*?\nend", code, re.S).group(0)
    assert "optimize_constants_batched(dataset, to_opt, options)" in cyc
