"""ctypes wrapper of the CPU restatement (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker or the timed CPU baseline. The
product (libsrhip.so / the srhip package) never uses it.

Parity status: restates DynamicExpressions.jl 0.4.x (unpinned patch,
not vendored) + SymbolicRegression.jl's Operators/LossFunctions; pinned by
the reference's known-answer tests (tests/test_oracle_kat.py), not by outputs
of the reference itself (Julia is absent from this image).
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
_libs = {}


def load(variant: str = "simd"):
    """variant: "scalar" (~turbo=false) or "simd" (~turbo=true)."""
    if variant in _libs:
        return _libs[variant]
    path = HERE / f"liboracle_{variant}.so"
    if not path.exists():
        raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
    L = C.CDLL(str(path))
    vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
    L.oracle_binop_f32.argtypes = [C.c_int, C.c_float, C.c_float]
    L.oracle_binop_f32.restype = C.c_float
    L.oracle_binop_f64.argtypes = [C.c_int, C.c_double, C.c_double]
    L.oracle_binop_f64.restype = C.c_double
    L.oracle_unop_f32.argtypes = [C.c_int, C.c_float]
    L.oracle_unop_f32.restype = C.c_float
    L.oracle_unop_f64.argtypes = [C.c_int, C.c_double]
    L.oracle_unop_f64.restype = C.c_double
    for sfx in ("f32", "f64"):
        f = getattr(L, f"oracle_eval_tree_{sfx}")
        f.argtypes = [vp, vp, vp, i32, vp, i64, i32, vp]
        f.restype = C.c_int
        g = getattr(L, f"oracle_eval_loss_batch_{sfx}")
        g.argtypes = [i32, vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, C.c_int, vp, vp, i64, C.c_int, vp, vp, vp]
        g.restype = None
    L.oracle_elem_loss_f64.argtypes = [C.c_int, vp, C.c_double, C.c_double]
    L.oracle_elem_loss_f64.restype = C.c_double
    L.oracle_elem_loss_f32.argtypes = [C.c_int, vp, C.c_float, C.c_float]
    L.oracle_elem_loss_f32.restype = C.c_float
    for sfx in ("f32", "f64"):
        f = getattr(L, f"oracle_eval_grad_consts_{sfx}")
        f.argtypes = [vp, vp, vp, i32, vp, i64, i32, vp, vp]
        f.restype = C.c_int
    L.oracle_max_threads.restype = C.c_int
    L.oracle_set_noise.argtypes = [C.c_double, C.c_uint64]
    L.oracle_set_noise.restype = None
    _libs[variant] = L
    return L


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _sfx(dtype) -> str:
    return "f32" if np.dtype(dtype) == np.float32 else "f64"


def binop(op: int, x, y, dtype=np.float32):
    L = load()
    return (L.oracle_binop_f32 if _sfx(dtype) == "f32" else L.oracle_binop_f64)(op, x, y)


def unop(op: int, x, dtype=np.float32):
    L = load()
    return (L.oracle_unop_f32 if _sfx(dtype) == "f32" else L.oracle_unop_f64)(op, x)


def elem_loss(loss: int, params, yhat, y, dtype=np.float32):
    """One elementwise loss value in T (sr_oracle_eval.h elem_loss)."""
    L = load()
    p = np.asarray(list(params) if params is not None else [0.0], dtype=np.float64)
    f = L.oracle_elem_loss_f32 if _sfx(dtype) == "f32" else L.oracle_elem_loss_f64
    return f(loss, _p(p), yhat, y)


def julia_X(X: np.ndarray, dtype) -> np.ndarray:
    """(nfeatures, n) → Julia column-major storage."""
    return np.asfortranarray(np.asarray(X, dtype=dtype))


def eval_tree(kind, arg, consts, X: np.ndarray, dtype=np.float32, variant="simd"):
    """One tree: (output[n], did_succeed)."""
    L = load(variant)
    Xj = julia_X(X, dtype)
    nfeat, n = Xj.shape
    kind = np.ascontiguousarray(kind, dtype=np.uint8)
    arg = np.ascontiguousarray(arg, dtype=np.uint16)
    c = np.ascontiguousarray(consts, dtype=dtype)
    out = np.empty(n, dtype=dtype)
    ok = getattr(L, f"oracle_eval_tree_{_sfx(dtype)}")(_p(kind), _p(arg), _p(c), len(kind), _p(Xj), n, nfeat,
                                                       _p(out))
    return out, bool(ok)


def eval_trees(flat, X: np.ndarray, dtype=np.float32, variant="simd"):
    outs, oks = [], []
    for t in range(flat.ntrees):
        k, a, c = flat.tree(t)
        o, ok = eval_tree(k, a, c, X, dtype, variant)
        outs.append(o)
        oks.append(ok)
    return np.stack(outs) if outs else np.zeros((0, X.shape[1]), dtype=dtype), np.asarray(oks, dtype=bool)


def eval_loss_batch(flat, X, y, w=None, loss=0, params=(0.0,), row_idx=None, nthreads=0, dtype=np.float32,
                    variant="simd"):
    """(Σ w ℓ per tree in fp64, reference loss in T, did_succeed)."""
    L = load(variant)
    Xj = julia_X(X, dtype)
    nfeat, n = Xj.shape
    ya = np.ascontiguousarray(y, dtype=dtype)
    wa = None if w is None else np.ascontiguousarray(w, dtype=dtype)
    par = np.asarray(params, dtype=np.float64)
    idx = None if row_idx is None else np.ascontiguousarray(row_idx, dtype=np.int64)
    nt = flat.ntrees
    sums = np.zeros(max(nt, 1), dtype=np.float64)
    losses = np.zeros(max(nt, 1), dtype=dtype)
    ok = np.zeros(max(nt, 1), dtype=np.uint8)
    consts = np.ascontiguousarray(flat.consts, dtype=dtype)
    getattr(L, f"oracle_eval_loss_batch_{_sfx(dtype)}")(
        nt, _p(flat.node_off), _p(flat.kind), _p(flat.arg), _p(flat.const_off), _p(consts), _p(Xj), _p(ya),
        _p(wa), n, nfeat, int(loss), _p(par), _p(idx), 0 if idx is None else len(idx), int(nthreads), _p(sums),
        _p(losses), _p(ok))
    return sums[:nt], losses[:nt], ok[:nt].astype(bool)


def eval_grad_consts(kind, arg, consts, X, nconst, dtype=np.float64):
    """Forward-mode ∂ŷ/∂c of one tree at every row: (ŷ, grad [nconst][n], ok),
    computed in dtype (float32: every intermediate rounded as the reference's
    Float32 evaluation rounds it)."""
    L = load()
    dt = np.dtype(dtype)
    Xj = julia_X(X, dt)
    nfeat, n = Xj.shape
    kind = np.ascontiguousarray(kind, dtype=np.uint8)
    arg = np.ascontiguousarray(arg, dtype=np.uint16)
    c = np.ascontiguousarray(consts, dtype=dt)
    out = np.empty(n, dtype=dt)
    grad = np.empty((max(nconst, 1), n), dtype=dt)
    ok = getattr(L, f"oracle_eval_grad_consts_{_sfx(dt)}")(_p(kind), _p(arg), _p(c), len(kind), _p(Xj), n, nfeat,
                                                           _p(out), _p(grad))
    return out, grad[:nconst], bool(ok)


def set_noise(eps: float, seed: int = 0, variant: str = "simd"):
    """Test-only: multiply every float64 transcendental value by (1 + eps u),
    u in [-1, 1) hashed from the operand and seed (0 = off); see sr_oracle.c."""
    load(variant).oracle_set_noise(float(eps), int(seed) & (2**64 - 1))


def max_threads() -> int:
    return load().oracle_max_threads()
