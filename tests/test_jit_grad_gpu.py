"""Gradient tree code (csrc/jit_grad.cpp): reverse-mode ∂L/∂c of every
constant in one pass, the fast path of srhip_eval_loss_grad for Float32
programs with the L2 loss (ConstantOptimization.jl:12-65's gradient;
eval_grad_tree_array(...; variable=false), InterfaceDynamicExpressions.jl:105-107).

Checked against the forward-mode interpreter kernel (SRHIP_GJIT=0) on the same
trees — did_succeed identical, loss sums to summation-order rounding — and
against Float64 oracle gradients. Tolerance: per constant, relative to
S_j = Σ_rows |w·ℓ'·∂ŷ/∂c_j| (from the Float64 oracle): in a tree each
constant has one path to the root, so ∂ŷ/∂c_j is a product of local
partials that both modes compute from the same forward values; 1e-4·S_j
bounds their Float32 differences, plus 4x the oracle's own spread of the
gradient N_j (perturbed inputs and its Float32 evaluation, `scales`), which
covers ill-conditioned local partials: no constant may exceed it."""
import os

import numpy as np
import pytest

import oracle
import srhip
from srhip import Node
from srhip import constants as K
from numerics import assert_close_conditioned, loss_spread

pytestmark = pytest.mark.gpu

OPSETS = {
    "cfg5": (["+", "-", "*", "/"], ["cos", "exp"]),
    "wide": (["+", "-", "*", "/"], ["sin", "cos", "exp", "neg", "square", "cube", "abs"]),
    # config #3's operators (round 5: safe_log, safe_sqrt and ^ in the
    # gradient tree code), on positive features so that most trees succeed
    "cfg3": (["+", "-", "*", "/", "^"], ["safe_log", "safe_sqrt", "cos", "exp"]),
}


def run(trees, o, X, y, w, gjit, T=np.float32):
    os.environ["SRHIP_GJIT"] = "1" if gjit else "0"
    try:
        ctx = srhip.get_context(0)
        ds = srhip.DeviceDataset(ctx, X, y, w)
        prog = srhip.Program(ctx, srhip.flatten(trees, o, dtype=T), T)
        sums, grads, wsum, ok = prog.eval_loss_grad(ds, K.LOSS["L2"])
        return sums, grads, wsum, ok, prog.grad_jit_info(), prog
    finally:
        del os.environ["SRHIP_GJIT"]


def scales(trees, o, X, y, w, with_noise=False):
    """S_j = Σ_rows |w·2r·∂ŷ/∂c_j| and the Float64 ∂L/∂c from the oracle;
    with_noise also returns N_j, the oracle's spread of the gradient: Σ_rows
    of the largest move of the row's term w·2r·∂ŷ/∂c_j under three 4-ulp
    Float32 perturbations of X and the constants and under the oracle's own
    Float32 evaluation (the reference's precision: every intermediate
    rounded, which input perturbations cannot show inside a cancellation
    such as x5 + (x1 - x5)), plus |w·2·∂ŷ/∂c_j|·4 ulp of |ŷ|+|y| (the
    residual's own rounding) — how far a correct Float32 evaluation may move
    the sum, through the residual or through an ill-conditioned local
    partial of ∂ŷ/∂c_j."""
    flat = srhip.flatten(trees, o, dtype=np.float64)
    X64, y64 = X.astype(np.float64), y.astype(np.float64)
    w64 = np.ones_like(y64) if w is None else w.astype(np.float64)
    eps = float(np.finfo(np.float32).eps)
    rng = np.random.default_rng(0)
    S, G, N = [], [], []
    for t in range(len(trees)):
        k, a, c = flat.tree(t)
        c = srhip.flatten([trees[t]], o, dtype=np.float32).consts.astype(np.float64)
        if len(c) == 0:
            continue
        with np.errstate(all="ignore"):
            out, g, ok = oracle.eval_grad_consts(k, a, c, X64, len(c))
            if not ok:
                for L in (S, G, N):
                    L.append(np.full(len(c), np.nan))
                continue
            term = w64 * 2.0 * (out - y64) * g
            if with_noise:
                dv = np.abs(w64 * 2.0 * g) * (4 * eps * (np.abs(out) + np.abs(y64)))
                mv = np.zeros_like(term)
                for _ in range(3):
                    o2, g2, ok2 = oracle.eval_grad_consts(k, a, c * (1 + 4 * eps * rng.uniform(-1, 1, c.shape)),
                                                          X64 * (1 + 4 * eps * rng.uniform(-1, 1, X.shape)), len(c))
                    if ok2:
                        mv = np.maximum(mv, np.abs(w64 * 2.0 * (o2 - y64) * g2 - term))
                    else:
                        mv[:] = np.inf
                o3, g3, ok3 = oracle.eval_grad_consts(k, a, c.astype(np.float32), X, len(c), dtype=np.float32)
                if ok3:
                    t3 = w64 * 2.0 * (o3.astype(np.float64) - y64) * g3.astype(np.float64)
                    mv = np.maximum(mv, np.where(np.isfinite(t3), np.abs(t3 - term), np.inf))
                else:
                    mv[:] = np.inf
                N.append((dv + mv).sum(axis=1))
        S.append(np.abs(term).sum(axis=1))
        G.append(term.sum(axis=1))
    out = (np.concatenate(S), np.concatenate(G))
    return out + (np.concatenate(N),) if with_noise else out


def scales32(trees, o, X, y, w):
    """The oracle's Float32 evaluation of ∂L/∂c (the reference's precision):
    per constant Σ|terms|, Σ terms, and what a 4-ulp move of ŷ (or y) moves
    the terms by — the tight bound of the direct comparison (no perturbation
    allowance)."""
    flat = srhip.flatten(trees, o, dtype=np.float32)
    y64 = y.astype(np.float64)
    w64 = np.ones_like(y64) if w is None else w.astype(np.float64)
    eps = float(np.finfo(np.float32).eps)
    S, G, DV = [], [], []
    for t in range(len(trees)):
        k, a, c = flat.tree(t)
        if len(c) == 0:
            continue
        with np.errstate(all="ignore"):
            out, g, ok = oracle.eval_grad_consts(k, a, c.astype(np.float32), X, len(c), dtype=np.float32)
            if not ok:
                for L in (S, G, DV):
                    L.append(np.full(len(c), np.nan))
                continue
            out, g = out.astype(np.float64), g.astype(np.float64)
            term = w64 * 2.0 * (out - y64) * g
            DV.append((np.abs(w64 * 2.0 * g) * (4 * eps * (np.abs(out) + np.abs(y64)))).sum(axis=1))
        S.append(np.abs(term).sum(axis=1))
        G.append(term.sum(axis=1))
    return np.concatenate(S), np.concatenate(G), np.concatenate(DV)


# Beyond this scale a constant's Float32 gradient overflows depending on the
# order of its products (reverse mode multiplies from the seed 2·w·r down the
# path, forward mode from 1 up): such trees have losses near 1e30 or more
# and are excluded from the comparison (both paths are then checked only for
# agreeing on did_succeed and on the loss).
S_MAX = 1e20


def check_grads(g, ref, S, ok_c, rtol, max_bad_frac, msg, noise=None):
    sel = ok_c & np.isfinite(S) & np.isfinite(ref) & (S < S_MAX)
    if noise is not None:
        sel &= np.isfinite(noise)
    a, b = g[sel], ref[sel]
    with np.errstate(invalid="ignore"):
        err = np.abs(a - b)
    bound = rtol * S[sel] + 1e-30 + (0 if noise is None else 4 * noise[sel])
    same = (a == b) | (np.isnan(a) & np.isnan(b))
    bad = ~same & ~(err <= bound)
    frac = bad.mean() if bad.size else 0.0
    with np.errstate(invalid="ignore"):
        worst = float(np.nanmax(err / bound)) if bad.size else 0.0
    assert frac <= max_bad_frac, (msg, int(bad.sum()), bad.size, worst)
    return int(sel.sum())


@pytest.mark.parametrize("opset", list(OPSETS))
@pytest.mark.parametrize("weighted", [False, True])
def test_grad_tree_code_matches_interpreter_and_oracle(gpu_ctx, opset, weighted):
    b_ops, u_ops = OPSETS[opset]
    o = srhip.Options(binary_operators=b_ops, unary_operators=u_ops)
    rng = np.random.default_rng(5 + weighted)
    n = 3001  # a partial last tile
    X = rng.standard_normal((5, n)).astype(np.float32)
    if opset == "cfg3":
        X = (np.abs(X) + np.float32(0.1)).astype(np.float32)
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
    w = np.abs(rng.standard_normal(n)).astype(np.float32) if weighted else None
    trees = srhip.random_population(600 if opset != "cfg3" else 1500, o, 5, np.float32, seed=91 + weighted)
    s1, g1, w1, ok1, info, prog = run(trees, o, X, y, w, True)
    s0, g0, w0, ok0, info0, _ = run(trees, o, X, y, w, False)
    assert info["ntrees"] >= 0.95 * len(trees), info
    assert info0["ntrees"] == 0
    assert np.array_equal(ok1, ok0)
    assert w1 == w0
    # the tree code's forward runs the guarded FAST routines (the interpreter
    # the PRECISE ones): within 2e-5, or within 4x the tree's conditioning
    rel = np.abs(s1 - s0) / np.abs(s0)
    out = np.flatnonzero(ok1 & ~(rel <= 2e-5))
    if out.size:
        sp = loss_spread([trees[i] for i in out], o, X, y, w, np.float32, nperturb=3)
        assert_close_conditioned(s1[out], s0[out], sp, rtol=2e-5, factor=4.0, msg="tree code vs interpreter losses")
    ok_c = np.repeat(ok1, np.diff(prog.flat.const_off))
    assert np.all(np.isnan(g1[~ok_c])) and np.all(np.isnan(g0[~ok_c]))
    S, ref, N = scales(trees, o, X, y, w, with_noise=True)
    # the tree code's forward is the guarded FAST one: the residuals may move
    # by what a correct Float32 evaluation may (N)
    # every constant within the bound (none allowed beyond it: tools/debug_grads.py
    # reports 0 of 1041-1554 in each case, profiles/r03_debug_grads.txt)
    n1 = check_grads(g1, g0, S, ok_c, 1e-4, 0.0, "tree code vs interpreter", noise=N)
    check_grads(g1, ref, S, ok_c, 1e-4, 0.0, "tree code vs Float64 oracle", noise=N)
    check_grads(g0, ref, S, ok_c, 1e-4, 0.0, "interpreter vs Float64 oracle", noise=N)
    assert n1 > 500
    # directly against the oracle's Float32 gradients, tight: 1e-5 of Σ|terms|
    # plus a 4-ulp move of ŷ (the sums' rounding and the FAST forward), none beyond
    # (config #3's safe_log and ^ included: with OCML's logf / powf, 1-ulp
    # differences turned into up to 1.4 % of the constants beyond this bound
    # on ill-conditioned trees; since log and pow of Float32 are evaluated in
    # Float64 and rounded once, as the oracle does, none is)
    S32, G32, DV = scales32(trees, o, X, y, w)
    check_grads(g1, G32, S32, ok_c, 1e-5, 0.0, "tree code vs Float32 oracle", noise=DV / 4)
    check_grads(g0, G32, S32, ok_c, 1e-5, 0.0, "interpreter vs Float32 oracle", noise=DV / 4)


def test_grad_tree_code_many_constants_fall_back(gpu_ctx):
    """A tree with more constants than accumulators runs on the interpreter,
    the others as tree code, in the same call."""
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(3)
    X = rng.standard_normal((3, 1000)).astype(np.float32)
    y = (X[0] * 2 - 1).astype(np.float32)
    big = Node(val=0.5)
    for k in range(20):  # 21 constants
        big = o.make_binary("+", o.make_binary("*", big, Node(val=1.0 + 0.01 * k)), Node("x1"))
    trees = srhip.random_population(300, o, 3, np.float32, seed=4) + [big]
    s1, g1, _, ok1, info, prog = run(trees, o, X, y, None, True)
    s0, g0, _, ok0, _, _ = run(trees, o, X, y, None, False)
    assert info["nrejected"] >= 1 and info["ntrees"] >= 280
    assert np.array_equal(ok1, ok0)
    co = prog.flat.const_off
    np.testing.assert_array_equal(g1[co[-2]:co[-1]], g0[co[-2]:co[-1]])  # the big tree: same kernel
    ok_c = np.repeat(ok1, np.diff(co))
    S, _, N = scales(trees, o, X, y, None, with_noise=True)
    check_grads(g1, g0, S, ok_c, 1e-4, 2e-3, "mixed batch", noise=N)


def test_grad_tree_code_new_constants(gpu_ctx):
    """set_constants: the tree code reads the new constants (no new code)."""
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(8)
    X = rng.standard_normal((4, 2000)).astype(np.float32)
    y = (np.cos(X[1]) * 1.5 - X[2]).astype(np.float32)
    trees = srhip.random_population(400, o, 4, np.float32, seed=12)
    os.environ["SRHIP_GJIT"] = "1"
    try:
        ctx = srhip.get_context(0)
        ds = srhip.DeviceDataset(ctx, X, y)
        flat = srhip.flatten(trees, o, dtype=np.float32)
        prog = srhip.Program(ctx, flat, np.float32)
        prog.eval_loss_grad(ds, K.LOSS["L2"])
        new = (flat.consts * (1 + 0.25 * rng.standard_normal(flat.consts.shape))).astype(np.float32)
        prog.set_constants(new)
        s1, g1, _, ok1 = prog.eval_loss_grad(ds, K.LOSS["L2"])
        assert prog.grad_jit_info()["ntrees"] > 300
        flat2 = srhip.flatten(trees, o, dtype=np.float32)
        flat2.consts[:] = new
        prog2 = srhip.Program(ctx, flat2, np.float32)
        s2, g2, _, ok2 = prog2.eval_loss_grad(ds, K.LOSS["L2"])
    finally:
        del os.environ["SRHIP_GJIT"]
    assert np.array_equal(ok1, ok2)
    np.testing.assert_array_equal(s1[ok1], s2[ok2])
    ok_c = np.repeat(ok1, np.diff(flat.const_off))
    np.testing.assert_array_equal(g1[ok_c], g2[ok_c])


def test_constant_optimisation_on_grad_tree_code(gpu_ctx):
    """The batched BFGS driver on the tree-code gradients recovers the
    known constants (tests/test_constant_optimization.py's problem)."""
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(1)
    X = rng.standard_normal((5, 400)).astype(np.float32)
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
    B, U = o.make_binary, o.make_unary
    three = B("+", B("+", B("*", Node(val=1.0), U("cos", Node("x4"))), B("*", Node(val=0.5),
                                                                         B("*", Node("x1"), Node("x1")))),
              Node(val=0.0))
    os.environ["SRHIP_GJIT"] = "1"
    try:
        res = srhip.optimize_constants_batch(srhip.Dataset(X, y), [three], o, rng=np.random.default_rng(0))
    finally:
        del os.environ["SRHIP_GJIT"]
    assert res.converged[0]
    assert np.allclose(srhip.get_constants(three), [2.0, 1.0, -2.0], atol=2e-3)
    assert res.losses[0] < 1e-5
