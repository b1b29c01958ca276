"""Constant gradients (eval_grad_tree_array(...; variable=false),
src/InterfaceDynamicExpressions.jl:105-107; the batched ∂loss/∂c for
src/ConstantOptimization.jl). Ported from test/test_derivatives.jl:88-123
(analytic gradients, rtol 0.1 there; tighter here) plus engine-vs-oracle
forward-mode parity on random trees."""
import numpy as np
import pytest

import oracle
import srhip
from numerics import EPS, assert_close_conditioned
from srhip import Node


def eq5_tree(o, c1=2.1, c2=-3.2):
    """pow_abs2(x1, x2) + x3 + custom_cos(c1 + x3) + c2 / x1 with the custom
    operators spelled with supported ones: |x1|^x2, cos(.)^2 = square(cos(.))."""
    x1, x2, x3 = Node("x1"), Node("x2"), Node("x3")
    B, U = o.make_binary, o.make_unary
    t = B("+", B("^", U("abs", x1), x2), x3)
    t = B("+", t, U("square", U("cos", B("+", Node(val=c1), x3))))
    return B("+", t, B("/", Node(val=c2), x1))


def analytic_eq5(X, c1=2.1, c2=-3.2):
    x1, x3 = X[0], X[2]
    return np.stack([-2 * np.cos(c1 + x3) * np.sin(c1 + x3), 1.0 / x1])


OPTS = dict(binary_operators=["+", "*", "-", "/", "^"], unary_operators=["cos", "exp", "sin", "abs", "square"])


def oracle_grad(tree, o, X):
    flat = srhip.flatten([tree], o, dtype=np.float64)
    k, a, c = flat.tree(0)
    return oracle.eval_grad_consts(k, a, c, X, len(c))


def test_oracle_derivatives_kat():
    """test_derivatives.jl:88-123 on the oracle."""
    o = srhip.Options(**OPTS)
    X = np.random.default_rng(0).random((3, 100)) * 5
    # equation4 = 3.2 * x1 → ∂/∂c = x1
    t4 = o.make_binary("*", Node(val=3.2), Node("x1"))
    _, g, ok = oracle_grad(t4, o, X)
    assert ok and np.allclose(g[0], X[0], rtol=1e-12)
    _, g, ok = oracle_grad(eq5_tree(o), o, X)
    assert ok and np.allclose(g, analytic_eq5(X), rtol=1e-9)


@pytest.mark.gpu
def test_engine_derivatives_kat(gpu_ctx):
    o = srhip.Options(**OPTS)
    X = np.random.default_rng(0).random((3, 100)) * 5
    t4 = o.make_binary("*", Node(val=3.2), Node("x1"))
    v, g, ok = srhip.eval_grad_tree_array(t4, X, o)
    assert ok and np.allclose(g[0], X[0], rtol=1e-12)
    v, g, ok = srhip.eval_grad_tree_array(eq5_tree(o), X, o)
    assert ok and np.allclose(g, analytic_eq5(X), rtol=1e-9)
    for T in (np.float32,):
        v, g, ok = srhip.eval_grad_tree_array(eq5_tree(o), X.astype(T), o)
        assert ok and np.allclose(g, analytic_eq5(X), rtol=1e-3, atol=1e-4)


def grad_spread(tree, o, X, T, nperturb=3, seed=0):
    """Spread of the oracle's (value, gradient) under ulp-scale perturbations
    of X and the constants (float64 evaluation)."""
    rng = np.random.default_rng(seed)
    flat = srhip.flatten([tree], o, dtype=np.float64)
    k, a, c = flat.tree(0)
    c = srhip.flatten([tree], o, dtype=T).consts.astype(np.float64)
    X64 = X.astype(np.float64)
    v0, g0, ok0 = oracle.eval_grad_consts(k, a, c, X64, len(c))
    sv, sg = np.zeros_like(v0), np.zeros_like(g0)
    eps = EPS[np.dtype(T)]
    with np.errstate(invalid="ignore", over="ignore"):
        for _ in range(nperturb):
            v, g, _ = oracle.eval_grad_consts(k, a, c * (1 + eps * rng.uniform(-1, 1, c.shape)),
                                              X64 * (1 + eps * rng.uniform(-1, 1, X.shape)), len(c))
            sv = np.where(np.isfinite(v - v0), np.maximum(sv, np.abs(v - v0)), np.inf)
            sg = np.where(np.isfinite(g - g0), np.maximum(sg, np.abs(g - g0)), np.inf)
    return v0, g0, ok0, sv, sg


@pytest.mark.gpu
@pytest.mark.parametrize("T", [np.float64, np.float32])
def test_engine_gradients_vs_oracle_random(gpu_ctx, T):
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(300, o, 4, T, seed=61)
    X = np.random.default_rng(62).standard_normal((4, 777)).astype(T)
    val, grads, ok = srhip.eval_grad_tree_array(trees, X, o)
    ncheck = 0
    vals, refs, svs, grs, rgs, sgs = [], [], [], [], [], []
    # did_succeed in T (f32 overflows where f64 does not): from the T oracle
    _, ok_T = oracle.eval_trees(srhip.flatten(trees, o, dtype=T), X, dtype=T)
    assert np.array_equal(ok, ok_T)
    for t, tree in enumerate(trees):
        rv, rg, rok, sv, sg = grad_spread(tree, o, X, T)
        if not (ok[t] and rok):
            continue
        vals.append(val[t])
        refs.append(rv)
        svs.append(sv)
        grs.append(grads[t].ravel())
        rgs.append(rg.ravel())
        sgs.append(sg.ravel())
        ncheck += rg.size
    rtol = 1e-11 if T == np.float64 else 1e-5
    bad = 0.0 if T == np.float64 else 2e-3
    cat = np.concatenate
    assert_close_conditioned(cat(vals), cat(refs), cat(svs), rtol=rtol, atol=rtol, msg="values", max_bad_frac=bad)
    assert_close_conditioned(cat(grs), cat(rgs), cat(sgs), rtol=rtol, atol=rtol, msg="gradients", max_bad_frac=bad)
    assert ncheck > 100


@pytest.mark.gpu
def test_loss_gradient_matches_finite_differences(gpu_ctx):
    """∂loss/∂c (fused kernel) against central differences of the oracle's
    loss, on trees where the difference quotient is stable (two step sizes
    agree)."""
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(120, o, 3, np.float64, seed=71)
    trees = [t for t in trees if srhip.has_constants(t)]
    rng = np.random.default_rng(72)
    X = rng.standard_normal((3, 3000))
    y = 2 * np.cos(X[2]) + X[0] ** 2 - 2
    w = np.abs(rng.standard_normal(3000))
    nchecked = 0
    for weights in (None, w):
        ds = srhip.Dataset(X, y, weights=weights)
        losses, grads, ok = srhip.eval_loss_grad_batch(trees, ds, o)
        ref_l, ref_ok = srhip.eval_loss_batch_ok(trees, ds, o)
        assert np.array_equal(ok, ref_ok)
        np.testing.assert_allclose(losses[ok], ref_l[ok], rtol=1e-9)
        flat = srhip.flatten(trees, o, dtype=np.float64)
        for t in np.flatnonzero(ok)[:40]:
            k, a, c = flat.tree(t)
            c = c.astype(np.float64)
            for j in range(len(c)):
                fds = []
                for h in (1e-5 * max(1.0, abs(c[j])), 1e-6 * max(1.0, abs(c[j]))):
                    cp, cm = c.copy(), c.copy()
                    cp[j] += h
                    cm[j] -= h
                    fds.append((loss_of(k, a, cp, X, y, weights) - loss_of(k, a, cm, X, y, weights)) / (2 * h))
                if not np.all(np.isfinite(fds)) or abs(fds[0] - fds[1]) > 1e-5 * max(1.0, abs(fds[1])):
                    continue  # difference quotient not converged (pole / cancellation nearby)
                assert abs(grads[t][j] - fds[1]) <= 1e-4 * max(1.0, abs(fds[1])), (t, j, grads[t][j], fds)
                nchecked += 1
    assert nchecked > 50


def loss_of(kind, arg, consts, X, y, w):
    out, ok = oracle.eval_tree(kind, arg, consts, X, dtype=np.float64)
    if not ok:
        return np.nan
    r = (out - y) ** 2
    return np.sum(r * w) / np.sum(w) if w is not None else np.mean(r)


@pytest.mark.gpu
def test_many_constants_and_deep_trees(gpu_ctx):
    """Trees with > kGradG constants (several tangent groups) and trees that
    need the 16-slot kernel."""
    o = srhip.Options(binary_operators=["+", "-", "*"], unary_operators=["cos"])
    rng = np.random.default_rng(81)

    def balanced(d):
        if d == 0:
            return Node(val=float(rng.standard_normal())) if rng.random() < 0.5 else Node(feature=int(rng.integers(1, 4)))
        return Node(int(rng.integers(1, 4)), balanced(d - 1), balanced(d - 1))

    trees = [balanced(d) for d in (3, 4, 5, 6, 7) for _ in range(3)]
    X = rng.standard_normal((3, 300))
    val, grads, ok = srhip.eval_grad_tree_array(trees, X, o)
    for t, tree in enumerate(trees):
        rv, rg, rok = oracle_grad(tree, o, X)
        assert ok[t] == rok
        if ok[t]:
            np.testing.assert_allclose(val[t], rv, rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(grads[t], rg, rtol=1e-10, atol=1e-10)
