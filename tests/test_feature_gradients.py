"""Derivatives with respect to the features: eval_grad_tree_array(...;
variable=true) and eval_diff_tree_array (src/InterfaceDynamicExpressions.jl:55-107),
ported from test/test_derivatives.jl:31-87 (equations 1-2, analytic
gradients instead of Zygote; rtol 0.1 there, far tighter here).

The engine seeds every feature leaf x_f as (x_f + c), c = -0.0, and sums the
constant tangents per feature; the CPU tests check that construction on the
oracle, the GPU tests run it on the engine."""
import numpy as np
import pytest

import oracle
import srhip
from numerics import assert_close_conditioned
from srhip import Node
from srhip.interface import _seed_features
from test_gradients import grad_spread

OPTS = dict(binary_operators=["+", "*", "-", "/", "^"], unary_operators=["cos", "exp", "sin", "abs", "square"])


def eq1(o):
    B = o.make_binary
    return B("+", B("+", B("+", Node("x1"), Node("x2")), Node("x3")), Node(val=3.2))


def eq2(o):
    """pow_abs2(x1, x2) + x3 + custom_cos(1.0 + x3) + 3.0 / x1."""
    B, U = o.make_binary, o.make_unary
    t = B("+", B("+", B("^", U("abs", Node("x1")), Node("x2")), Node("x3")),
          U("square", U("cos", B("+", Node(val=1.0), Node("x3")))))
    return B("+", t, B("/", Node(val=3.0), Node("x1")))


def analytic(j, X):
    x1, x2, x3 = X
    if j == 1:
        return np.ones_like(X)
    return np.stack([x2 * np.abs(x1) ** (x2 - 1) * np.sign(x1) - 3.0 / x1 ** 2,
                     np.abs(x1) ** x2 * np.log(np.abs(x1)),
                     1.0 - 2.0 * np.cos(1.0 + x3) * np.sin(1.0 + x3)])


def oracle_feature_grad(tree, o, X, direction=None):
    plus = o.binary_operators.index("+") + 1
    aug, seeds = _seed_features(tree, plus, direction)
    flat = srhip.flatten([aug], o, dtype=np.float64)
    k, a, c = flat.tree(0)
    v, g, ok = oracle.eval_grad_consts(k, a, c, X, len(c))
    seeds = np.asarray(seeds)
    G = np.stack([g[seeds == f].sum(axis=0) if (seeds == f).any() else np.zeros(X.shape[1])
                  for f in range(1, X.shape[0] + 1)])
    return v, G, ok


def test_seeding_is_value_preserving():
    """x + (-0.0) == x bit for bit, including ±0, ±Inf and NaN."""
    x = np.array([0.0, -0.0, 1.5, -np.inf, np.inf, np.nan, 5e-324, -5e-324])
    for T in (np.float32, np.float64):
        xs = x.astype(T)
        r = xs + T(-0.0)
        assert np.array_equal(r.view(np.uint8), xs.view(np.uint8))


def test_oracle_feature_derivatives_kat():
    o = srhip.Options(**OPTS)
    rng = np.random.default_rng(0)
    X = rng.random((3, 100)) * 5
    for j, eq in ((1, eq1), (2, eq2)):
        tree = eq(o)
        v, G, ok = oracle_feature_grad(tree, o, X)
        v0, ok0 = oracle.eval_trees(srhip.flatten([tree], o, dtype=np.float64), X, dtype=np.float64)
        assert ok and ok0[0] and np.array_equal(v, v0[0])
        np.testing.assert_allclose(G, analytic(j, X), rtol=1e-9, atol=1e-12)
        for d in (1, 2, 3):
            _, Gd, _ = oracle_feature_grad(tree, o, X, d)
            np.testing.assert_allclose(Gd[d - 1], G[d - 1], rtol=1e-15)
            assert not Gd[np.arange(3) != d - 1].any()


def test_absent_feature_has_zero_gradient():
    o = srhip.Options(**OPTS)
    X = np.random.default_rng(1).random((4, 50))
    tree = o.make_binary("*", Node("x2"), Node(val=2.0))
    _, G, ok = oracle_feature_grad(tree, o, X)
    assert ok and np.array_equal(G[1], np.full(50, 2.0)) and not G[[0, 2, 3]].any()


@pytest.mark.gpu
@pytest.mark.parametrize("T", [np.float64, np.float32])
def test_engine_feature_derivatives_kat(gpu_ctx, T):
    o = srhip.Options(**OPTS)
    X = (np.random.default_rng(0).random((3, 100)) * 5).astype(T)
    rtol = 1e-9 if T == np.float64 else 2e-4
    for j, eq in ((1, eq1), (2, eq2)):
        tree = eq(o)
        v, G, ok = srhip.eval_grad_tree_array(tree, X, o, variable=True)
        v0, ok0 = srhip.eval_tree_array(tree, X, o)
        assert ok and ok0 and np.array_equal(v, v0)
        assert G.shape == (3, 100) and G.dtype == T
        np.testing.assert_allclose(G, analytic(j, X.astype(np.float64)), rtol=rtol, atol=rtol)
        for d in (1, 2, 3):
            vd, gd, okd = srhip.eval_diff_tree_array(tree, X, o, d)
            assert okd and np.array_equal(vd, v)
            np.testing.assert_allclose(gd, G[d - 1], rtol=4 * np.finfo(T).eps, atol=0)
        assert not np.allclose(G * 0, analytic(j, X.astype(np.float64)), rtol=0.1)


@pytest.mark.gpu
def test_engine_feature_gradients_vs_oracle_random(gpu_ctx):
    """Random trees, Float64: engine ∂ŷ/∂x against the oracle's forward mode on
    the same seeded trees, within the ulp-perturbation spread."""
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(150, o, 4, np.float64, seed=81)
    X = np.random.default_rng(82).standard_normal((4, 500))
    val, grads, ok = srhip.eval_grad_tree_array(trees, X, o, variable=True)
    plus = o.binary_operators.index("+") + 1
    got, ref, spread = [], [], []
    nchecked = 0
    for t, tree in enumerate(trees):
        aug, seeds = _seed_features(tree, plus, None)
        rv, rg, rok, sv, sg = grad_spread(aug, o, X, np.float64)
        assert bool(ok[t]) == bool(rok)
        if not ok[t]:
            continue
        seeds = np.asarray(seeds)
        for f in range(1, 5):
            m = seeds == f
            got.append(grads[t][f - 1])
            ref.append(rg[m].sum(axis=0) if m.any() else np.zeros(500))
            spread.append(sg[m].sum(axis=0) if m.any() else np.zeros(500))
            nchecked += int(m.any())
    cat = np.concatenate
    assert_close_conditioned(cat(got), cat(ref), cat(spread), rtol=1e-11, atol=1e-11, msg="feature gradients")
    assert nchecked > 50
