"""The reference's known-answer tests for the hot path, ported.

Each runs on the oracle (pins the CPU restatement, no GPU) and on the engine
(`-m gpu`). Sources: test/test_operators.jl, test/test_nan_detection.jl,
test/test_turbo_nan.jl, test/test_evaluation.jl, test/test_losses.jl,
test/test_tree_construction.jl.
"""
import math

import numpy as np
import pytest

import oracle
import srhip
from srhip import Node
from srhip import constants as K
from backends import BACKENDS

# ---------------------------------------------------------------- test_operators.jl:25-64


@pytest.mark.parametrize("T", [np.float32, np.float64])
def test_operators_exact(T):
    """Exact safe-operator known answers (test_operators.jl:187-223)."""
    u = lambda name, x: T(oracle.unop(K.UOP[name], T(x), T))
    b = lambda name, x, y: T(oracle.binop(K.BOP[name], T(x), T(y), T))
    val, val2 = T(0.5), T(3.2)
    assert abs(u("LOG", val) - np.log(val)) < 1e-6
    assert np.isnan(u("LOG", -val))
    assert abs(u("LOG2", val) - np.log2(val)) < 1e-6
    assert np.isnan(u("LOG2", -val))
    assert abs(u("LOG10", val) - np.log10(val)) < 1e-6
    assert np.isnan(u("LOG10", -val))
    assert abs(u("ACOSH", val2) - np.arccosh(val2)) < 1e-6
    assert np.isnan(u("ACOSH", -val2))
    assert u("NEG", -val) == val
    assert u("SQRT", val) == np.sqrt(val)
    assert np.isnan(u("SQRT", -val))
    assert b("MUL", val, val2) == val * val2
    assert b("ADD", val, val2) == val + val2
    assert b("SUB", val, val2) == val - val2
    assert u("SQUARE", val) == val * val
    assert u("CUBE", val) == val * val * val
    assert np.isnan(b("POW", 0.0, -1.0))
    assert np.isnan(b("POW", -val, val2))
    assert np.isnan(b("POW", -val, -val2)) and np.isnan(b("POW", 0.0, -val2))
    assert abs(b("POW", val, val2) - val ** val2) < 1e-6
    assert abs(b("POW", val, -val2) - val ** (-val2)) < 1e-6
    assert not np.isnan(b("POW", -1.0, 2.0))
    assert np.isnan(b("POW", -1.0, 2.1))
    assert np.isnan(u("LOG", 0.0)) and np.isnan(u("LOG2", 0.0)) and np.isnan(u("LOG10", 0.0))
    assert b("DIV", val, val2) == val / val2
    assert b("GREATER", val, val2) == 0.0
    assert b("GREATER", val2, val) == 1.0
    assert u("RELU", -val) == 0.0
    assert u("RELU", val) == val
    assert b("LOGICAL_OR", val, val2) == 1.0
    assert b("LOGICAL_OR", 0.0, val2) == 1.0
    assert b("LOGICAL_AND", 0.0, val2) == 0.0


@pytest.mark.parametrize("T", [np.float32, np.float64])
def test_julia_base_semantics(T):
    """Base semantics the engine relies on: mod, max/min signed zeros, sign,
    round ties-to-even, gamma Inf → NaN, atanh_clip wrap."""
    u = lambda name, x: T(oracle.unop(K.UOP[name], T(x), T))
    b = lambda name, x, y: T(oracle.binop(K.BOP[name], T(x), T(y), T))
    assert b("MOD", 5.5, 2.0) == 1.5
    assert b("MOD", -5.5, 2.0) == 0.5
    assert b("MOD", 5.5, -2.0) == -0.5
    assert math.copysign(1.0, b("MOD", 4.0, -2.0)) == -1.0  # r == 0 → copysign(r, y)
    assert np.isnan(b("MOD", 1.0, 0.0))
    assert math.copysign(1.0, b("MAX", -0.0, 0.0)) == 1.0
    assert math.copysign(1.0, b("MIN", 0.0, -0.0)) == -1.0
    assert u("SIGN", -3.0) == -1.0 and u("SIGN", 2.0) == 1.0 and u("SIGN", 0.0) == 0.0
    assert u("ROUND", 2.5) == 2.0 and u("ROUND", 3.5) == 4.0 and u("ROUND", -2.5) == -2.0
    assert np.isnan(u("GAMMA", 0.0))  # Inf → NaN (Operators.jl:8-11)
    assert np.isnan(u("GAMMA", -1.0))
    assert abs(u("GAMMA", 5.0) - 24.0) < 1e-4
    assert abs(u("ATANH_CLIP", 0.5) - np.arctanh(0.5)) < 1e-6
    assert abs(u("ATANH_CLIP", 2.5) - np.arctanh(0.5)) < 1e-6  # mod(3.5, 2) - 1 = 0.5
    assert u("INV", 4.0) == 0.25


# ---------------------------------------------------------------- test_nan_detection.jl:5-49


def nan_cases(T):
    o = srhip.Options(binary_operators=["+", "*", "/", "-", "^"], unary_operators=["cos", "sin", "exp", "sqrt"])
    x1 = Node(feature=1)
    B = lambda name, a, b: o.make_binary(name, a, b if isinstance(b, Node) else Node(val=T(b)))
    U = o.make_unary
    X100 = np.full((1, 10), 100, dtype=T)
    X0 = np.full((1, 10), 0, dtype=T)
    return o, [
        ("exp^4 overflow", U("exp", U("exp", U("exp", U("exp", B("+", x1, 1))))), X100),
        ("division by constant zero", U("cos", B("/", x1, 0.0)), X100),
        ("safe_sqrt(-1)", U("sqrt", B("-", x1, 1)), X0),
        ("safe_pow(-1, 0.5)", B("^", B("-", x1, 1), 0.5), X0),
        ("Inf constant", U("cos", B("+", x1, np.inf)), X0),
        ("NaN constant", U("cos", B("+", x1, np.nan)), X0),
    ]


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("T", [np.float32, np.float64])
def test_nan_detection(backend, T):
    o, cases = nan_cases(T)
    for name, tree, X in cases:
        _, flag = backend.eval_tree_array(tree, X, o)
        assert not flag, name


@pytest.mark.parametrize("backend", BACKENDS)
def test_turbo_nan_no_throw(backend):
    """test_turbo_nan.jl: domain errors never throw; sqrt(sin(-π/2)) fails."""
    o = srhip.Options(binary_operators=["+", "*"], unary_operators=["sin", "exp", "sqrt"], turbo=True)
    tree = Node(3, Node(1, Node(val=-math.pi / 2)))
    _, flag = backend.eval_tree_array(tree, np.zeros((1, 1)), o)
    assert not flag
    tree = Node(3, Node(1, Node(feature=1)))
    _, flag = backend.eval_tree_array(tree, np.array([[-math.pi / 2]]), o)
    assert not flag


# ---------------------------------------------------------------- test_evaluation.jl:7-75


def evaluation_cases():
    """(tree builder, closure) pairs exercising every fused pattern."""
    f32 = np.float32
    sin, cos = np.sin, np.cos
    return [
        ("deg2_l0_r0 x*x", lambda b: b.mul(b.x1, b.x2), lambda x1, x2, x3: x1 * x2),
        ("deg2_l0_r0 x*c", lambda b: b.mul(b.x1, b.c(3.0)), lambda x1, x2, x3: x1 * f32(3.0)),
        ("deg2_l0_r0 c*x", lambda b: b.mul(b.c(3.0), b.x2), lambda x1, x2, x3: f32(3.0) * x2),
        ("deg2_l0_r0 c*c", lambda b: b.mul(b.c(3.0), b.c(6.0)), lambda x1, x2, x3: f32(3.0) * f32(6.0) + 0 * x1),
        ("deg2_l0 x*sin", lambda b: b.mul(b.x1, b.sin(b.x2)), lambda x1, x2, x3: x1 * sin(x2)),
        ("deg2_l0 c*sin", lambda b: b.mul(b.c(3.0), b.sin(b.x2)), lambda x1, x2, x3: f32(3.0) * sin(x2)),
        ("deg2_r0 sin*x", lambda b: b.mul(b.sin(b.x1), b.x2), lambda x1, x2, x3: sin(x1) * x2),
        ("deg2_r0 sin*c", lambda b: b.mul(b.sin(b.x1), b.c(3.0)), lambda x1, x2, x3: sin(x1) * f32(3.0)),
        ("deg1_l2 cos(x*x)", lambda b: b.cos(b.mul(b.x1, b.x2)), lambda x1, x2, x3: cos(x1 * x2)),
        ("deg1_l2 cos(x*c)", lambda b: b.cos(b.mul(b.x1, b.c(3.0))), lambda x1, x2, x3: cos(x1 * f32(3.0))),
        ("deg1_l2 cos(c*x)", lambda b: b.cos(b.mul(b.c(3.0), b.x2)), lambda x1, x2, x3: cos(f32(3.0) * x2)),
        ("deg1_l2 cos(c*c)", lambda b: b.cos(b.mul(b.c(3.0), b.c(-0.5))),
         lambda x1, x2, x3: cos(f32(3.0) * f32(-0.5)) + 0 * x1),
        ("deg1_l1 cos(sin(x))", lambda b: b.cos(b.sin(b.x1)), lambda x1, x2, x3: cos(sin(x1))),
        ("deg1_l1 cos(sin(c))", lambda b: b.cos(b.sin(b.c(3.0))), lambda x1, x2, x3: cos(sin(f32(3.0))) + 0 * x1),
        ("generic", lambda b: b.mul(b.add(b.sin(b.mul(b.cos(b.mul(b.sin(b.mul(b.cos(b.x1), b.x3)), b.c(3.0))),
                                                   b.c(-0.5))), b.c(2.0)), b.c(5.0)),
         lambda x1, x2, x3: (sin(cos(sin(cos(x1) * x3) * f32(3.0)) * f32(-0.5)) + f32(2.0)) * f32(5.0)),
    ]


class Builder:
    def __init__(self, o, T):
        self.o, self.T = o, T
        self.x1, self.x2, self.x3 = Node("x1"), Node("x2"), Node("x3")

    def c(self, v):
        return Node(val=self.T(v))

    def mul(self, a, b):
        return self.o.make_binary("*", a, b)

    def add(self, a, b):
        return self.o.make_binary("+", a, b)

    def sin(self, a):
        return self.o.make_unary("sin", a)

    def cos(self, a):
        return self.o.make_unary("cos", a)


@pytest.mark.parametrize("backend", BACKENDS)
def test_evaluation_fused_patterns(backend):
    o = srhip.Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "sin"])
    N, nfeat = 100, 3
    X = np.random.default_rng(0).standard_normal((nfeat, N)).astype(np.float32)
    b = Builder(o, np.float32)
    for name, mk, fn in evaluation_cases():
        test_y, ok = backend.eval_tree_array(mk(b), X, o)
        true_y = fn(X[0], X[1], X[2]).astype(np.float32)
        assert ok, name
        assert np.all(np.abs(test_y - true_y) / N < 1e-6), name


# ---------------------------------------------------------------- test_losses.jl:14-31


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("loss,fn", [
    (srhip.L1DistLoss(), lambda x, y: np.abs(x - y)),
    (srhip.LPDistLoss(2.5), lambda x, y: np.abs(x - y) ** 2.5),  # customloss(x, y) = abs(x-y)^2.5
])
def test_losses(backend, loss, fn):
    """_loss / _weighted_loss vs a manual (weighted) mean; predictions are the
    tree x1 so the loss sees exactly x (test_losses.jl:245-253)."""
    o = srhip.Options(binary_operators=["+", "*", "-", "/"], unary_operators=["cos", "exp"],
                      elementwise_loss=loss)
    x = np.random.default_rng(0).standard_normal(100).astype(np.float32)
    y = np.random.default_rng(1).standard_normal(100).astype(np.float32)
    w = np.abs(np.random.default_rng(2).standard_normal(100)).astype(np.float32)
    tree = Node("x1")
    ds = srhip.Dataset(x[None, :], y)
    dsw = srhip.Dataset(x[None, :], y, weights=w)
    xd, yd, wd = x.astype(np.float64), y.astype(np.float64), w.astype(np.float64)
    assert abs(backend.eval_loss(tree, ds, o) - np.sum(fn(xd, yd)) / 100) < 1e-6
    assert abs(backend.eval_loss(tree, dsw, o) - np.sum(fn(xd, yd) * wd) / np.sum(wd)) < 1e-6


# ---------------------------------------------------------------- test_tree_construction.jl:10-116

UNAOPS = ["cos", "exp", "safe_log", "safe_log2", "safe_log10", "safe_sqrt", "relu", "gamma", "safe_acosh"]
NUMPY_U = {"cos": np.cos, "exp": np.exp, "safe_log": np.log, "safe_log2": np.log2, "safe_log10": np.log10,
           "safe_sqrt": np.sqrt, "relu": lambda v: (v + np.abs(v)) / 2, "safe_acosh": np.arccosh,
           "gamma": np.vectorize(math.gamma)}


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("unaop", UNAOPS)
@pytest.mark.parametrize("T", [np.float32, np.float64])
def test_tree_construction(backend, unaop, T):
    o = srhip.Options(binary_operators=["+", "*", "^", "/", "-"], unary_operators=[unaop, "abs"],
                      npopulations=4)
    o0 = srhip.Options(binary_operators=["+", "*", "^", "/", "-"], unary_operators=[unaop, "abs"], parsimony=0.0)
    o1 = srhip.Options(binary_operators=["+", "*", "^", "/", "-"], unary_operators=[unaop, "abs"], parsimony=1.0)
    # const_tree = sub(safe_pow(abs(3.0 * unaop(x1)), 2.0), -1.2)
    inner = Node(2, Node(2, Node(val=T(3.0)), Node(1, Node("x1"))))
    tree = Node(5, Node(3, inner, Node(val=T(2.0))), Node(val=T(-1.2)))
    inner_b = Node(2, Node(2, Node(val=T(3.0)), Node(1, Node("x1"))))
    tree_bad = Node(5, Node(3, inner_b, Node(val=T(2.1))), Node(val=T(-1.3)))
    assert srhip.count_nodes(tree) == 9
    N = 100
    rng = np.random.default_rng(0)
    if unaop in ("safe_log", "safe_log2", "safe_log10", "safe_acosh", "safe_sqrt"):
        X = (rng.random((5, N)) / 3).astype(T)
    else:
        X = (rng.standard_normal((5, N)) / 3).astype(T)
    X = X + np.sign(X) * T(0.1)
    if unaop == "safe_acosh":
        X = X + T(1.0)
    x = X[0].astype(np.float64)
    y = (np.abs(3.0 * NUMPY_U[unaop](x)) ** 2.0 - (-1.2)).astype(T)
    tol = 3e-2 if unaop == "gamma" else 1e-6
    dataset = srhip.Dataset(X, y)
    test_y, complete = backend.eval_tree_array(tree, X, o)
    assert complete
    assert np.all(np.abs(test_y.astype(np.float64) - y) / N < tol)
    l = backend.eval_loss(tree, dataset, o)
    assert abs(l) < tol
    assert l == backend.score_func(dataset, tree, o)[1]
    assert abs(backend.score_func(dataset, tree, o0)[0]) < tol
    assert backend.score_func(dataset, tree, o1)[0] > 1.0
    assert backend.score_func(dataset, tree, o)[0] < backend.score_func(dataset, tree_bad, o)[0]
    big = srhip.Dataset(X, y)
    big.baseline_loss = T(10)
    assert backend.score_func(big, tree_bad, o)[0] < backend.score_func(dataset, tree_bad, o)[0]
