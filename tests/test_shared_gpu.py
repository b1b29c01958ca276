"""Shared subtrees of the Float32 tree code (jit.h Columns::gkey, round 6).

A constant-free subtree that several trees of a batch contain (cos(x4),
exp(cos(x1)), x1 / x3, ...) is evaluated once per row per call by the derive
pass (kernels.hip derive_columns_kernel: the interpreter's operators, NaN on a
row where any node of it is non-finite) and read by the tree code with one
global load per tile. Checks, on batches where the columns are in use:
did_succeed identical to the oracle and to the same program built without
shared columns (SRHIP_JIT_GCOLS=0), losses within 1e-5 of the oracle beyond
the conditioned spread of tests/numerics.py, and shared subtrees that fail
(overflow, 0/0) failing exactly the trees the oracle fails.
Reference: DynamicExpressions' eval_tree_array contract,
/root/reference/src/InterfaceDynamicExpressions.jl:17-52 (a node with a
non-finite value on any row fails the tree), LossFunctions.jl:34-50.
"""
import os

import numpy as np
import pytest

import oracle
import srhip
from numerics import assert_close_conditioned, loss_spread
from srhip import Node

pytestmark = pytest.mark.gpu
F32_OPS = (["+", "-", "*", "/"], ["cos", "exp"])


def program(dev, trees, o, gcols=None):
    old = os.environ.get("SRHIP_JIT_GCOLS")
    try:
        if gcols is not None:
            os.environ["SRHIP_JIT_GCOLS"] = str(gcols)
        return srhip.engine.Program(dev.ctx, srhip.flatten(trees, o, dtype=np.float32), np.float32)
    finally:
        if gcols is not None:
            if old is None:
                del os.environ["SRHIP_JIT_GCOLS"]
            else:
                os.environ["SRHIP_JIT_GCOLS"] = old


def check_batch(trees, o, X, y, w=None, rtol=1e-5):
    ds = srhip.Dataset(X, y, weights=w)
    dev = ds.device()
    p_on = program(dev, trees, o)
    p_off = program(dev, trees, o, gcols=0)
    assert p_on.jit_info()["ntrees"] > 0
    s1, w1, k1 = p_on.eval_loss(dev, 0)
    assert dev.ctx.last_tree_code() > 0
    s0, w0, k0 = p_off.eval_loss(dev, 0)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    _, rl, rok = oracle.eval_loss_batch(flat, X, y, w, dtype=np.float32)
    assert np.array_equal(k1, rok), f"did_succeed: {np.flatnonzero(k1 != rok)[:10]}"
    assert np.array_equal(k0, rok)
    m = k1 & np.isfinite(rl)
    sp = loss_spread(trees, o, X, y, w, np.float32) / w1
    l1 = (s1 / w1).astype(np.float32)
    assert_close_conditioned(l1[m], rl[m], sp[m], rtol=rtol, msg="shared columns vs oracle")
    return k1


def test_shared_columns_config2_like(gpu_ctx):
    o = srhip.Options(binary_operators=F32_OPS[0], unary_operators=F32_OPS[1])
    trees = srhip.random_population(1500, o, 5, np.float32, seed=1000, maxsize=30)
    rng = np.random.default_rng(1)
    X = rng.standard_normal((5, 40_000)).astype(np.float32)
    y = (2 * np.cos(X[3]) + X[0] * X[0] - 2).astype(np.float32)
    w = np.abs(rng.standard_normal(40_000)).astype(np.float32)
    check_batch(trees, o, X, y)
    check_batch(trees, o, X, y, w)


def test_shared_columns_that_fail(gpu_ctx):
    """Shared subtrees that overflow (exp(exp(x))) or divide 0 by 0 (x / x on a
    zero row) on some rows: every tree holding them fails, as in the oracle;
    a lossy consumer (exp(-exp(exp(x))) → 0) still fails."""
    o = srhip.Options(binary_operators=F32_OPS[0], unary_operators=F32_OPS[1])
    x1, x2 = Node(feature=1), Node(feature=2)
    ee = lambda: o.make_unary("exp", o.make_unary("exp", x1.copy()))  # noqa: E731
    dd = lambda: o.make_binary("/", x2.copy(), x2.copy())  # noqa: E731
    special = []
    for k in range(12):
        c = Node(val=0.5 + k)
        special.append(o.make_binary("+", ee(), c))
        special.append(o.make_binary("*", dd(), c.copy()))
        special.append(o.make_unary("exp", o.make_binary("-", Node(val=-1.0 - k), ee())))
    trees = special + srhip.random_population(500, o, 5, np.float32, seed=7, maxsize=30)
    rng = np.random.default_rng(2)
    X = rng.standard_normal((5, 20_000)).astype(np.float32)
    X[0, 123] = 4.0   # exp(exp(4)) = exp(54.6) ok; 5 overflows: exp(148)
    X[0, 777] = 5.0
    X[1, 999] = 0.0   # x2 / x2 = NaN there
    y = (2 * np.cos(X[3]) + X[0] * X[0] - 2).astype(np.float32)
    ok = check_batch(trees, o, X, y)
    assert not ok[:len(special)].any(), "every tree with a failing shared subtree fails"


def grad_eval(dev, trees, o, gcols=None):
    """A program's first eval_loss_grad (its gradient tree code is built
    there, reading SRHIP_GJIT_GCOLS) and the code's size."""
    from srhip import constants as K
    old = os.environ.get("SRHIP_GJIT_GCOLS")
    try:
        if gcols is not None:
            os.environ["SRHIP_GJIT_GCOLS"] = str(gcols)
        p = srhip.engine.Program(dev.ctx, srhip.flatten(trees, o, dtype=np.float32), np.float32)
        return p, p.eval_loss_grad(dev, K.LOSS["L2"])
    finally:
        if gcols is not None:
            if old is None:
                del os.environ["SRHIP_GJIT_GCOLS"]
            else:
                os.environ["SRHIP_GJIT_GCOLS"] = old


@pytest.mark.parametrize("weighted", [False, True])
def test_gradient_shared_columns_bit_identical(gpu_ctx, weighted):
    """The gradient tree code reading shared constant-free subtrees from
    columns (jit.h kGradGbase) gives the losses, ∂L/∂c and did_succeed of the
    same program built without them (SRHIP_GJIT_GCOLS=0) bit for bit: the
    columns hold the interpreter's values, which the gradient code's PRECISE
    forward equals; failing shared subtrees (exp(exp(x)) overflow, x / x at
    a zero) fail exactly the oracle's trees."""
    from srhip import constants as K
    o = srhip.Options(binary_operators=F32_OPS[0], unary_operators=F32_OPS[1])
    x1 = Node(feature=1)
    special = []
    for k in range(12):
        ee = o.make_unary("exp", o.make_unary("exp", x1.copy()))
        special.append(o.make_binary("*", ee, Node(val=0.5 + k)))
        dd = o.make_binary("/", Node(feature=2), Node(feature=2))
        special.append(o.make_binary("-", o.make_binary("*", dd, Node(val=1.0 + k)), Node(val=0.25)))
    trees = special + srhip.random_population(1500, o, 20, np.float32, seed=17, maxsize=30)
    rng = np.random.default_rng(3 + weighted)
    n = 20_001
    X = rng.standard_normal((20, n)).astype(np.float32)
    X[0, 777] = 5.0   # exp(exp(5)) overflows
    X[1, 999] = 0.0   # x2 / x2 = NaN there
    y = (2 * np.cos(X[3]) + X[0] * X[0] - 2).astype(np.float32)
    w = np.abs(rng.standard_normal(n)).astype(np.float32) if weighted else None
    ds = srhip.Dataset(X, y, weights=w)
    dev = ds.device()
    p_on, (s1, g1, w1, k1) = grad_eval(dev, trees, o)
    p_off, (s0, g0, w0, k0) = grad_eval(dev, trees, o, gcols=0)
    info_on, info_off = p_on.grad_jit_info(), p_off.grad_jit_info()
    assert info_on["ntrees"] >= 0.95 * len(trees) and info_on["ntrees"] == info_off["ntrees"]
    assert info_on["code_bytes"] != info_off["code_bytes"], "no shared columns in use"
    s2, g2, _, k2 = p_on.eval_loss_grad(dev, K.LOSS["L2"])  # again: the cached subtree program
    assert np.array_equal(k2, k1)
    np.testing.assert_array_equal(g2, g1)
    assert np.array_equal(k1, k0)
    assert not k1[:len(special)].any(), "every tree with a failing shared subtree fails"
    assert w1 == w0
    np.testing.assert_array_equal(s1[k1], s0[k0])
    ok_c = np.repeat(k1, np.diff(p_on.flat.const_off))
    np.testing.assert_array_equal(g1[ok_c], g0[ok_c])
    assert np.all(np.isnan(g1[~ok_c]))
    flat = srhip.flatten(trees, o, dtype=np.float32)
    _, _, rok = oracle.eval_loss_batch(flat, X, y, w, dtype=np.float32)
    assert np.array_equal(k1, rok)
