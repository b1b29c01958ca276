"""The threaded interpreter (gen_asm_interp.py) against the C++ dispatch.

Both paths run the same operator code (the handler bodies are compiled from
device_ops.h), so per-row outputs, did_succeed and loss sums must be
bit-identical. SRHIP_TI=0 switches the engine to the C++ dispatch for one call
(api.cpp reads it per launch). The oracle comparisons of test_gpu_parity.py
and test_golden.py already run through the threaded path (it is the default).
"""
import os

import numpy as np
import pytest

import srhip
from srhip import Node
from srhip import constants as K

ALL_BIN = ["+", "-", "*", "/", "^", "greater", "logical_or", "logical_and", "mod", "max", "min"]
ALL_UNA = [n for n in K.OP_NAMES if K.OP_NAMES[n][0] == 1 and not n.startswith("safe_")]


def both_paths(fn):
    old = os.environ.get("SRHIP_TI")
    try:
        os.environ["SRHIP_TI"] = "1"
        a = fn()
        os.environ["SRHIP_TI"] = "0"
        b = fn()
    finally:
        if old is None:
            os.environ.pop("SRHIP_TI", None)
        else:
            os.environ["SRHIP_TI"] = old
    return a, b


def same_bits(a, b):
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


def data(n, nfeat=5, seed=0, scale=2.0):
    rng = np.random.default_rng(seed)
    X = (scale * rng.standard_normal((nfeat, n))).astype(np.float32)
    y = (np.cos(X[min(3, nfeat - 1)]) * 2 + X[0] ** 2 - 2).astype(np.float32)
    return X, y


@pytest.mark.gpu
@pytest.mark.parametrize("ops,n", [
    ((["+", "-", "*", "/"], ["cos", "exp"]), 3000),
    ((ALL_BIN, ALL_UNA), 2500),
    ((["+", "*", "/"], ["sin", "tanh", "log", "sqrt", "atan", "erf"]), 70000),
])
def test_outputs_bitwise_equal(gpu_ctx, ops, n):
    o = srhip.Options(binary_operators=ops[0], unary_operators=ops[1])
    trees = srhip.random_population(600, o, 5, np.float32, seed=n)
    X, _ = data(n, seed=n)
    (out_t, ok_t), (out_c, ok_c) = both_paths(lambda: srhip.eval_tree_array(trees, X, o))
    assert np.array_equal(ok_t, ok_c)
    for t in np.flatnonzero(ok_t):
        assert same_bits(out_t[t], out_c[t]), srhip.string_tree(trees[t], o)


@pytest.mark.gpu
@pytest.mark.parametrize("weighted", [False, True])
def test_losses_bitwise_equal(gpu_ctx, weighted):
    X, y = data(40000, seed=4)
    w = np.random.default_rng(5).uniform(0.5, 2.0, 40000).astype(np.float32) if weighted else None
    ds = srhip.Dataset(X, y, weights=w)
    for loss in (srhip.L2DistLoss(), srhip.L1DistLoss(), srhip.HuberLoss(0.5)):
        o = srhip.Options(binary_operators=ALL_BIN, unary_operators=ALL_UNA, elementwise_loss=loss)
        trees = srhip.random_population(1500, o, 5, np.float32, seed=3)
        (l_t, ok_t), (l_c, ok_c) = both_paths(lambda: srhip.eval_loss_batch_ok(trees, ds, o))
        assert np.array_equal(ok_t, ok_c), loss
        assert np.array_equal(l_t[ok_t], l_c[ok_c]), loss


@pytest.mark.gpu
def test_trig_fallback_and_extreme_arguments(gpu_ctx):
    """sin/cos of |x| > 105615 leave the fast path (the block bails, the C++
    interpreter redoes the tile); Inf/NaN arguments fail the tree."""
    o = srhip.Options(binary_operators=["*", "+"], unary_operators=["cos", "sin", "exp"])
    MUL, ADD, COS, SIN, EXP = 1, 2, 1, 2, 3
    x1 = Node("x1")
    trees = [Node(COS, Node(MUL, x1, Node(val=1e6))), Node(SIN, Node(MUL, x1, Node(val=3e5))),
             Node(COS, Node(EXP, Node(MUL, x1, Node(val=50.0)))), Node(SIN, x1),
             Node(ADD, Node(COS, Node(MUL, x1, Node(val=2e5))), Node(SIN, x1))]
    X = np.linspace(-3, 3, 5000, dtype=np.float32)[None, :]
    (out_t, ok_t), (out_c, ok_c) = both_paths(lambda: srhip.eval_tree_array(trees, X, o))
    assert np.array_equal(ok_t, ok_c)
    for t in np.flatnonzero(ok_t):
        assert same_bits(out_t[t], out_c[t]), t
    assert ok_t[0] and ok_t[1] and ok_t[3]


@pytest.mark.gpu
def test_every_opcode_and_operand_variant(gpu_ctx):
    """One tree per (binary op, operand sources): leaf/leaf, leaf/const,
    const/leaf, subtree/leaf, leaf/subtree, subtree/const, const/subtree,
    subtree/subtree (push/pop), plus every unary operator."""
    o = srhip.Options(binary_operators=ALL_BIN, unary_operators=ALL_UNA)
    x1, x2, x3 = Node("x1"), Node("x2"), Node("x3")
    trees = []
    for b in range(1, len(ALL_BIN) + 1):
        sub = Node(1, x1, x3)  # x1 + x3 (a computed operand)
        sub2 = Node(3, x2, Node(val=0.75))  # x2 * 0.75
        for lhs, rhs in [(x1, x2), (x1, Node(val=1.5)), (Node(val=-2.25), x2), (sub, x2), (x2, sub),
                         (sub, Node(val=0.5)), (Node(val=3.0), sub), (sub, sub2), (sub2, sub)]:
            trees.append(Node(b, lhs, rhs))
    for u in range(1, len(ALL_UNA) + 1):
        trees.append(Node(u, Node(1, x1, Node(val=0.25))))
    X, _ = data(3000, nfeat=3, seed=11, scale=1.5)
    (out_t, ok_t), (out_c, ok_c) = both_paths(lambda: srhip.eval_tree_array(trees, X, o))
    assert np.array_equal(ok_t, ok_c)
    for t in np.flatnonzero(ok_t):
        assert same_bits(out_t[t], out_c[t]), srhip.string_tree(trees[t], o)


@pytest.mark.gpu
def test_long_programs(gpu_ctx):
    """Programs near the 63-instruction limit of the threaded block (records
    0..63 of a list slot) and trees beyond it (C++ path)."""
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "neg"])
    trees = srhip.random_population(300, o, 5, np.float32, seed=21, maxsize=70)
    X, _ = data(9000, seed=22)
    (out_t, ok_t), (out_c, ok_c) = both_paths(lambda: srhip.eval_tree_array(trees, X, o))
    assert np.array_equal(ok_t, ok_c)
    for t in np.flatnonzero(ok_t):
        assert same_bits(out_t[t], out_c[t]), t
