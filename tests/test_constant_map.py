"""The host side of srhip_program_set_constants (api.cpp patch_image), no
device needed: new constants written through the constant map must give
every tree the instruction stream and static verdict a fresh compile of the
new constants gives (compile.cpp, the reference's `_eval_constant_tree`
folding, src/InterfaceDynamicExpressions.jl eval_tree_array). Trees whose
immediates are their constants or folded subtrees of them are patched with no
recompile; non-finite values recompile just their trees."""
import numpy as np
import pytest

import srhip
from srhip.engine import debug_constant_map

OPS = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])


def _flat(n, T, seed):
    """n random trees, without those that fail statically for their own
    constants (they have no code: new constants that make them compile need
    a new layout, which set_constants handles by a rebuild)"""
    trees = srhip.random_population(n, OPS, 5, T, seed=seed)
    keep = []
    for t in trees:
        f = srhip.flatten([t], OPS, dtype=T)
        # patched in place with no recompile when its constants move by an ulp:
        # it has code (a failing tree is recompiled at every change; with the
        # same constants it is skipped, so the same constants cannot tell)
        nudged = np.nextafter(np.asarray(f.consts, dtype=T), T(np.inf))
        if debug_constant_map(f, nudged, T)[1] == 0:
            keep.append(t)
    assert len(keep) > 0.8 * n
    return srhip.flatten(keep, OPS, dtype=T)


@pytest.mark.parametrize("T", [np.float32, np.float64])
@pytest.mark.parametrize("grad", [False, True])
def test_scaled_constants_patch_without_recompile(T, grad):
    flat = _flat(3000, T, 21)
    c = np.asarray(flat.consts, dtype=T)
    for k, new in enumerate((c * T(1.01), c + T(0.25), -c)):
        mismatch, recompiled, relayout = debug_constant_map(flat, new, T, grad)
        assert relayout == 0 and mismatch == 0, (k, mismatch, relayout)
        assert recompiled <= 0.02 * flat.ntrees, (k, recompiled)  # only folds that newly overflow


@pytest.mark.parametrize("grad", [False, True])
def test_folded_subtrees_are_re_evaluated(grad):
    """exp(c1 * c2)-style folds: new values move the folded immediate; a fold
    that overflows makes its tree fail statically (recompiled, old code kept)."""
    B, U = OPS.make_binary, OPS.make_unary

    def x():
        return srhip.Node(feature=1)

    def c(v):
        return srhip.Node(val=v)

    trees = [B("+", B("*", x(), U("exp", B("*", c(0.5), c(2.0)))), c(3.0)),
             B("/", U("cos", B("-", c(0.5), c(2.0))), x()),
             B("+", x(), c(0.5))]
    T = np.float32
    flat = srhip.flatten(trees, OPS, dtype=T)
    c0 = np.asarray(flat.consts, dtype=T)
    assert debug_constant_map(flat, c0 * T(1.5), T, grad)[:2] == (0, 0)
    big = c0.copy()
    big[0] = T(1e30)  # exp(1e30 * 2) overflows: tree 0 fails statically
    mismatch, recompiled, relayout = debug_constant_map(flat, big, T, grad)
    # gradient programs fold nothing: a large finite constant is just written
    assert mismatch == 0 and relayout == 0 and recompiled == (0 if grad else 1)


@pytest.mark.parametrize("T", [np.float32, np.float64])
def test_non_finite_constants(T):
    flat = _flat(2000, T, 22)
    c = np.asarray(flat.consts, dtype=T)
    rng = np.random.default_rng(3)
    new = c.copy()
    hit = rng.choice(len(c), size=len(c) // 10, replace=False)
    new[hit[: len(hit) // 2]] = np.inf
    new[hit[len(hit) // 2:]] = np.nan
    for grad in (False, True):
        mismatch, recompiled, relayout = debug_constant_map(flat, new, T, grad)
        assert relayout == 0 and mismatch == 0 and recompiled > 0
    # and back to finite values: the failing trees' kept code is patched again
    mismatch, recompiled, relayout = debug_constant_map(flat, c * T(0.9), T, False)
    assert relayout == 0 and mismatch == 0


@pytest.mark.parametrize("T", [np.float32, np.float64])
@pytest.mark.parametrize("grad", [False, True])
def test_keep_layout_failing_trees_patch_back(T, grad):
    """Programs whose constants change (the optimiser's, compile_batch
    keep_layout): a tree that fails statically for its constants (a folded
    overflow, a NaN constant) keeps its code, so constants that make it
    finite again are patched in place — no rebuild, no recompile: the verdict
    follows from the patched immediates — and every tree matches a fresh
    compile (instruction stream and verdict)."""
    trees = srhip.random_population(1500, OPS, 5, T, seed=23)
    flat = srhip.flatten(trees, OPS, dtype=T)
    c0 = np.asarray(flat.consts, dtype=T)
    rng = np.random.default_rng(24)
    bad = c0.copy()
    bad[rng.choice(len(c0), len(c0) // 8, replace=False)] = T(1e30)
    bad[rng.choice(len(c0), len(c0) // 20, replace=False)] = T(np.nan)
    failing = srhip.node.FlatTrees(flat.node_off, flat.kind, flat.arg, flat.const_off, bad, flat.nodes)
    # compiled with the failing constants, patched back to finite ones
    mismatch, recompiled, relayout = debug_constant_map(failing, c0, T, grad, keep_layout=True)
    assert relayout == 0 and mismatch == 0, (mismatch, relayout)
    assert recompiled == 0  # verdicts decided from the patched immediates, no compile
    # and the other way
    mismatch, _, relayout = debug_constant_map(flat, bad, T, grad, keep_layout=True)
    assert relayout == 0 and mismatch == 0, (mismatch, relayout)
    # the same failing constants again: nothing to recompile
    assert debug_constant_map(failing, bad, T, grad, keep_layout=True)[:3] == (0, 0, 0)
    # without keep_layout the first direction needs a rebuild (the failing trees have no code)
    assert debug_constant_map(failing, c0, T, grad)[2] == 1


@pytest.mark.parametrize("grad", [False, True])
def test_keep_layout_verdicts_with_nan_absorbing_operators(grad):
    """max / min fold a NaN operand away (fmax): a NaN constant inside a folded
    subtree need not fail the tree, one in an operand does — the in-place
    verdicts match a fresh compile's either way."""
    ops = srhip.Options(binary_operators=["+", "*", "max", "min"], unary_operators=["exp", "cos"])
    T = np.float32
    trees = srhip.random_population(1200, ops, 4, T, seed=25)
    flat = srhip.flatten(trees, ops, dtype=T)
    c0 = np.asarray(flat.consts, dtype=T)
    rng = np.random.default_rng(26)
    bad = c0.copy()
    bad[rng.choice(len(c0), len(c0) // 6, replace=False)] = T(np.nan)
    bad[rng.choice(len(c0), len(c0) // 10, replace=False)] = T(1e30)
    failing = srhip.node.FlatTrees(flat.node_off, flat.kind, flat.arg, flat.const_off, bad, flat.nodes)
    for src, new in ((failing, c0), (flat, bad)):
        mismatch, recompiled, relayout = debug_constant_map(src, new, T, grad, keep_layout=True)
        assert (mismatch, relayout) == (0, 0)
