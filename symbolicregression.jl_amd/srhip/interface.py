"""The reference's scoring surface, evaluated on the MI355X engine.

Single-tree functions keep the reference signatures
  eval_tree_array(tree, X, options)        src/InterfaceDynamicExpressions.jl:50-52
  eval_loss(tree, dataset, options)        src/LossFunctions.jl:60-67
  score_func(dataset, tree, options)       src/LossFunctions.jl:86-92
  score_func_batch(dataset, tree, options) src/LossFunctions.jl:95-115
  update_baseline_loss_(dataset, options)  src/LossFunctions.jl:122-126
  loss_to_score(loss, baseline, tree, options)  src/LossFunctions.jl:70-83
  compute_complexity(tree, options)        src/Complexity.jl:13-40
and each has a batched form over a list of trees (one device launch), which
is what the search's callers are meant to use.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple, Union

import numpy as np

from .dataset import Dataset
from .engine import DeviceDataset, Program, get_context
from .node import Node, count_nodes, flatten
from .options import Options

TreeOrTrees = Union[Node, Sequence[Node]]


def _as_list(trees: TreeOrTrees) -> Tuple[List[Node], bool]:
    if isinstance(trees, Node):
        return [trees], True
    return list(trees), False


def compile_trees(trees: Sequence[Node], options: Options, dtype, device: Optional[int] = None) -> Program:
    """Flatten + compile + upload a batch of trees (srhip_program_create)."""
    ctx = get_context(device)
    return Program(ctx, flatten(trees, options, dtype=dtype), dtype)


# ---- eval_tree_array ----------------------------------------------------------------
def eval_tree_array(tree: TreeOrTrees, X: np.ndarray, options: Options, device: Optional[int] = None):
    """(output, did_succeed). X is (nfeatures, n). For a list of trees the
    outputs are (ntrees, n) and did_succeed is a bool array. On failure the
    output rows are unspecified (the reference returns an undef array)."""
    trees, single = _as_list(tree)
    X = np.asarray(X)
    T = X.dtype if X.dtype in (np.float32, np.float64) else np.dtype(np.float64)
    ctx = get_context(device)
    ds = DeviceDataset(ctx, X.astype(T, copy=False), np.zeros(X.shape[1], dtype=T))
    prog = Program(ctx, flatten(trees, options, dtype=T), T)
    out, ok = prog.eval_tree_array(ds)
    if single:
        return out[0], bool(ok[0])
    return out, ok


def _seed_features(tree: Node, plus: int, direction: Optional[int]):
    """Copy of `tree` where every feature leaf x_f (only f == direction, when
    given) becomes (x_f + c) with a new constant c = -0.0. x + (-0.0) == x for
    every x (including ±0, ±Inf, NaN), so values and did_succeed are those of
    the original tree, and ∂ŷ/∂x_f = Σ over the seeds of x_f of ∂ŷ/∂c.
    Returns the copy and, per constant in get_constants order, the feature it
    seeds (0 for the tree's own constants)."""
    def rec(t: Node) -> Node:
        if t.degree == 0:
            if t.constant or (direction is not None and t.feature != direction):
                return t.copy()
            return Node(plus, Node(feature=t.feature), Node(val=-0.0))
        if t.degree == 1:
            return Node(t.op, rec(t.l))
        return Node(t.op, rec(t.l), rec(t.r))

    aug = rec(tree)
    seeds: List[int] = []
    _mark(aug, tree, seeds)
    return aug, seeds


def _mark(aug: Node, orig: Node, seeds: List[int]) -> None:
    """Walk `aug` and the original tree together in post-order and list, per
    constant of `aug`, the feature it seeds (0 = an original constant)."""
    if orig.degree == 0:
        if orig.constant:
            seeds.append(0)
        elif aug.degree == 2:  # seeded feature leaf: (x_f + c)
            seeds.append(orig.feature)
        return
    _mark(aug.l, orig.l, seeds)
    if orig.degree == 2:
        _mark(aug.r, orig.r, seeds)


def _feature_grads(trees: List[Node], X: np.ndarray, options: Options, direction: Optional[int],
                   device: Optional[int]):
    """(ŷ (ntrees, n), per tree ∂ŷ/∂x (nfeat, n) or, with direction, (n,), ok)."""
    T = X.dtype if X.dtype in (np.float32, np.float64) else np.dtype(np.float64)
    X = X.astype(T, copy=False)
    nfeat, n = X.shape
    if direction is not None and not 1 <= direction <= nfeat:
        raise ValueError("direction must be a 1-based feature index")
    binops = tuple(options.binary_operators)
    if "+" in binops:
        o, plus = options, binops.index("+") + 1
    else:  # same operator indices, "+" appended for the seeds
        o = Options(binary_operators=binops + ("+",), unary_operators=options.unary_operators)
        plus = len(binops) + 1
    augs, seeds = zip(*[_seed_features(t, plus, direction) for t in trees]) if trees else ((), ())
    ctx = get_context(device)
    ds = DeviceDataset(ctx, X, np.zeros(n, dtype=T))
    prog = Program(ctx, flatten(list(augs), o, dtype=T), T)
    val, grad, ok = prog.eval_grad_tree_array(ds)
    co = prog.flat.const_off
    out = []
    for t, sd in enumerate(seeds):
        g = grad[co[t]:co[t + 1]]
        sd = np.asarray(sd, dtype=np.int64)
        if direction is not None:
            d = g[sd == direction].sum(axis=0, dtype=T) if (sd == direction).any() else np.zeros(n, dtype=T)
            out.append(d.astype(T))
        else:
            G = np.zeros((nfeat, n), dtype=T)
            for f in np.unique(sd[sd > 0]):
                G[f - 1] = g[sd == f].sum(axis=0, dtype=T)
            out.append(G)
    return val, out, ok


def eval_diff_tree_array(tree: TreeOrTrees, X: np.ndarray, options: Options, direction: int,
                         device: Optional[int] = None):
    """eval_diff_tree_array(tree, X, options, direction)
    (src/InterfaceDynamicExpressions.jl:55-80): (output, ∂output/∂x_direction,
    complete), forward mode on the engine (seeded-feature tangents)."""
    trees, single = _as_list(tree)
    val, d, ok = _feature_grads(trees, np.asarray(X), options, int(direction), device)
    if single:
        return val[0], d[0], bool(ok[0])
    return val, d, ok


def eval_grad_tree_array(tree: TreeOrTrees, X: np.ndarray, options: Options, variable: bool = False,
                         device: Optional[int] = None):
    """eval_grad_tree_array(tree, X, options; variable=false)
    (src/InterfaceDynamicExpressions.jl:83-107): (output, gradient, complete)
    with gradient[k, i] = ∂ŷ_i/∂c_k for the tree's constants in get_constants
    order, or with variable=true gradient[f, i] = ∂ŷ_i/∂x_f (nfeatures × n).
    For a list of trees: outputs (ntrees, n), a list of per-tree gradient
    matrices, and a bool array."""
    trees, single = _as_list(tree)
    X = np.asarray(X)
    if variable:
        val, grads, ok = _feature_grads(trees, X, options, None, device)
        if single:
            return val[0], grads[0], bool(ok[0])
        return val, grads, ok
    T = X.dtype if X.dtype in (np.float32, np.float64) else np.dtype(np.float64)
    ctx = get_context(device)
    ds = DeviceDataset(ctx, X.astype(T, copy=False), np.zeros(X.shape[1], dtype=T))
    prog = Program(ctx, flatten(trees, options, dtype=T), T)
    val, grad, ok = prog.eval_grad_tree_array(ds)
    co = prog.flat.const_off
    grads = [grad[co[t]:co[t + 1]] for t in range(len(trees))]
    if single:
        return val[0], grads[0], bool(ok[0])
    return val, grads, ok


def eval_loss_grad_batch(trees: Sequence[Node], dataset: Dataset, options: Options,
                         device: Optional[int] = None):
    """Batched loss + constant gradients for ConstantOptimization
    (src/ConstantOptimization.jl:12-65): per tree (loss in T, ∂loss/∂c as a
    float64 vector in get_constants order, did_succeed)."""
    dev = dataset.device(device)
    prog = compile_trees(trees, options, dataset.T, dev.ctx.device)
    loss = options.elementwise_loss
    sums, grads, wsum, ok = prog.eval_loss_grad(dev, loss.kind, loss.params)
    T = dataset.T
    with np.errstate(invalid="ignore", divide="ignore"):
        losses = (sums / wsum).astype(T)
    losses[~ok] = T(np.inf)
    co = prog.flat.const_off
    g = [grads[co[t]:co[t + 1]] / wsum for t in range(len(trees))]
    return losses, g, ok


# ---- losses -------------------------------------------------------------------------
def eval_loss_batch(trees: Sequence[Node], dataset: Dataset, options: Options,
                    row_idx: Optional[np.ndarray] = None, device: Optional[int] = None,
                    program: Optional[Program] = None) -> np.ndarray:
    """eval_loss for many trees in one launch: the reference's `_eval_loss`
    value in T per tree (T(Inf) where the evaluation fails)."""
    return eval_loss_batch_ok(trees, dataset, options, row_idx, device, program)[0]


def eval_loss_batch_ok(trees: Sequence[Node], dataset: Dataset, options: Options,
                       row_idx: Optional[np.ndarray] = None, device: Optional[int] = None,
                       program: Optional[Program] = None) -> Tuple[np.ndarray, np.ndarray]:
    """(losses in T, did_succeed per tree)."""
    if options.loss_function is not None:
        f = options.loss_function
        vals = np.asarray([f(t, dataset, options) for t in trees], dtype=dataset.T)
        return vals, np.isfinite(vals)
    dev = dataset.device(device)
    prog = program if program is not None else compile_trees(trees, options, dataset.T, dev.ctx.device)
    loss = options.elementwise_loss
    sums, wsum, ok = prog.eval_loss(dev, loss.kind, loss.params, row_idx)
    T = dataset.T
    with np.errstate(invalid="ignore", divide="ignore"):
        out = (sums / wsum).astype(T)
    out[~ok] = T(np.inf)
    return out, ok


def eval_loss_batch_rowsets(trees: Sequence[Node], dataset: Dataset, options: Options,
                            rows: Sequence[np.ndarray], device: Optional[int] = None
                            ) -> Tuple[np.ndarray, np.ndarray]:
    """score_func_batch's evaluation for many trees, tree t on its OWN row
    sample rows[t] (with replacement, LossFunctions.jl:95-115; the reference
    draws one sample per call, :98): (losses in T, did_succeed). One engine
    launch for all trees (srhip_eval_loss_rowsets) when the samples have one
    length (the reference's batch_size); one per distinct length otherwise.
    score_func_batch uses options.elementwise_loss even when loss_function is
    set (:101-111), and so does this."""
    T = dataset.T
    n = len(trees)
    losses = np.zeros(n, dtype=T)
    ok = np.zeros(n, dtype=bool)
    if n == 0:
        return losses, ok
    rows = [np.asarray(r, dtype=np.int64) for r in rows]
    if len(rows) != n:
        raise ValueError("one row sample per tree")
    dev = dataset.device(device)
    loss = options.elementwise_loss
    by_len = {}
    for t, r in enumerate(rows):
        by_len.setdefault(len(r), []).append(t)
    for bs, idx in by_len.items():
        sub = [trees[t] for t in idx]
        prog = Program(dev.ctx, flatten(sub, options, dtype=T), T, interpreted=True)
        R = np.stack([rows[t] for t in idx]) if bs else np.zeros((len(idx), 0), dtype=np.int64)
        sums, wsum, k = prog.eval_loss_rowsets(dev, loss.kind, R, loss.params)
        with np.errstate(invalid="ignore", divide="ignore"):
            lv = (sums / wsum).astype(T)
        lv[~k] = T(np.inf)
        losses[idx] = lv
        ok[idx] = k
    return losses, ok


def eval_loss(tree: Node, dataset: Dataset, options: Options) -> float:
    return eval_loss_batch([tree], dataset, options)[0]


def compute_complexity(tree: Node, options: Options) -> int:
    if not options.complexity_use:
        return count_nodes(tree)

    def rec(t: Node) -> float:
        if t.degree == 0:
            return options.constant_complexity if t.constant else options.variable_complexity
        if t.degree == 1:
            return options.unaop_complexities[t.op - 1] + rec(t.l)
        return options.binop_complexities[t.op - 1] + rec(t.l) + rec(t.r)

    return int(round(rec(tree)))


def loss_to_score(loss, baseline, tree: Node, options: Options):
    """LossFunctions.jl:69-82 in T; the parsimony term is Int × Float32
    (options.parsimony is a Float32 field, Options.jl:327)."""
    T = type(loss) if isinstance(loss, np.floating) else np.float64
    normalization = T(0.01) if baseline < T(0.01) else T(baseline)
    term = np.float32(compute_complexity(tree, options)) * np.float32(options.parsimony)
    with np.errstate(all="ignore"):
        return T(T(loss / normalization) + T(term))


def score_func_batched(dataset: Dataset, trees: Sequence[Node], options: Options,
                       device: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray]:
    """score_func over many trees: (scores, losses)."""
    losses = eval_loss_batch(trees, dataset, options, device=device)
    scores = np.asarray([loss_to_score(l, dataset.baseline_loss, t, options) for l, t in zip(losses, trees)],
                        dtype=dataset.T)
    return scores, losses


def score_func(dataset: Dataset, tree: Node, options: Options):
    s, l = score_func_batched(dataset, [tree], options)
    return s[0], l[0]


def score_func_batch(dataset: Dataset, tree: TreeOrTrees, options: Options,
                     rng: Optional[np.random.Generator] = None, row_idx: Optional[np.ndarray] = None):
    """Minibatch score (src/LossFunctions.jl:95-115): batch_size rows sampled
    with replacement; a failed evaluation scores (0, Inf) as in the reference."""
    trees, single = _as_list(tree)
    if row_idx is None:
        rng = rng or np.random.default_rng()
        row_idx = rng.integers(0, dataset.n, size=options.batch_size)
    losses, ok = eval_loss_batch_ok(trees, dataset, options, row_idx=row_idx)
    T = dataset.T
    scores = np.asarray(
        [loss_to_score(l, dataset.baseline_loss, t, options) if k else T(0)
         for l, t, k in zip(losses, trees, ok)],
        dtype=T,
    )
    if single:
        return scores[0], losses[0]
    return scores, losses


def update_baseline_loss_(dataset: Dataset, options: Options) -> None:
    """update_baseline_loss!: loss of the constant tree avg_y."""
    dataset.baseline_loss = eval_loss(Node(val=dataset.avg_y), dataset, options)
