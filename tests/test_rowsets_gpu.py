"""Per-tree minibatches: srhip_eval_loss_rowsets (score_func_batch,
/root/reference/src/LossFunctions.jl:95-115, samples batch_size rows with
replacement PER CALL, :98 — i.e. per candidate, src/Mutate.jl:41-47, 199-205).

Every tree of one launch is scored on its own sample; the oracle evaluates
each tree alone on that sample (oracle.eval_loss_batch with row_idx).
Bars: did_succeed identical on every tree; losses within 1e-5 relative
(Float32; 1e-9 Float64) beyond the conditioned perturbation spread of
tests/numerics.py; and, with every tree given the same sample, the rowsets
launch equals the shared-sample path (srhip_eval_loss with row_idx) bit for
bit, since both sum each tree's rows in the same order.
"""
import numpy as np
import pytest

import oracle
import srhip
from numerics import assert_close_conditioned, loss_spread
from srhip import Node
L2 = 0  # SRHIP_LOSS_L2 (include/srhip.h)

pytestmark = pytest.mark.gpu

F32_OPS = (["+", "-", "*", "/"], ["cos", "exp"])
NAN_OPS = (["+", "-", "*", "/", "^"], ["safe_log", "safe_sqrt", "cos", "exp"])


def deep_tree(depth, rng):
    if depth == 0:
        return Node(feature=int(rng.integers(1, 4))) if rng.random() < 0.7 else Node(val=float(rng.standard_normal()))
    return Node(int(rng.integers(1, 4)), deep_tree(depth - 1, rng), deep_tree(depth - 1, rng))


def oracle_rowsets(trees, o, X, y, w, rows, T, loss=None):
    """Each tree alone on its own sample: (losses in T, ok)."""
    loss = loss or o.elementwise_loss
    out = np.zeros(len(trees), dtype=T)
    oks = np.zeros(len(trees), dtype=bool)
    for t, (tree, r) in enumerate(zip(trees, rows)):
        flat = srhip.flatten([tree], o, dtype=T)
        _, l, ok = oracle.eval_loss_batch(flat, X, y, w, loss.kind, loss.params, row_idx=r, dtype=T)
        out[t], oks[t] = l[0], ok[0]
    return out, oks


def spread_rowsets(trees, o, X, y, w, rows, T):
    sp = np.zeros(len(trees))
    for t, (tree, r) in enumerate(zip(trees, rows)):
        wv = None if w is None else w[r]
        sp[t] = loss_spread([tree], o, X[:, r], y[r], wv, T)[0] / (len(r) if wv is None else wv.sum())
    return sp


@pytest.mark.parametrize("T,ops,bs", [(np.float32, F32_OPS, 50), (np.float32, F32_OPS, 3000),
                                      (np.float64, NAN_OPS, 50), (np.float64, NAN_OPS, 700)])
def test_rowsets_match_oracle_tree_by_tree(gpu_ctx, T, ops, bs):
    o = srhip.Options(binary_operators=ops[0], unary_operators=ops[1], batching=True, batch_size=bs)
    rng = np.random.default_rng(41)
    trees = srhip.random_population(150, o, 5, T, seed=42)
    trees += [deep_tree(d, rng) for d in (6, 7, 8) for _ in range(3)]  # the deep interpreter pass too
    n = 5000
    if T == np.float32:
        X = rng.standard_normal((5, n)).astype(T)
        y = (2 * np.cos(X[3]) + X[0] * X[0] - 2).astype(T)
    else:
        X = rng.uniform(-3, 3, (5, n))  # mixed sign: safe_log / safe_sqrt / ^ fail on some rows
        y = 2 * np.cos(X[3]) + X[0] * X[0] - 2
    w = np.abs(rng.standard_normal(n)).astype(T)
    # distinct samples per tree, with repeated indices (with replacement)
    rows = [rng.integers(0, n, bs) for _ in trees]
    rows[0][:] = rows[0][0]  # one sample that is a single row repeated
    rows[1][: bs // 2] = rows[1][bs // 2:bs // 2 * 2]  # halves repeated
    rtol = 1e-5 if T == np.float32 else 1e-9
    for weights in (None, w):
        ds = srhip.Dataset(X, y, weights=weights)
        l, ok = srhip.eval_loss_batch_rowsets(trees, ds, o, rows)
        rl, rok = oracle_rowsets(trees, o, X, y, weights, rows, T)
        assert np.array_equal(ok, rok), "did_succeed differs from the oracle"
        assert 0 < ok.sum() < len(trees) or T == np.float32
        m = ok & np.isfinite(rl)
        sp = spread_rowsets([t for t, k in zip(trees, m) if k], o, X, y, weights,
                            [r for r, k in zip(rows, m) if k], T)
        assert_close_conditioned(l[m], rl[m], sp, rtol=rtol, msg=f"rowsets {T.__name__} bs={bs}")
        assert np.all(np.isinf(l[~ok]))


def test_rowsets_long_samples_multiple_row_groups(gpu_ctx):
    """batch_size above one segment of 8192 rows (segment = a multiple of 8192)."""
    o = srhip.Options(binary_operators=F32_OPS[0], unary_operators=F32_OPS[1])
    trees = srhip.random_population(40, o, 5, np.float32, seed=51)
    rng = np.random.default_rng(52)
    n = 30_000
    X = rng.standard_normal((5, n)).astype(np.float32)
    y = (2 * np.cos(X[3]) + X[0] * X[0] - 2).astype(np.float32)
    rows = [rng.integers(0, n, 10_000) for _ in trees]
    ds = srhip.Dataset(X, y)
    l, ok = srhip.eval_loss_batch_rowsets(trees, ds, o, rows)
    rl, rok = oracle_rowsets(trees, o, X, y, None, rows, np.float32)
    assert np.array_equal(ok, rok)
    m = ok & np.isfinite(rl)
    sp = spread_rowsets([t for t, k in zip(trees, m) if k], o, X, y, None, [r for r, k in zip(rows, m) if k],
                        np.float32)
    assert_close_conditioned(l[m], rl[m], sp, rtol=1e-5, msg="bs=10000")


@pytest.mark.parametrize("T", [np.float32, np.float64])
def test_rowsets_same_sample_equals_shared_row_idx_bit_for_bit(gpu_ctx, T):
    o = srhip.Options(binary_operators=F32_OPS[0], unary_operators=F32_OPS[1])
    trees = srhip.random_population(200, o, 5, T, seed=61)  # < 256: the shared path is interpreted too
    rng = np.random.default_rng(62)
    X = rng.standard_normal((5, 3000)).astype(T)
    y = (2 * np.cos(X[3]) + X[0] * X[0] - 2).astype(T)
    w = np.abs(rng.standard_normal(3000)).astype(T)
    idx = rng.integers(0, 3000, 333)
    for weights in (None, w):
        ds = srhip.Dataset(X, y, weights=weights)
        dev = ds.device()
        prog = srhip.engine.Program(dev.ctx, srhip.flatten(trees, o, dtype=T), T)
        s1, w1, k1 = prog.eval_loss(dev, L2, None, idx)
        s2, w2, k2 = prog.eval_loss_rowsets(dev, L2, np.tile(idx, (len(trees), 1)))
        assert np.array_equal(k1, k2)
        assert np.array_equal(s1[k1], s2[k2])
        assert np.all(w2 == w1)


def test_rowsets_on_a_tree_code_program_run_interpreted(gpu_ctx):
    """A program large enough for tree code scores its row sets in the
    interpreter (one tree per workgroup); the same trees' full-data losses
    still come from the tree code."""
    o = srhip.Options(binary_operators=F32_OPS[0], unary_operators=F32_OPS[1])
    trees = srhip.random_population(400, o, 5, np.float32, seed=71)
    rng = np.random.default_rng(72)
    n = 4000
    X = rng.standard_normal((5, n)).astype(np.float32)
    y = (2 * np.cos(X[3]) + X[0] * X[0] - 2).astype(np.float32)
    ds = srhip.Dataset(X, y)
    dev = ds.device()
    prog = srhip.engine.Program(dev.ctx, srhip.flatten(trees, o, dtype=np.float32), np.float32)
    assert prog.jit_info()["ntrees"] > 0
    rows = rng.integers(0, n, (len(trees), 64))
    s, ws, k = prog.eval_loss_rowsets(dev, L2, rows)
    assert dev.ctx.last_tree_code() == 0
    rl, rok = oracle_rowsets(trees, o, X, y, None, list(rows), np.float32)
    assert np.array_equal(k, rok)
    m = k & np.isfinite(rl)
    sp = spread_rowsets([t for t, q in zip(trees, m) if q], o, X, y, None, [r for r, q in zip(rows, m) if q],
                        np.float32)
    assert_close_conditioned((s / ws).astype(np.float32)[m], rl[m], sp, rtol=1e-5, msg="rowsets on tree-code program")
    # and the batched convenience makes no tree code at all
    l2, k2 = srhip.eval_loss_batch_rowsets(trees, ds, o, list(rows))
    assert np.array_equal(k2, k)


def test_rowsets_edge_cases(gpu_ctx):
    o = srhip.Options(binary_operators=F32_OPS[0], unary_operators=F32_OPS[1])
    X = np.random.default_rng(81).standard_normal((5, 100)).astype(np.float32)
    y = X[0].copy()
    ds = srhip.Dataset(X, y)
    dev = ds.device()
    trees = [Node(feature=1), Node(val=np.inf), Node(1, Node(feature=2), Node(val=1.5))]
    prog = srhip.engine.Program(dev.ctx, srhip.flatten(trees, o, dtype=np.float32), np.float32)
    # a constant-Inf tree fails statically; x1 vs y = x1 is exact
    s, ws, k = prog.eval_loss_rowsets(dev, L2, np.array([[3, 3, 7], [1, 2, 3], [99, 0, 0]]))
    assert list(k) == [True, False, True] and s[0] == 0.0 and np.all(ws == 3)
    # out-of-range indices are rejected
    with pytest.raises(srhip.SrhipError):
        prog.eval_loss_rowsets(dev, L2, np.array([[0], [1], [100]]))
    with pytest.raises(ValueError):
        prog.eval_loss_rowsets(dev, L2, np.array([[0], [1]]))
    # empty tree list
    l, k = srhip.eval_loss_batch_rowsets([], ds, o, [])
    assert l.shape == (0,) and k.shape == (0,)


def test_lockstep_search_scores_each_minibatch_request_in_one_launch(gpu_ctx, monkeypatch):
    """With batching=True the lockstep search answers every ScoreRows request
    of a round (all islands' parents or babies, each on its own sample) with
    ONE engine launch: srhip_eval_loss_rowsets is called once per request batch."""
    from srhip import evolution as ev

    calls = {"rowsets": 0, "answers": 0}
    orig = srhip.engine.Program.eval_loss_rowsets

    def counted(self, *a, **kw):
        calls["rowsets"] += 1
        return orig(self, *a, **kw)

    monkeypatch.setattr(srhip.engine.Program, "eval_loss_rowsets", counted)
    orig_rows = ev.EngineEvaluator.losses_rows

    def rows_answer(self, trees, rows):
        calls["answers"] += 1
        assert len({len(r) for r in rows}) == 1
        return orig_rows(self, trees, rows)

    monkeypatch.setattr(ev.EngineEvaluator, "losses_rows", rows_answer)
    rng = np.random.default_rng(0)
    X = rng.standard_normal((5, 500)).astype(np.float32)
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
    o = srhip.Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp"], batching=True,
                      batch_size=50, npopulations=4, npop=20, ncycles_per_iteration=5)
    hof, stats = srhip.equation_search(X, y, o, niterations=1, seed=3)
    assert calls["answers"] > 0 and calls["rowsets"] == calls["answers"]
