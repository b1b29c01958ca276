"""BASELINE.json configs #5 and #4 at their workloads on one MI355X.

#5  20 features x 10M rows Float32, 16384 trees (SURVEY.md §8 e/f):
    * eval_loss over all 10M rows; the oracle re-evaluates a sample of 384
      trees over every row (did_succeed identical, losses within the
      north_star's 1e-5 or the tree's conditioning);
    * config #5's row partition (8 shards of 1.25M rows): per-shard sums add
      up to the full-size sums, did_succeed is the AND over shards;
    * eval_loss_grad (∂L/∂c of every constant) over one 1.25M-row shard
      against the oracle's Float64 forward-mode derivatives.
#4  EquationSearch with 64 islands, 10 features x 100k rows, every island on
    this GPU (the lockstep search scores all islands' babies per launch); the
    hall of fame's losses re-checked by the oracle.
"""
import numpy as np
import pytest

import oracle
import srhip
from srhip import constants as K
from numerics import assert_close_conditioned, loss_spread
from test_full_size import _check_losses
from test_search import oracle_scorer

pytestmark = pytest.mark.gpu

CFG = dict(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])


@pytest.mark.timeout(600)
def test_config5_20feat_10M_rows_16k_trees(gpu_ctx):
    o = srhip.Options(**CFG)
    rng = np.random.default_rng(51)
    n, F, NT = 10_000_000, 20, 16384
    X = rng.standard_normal((F, n), dtype=np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    trees = srhip.random_population(NT, o, F, np.float32, seed=52)
    ctx = gpu_ctx
    flat = srhip.flatten(trees, o, dtype=np.float32)
    prog = srhip.Program(ctx, flat, np.float32)
    ds = srhip.DeviceDataset(ctx, X, y)
    s, w, ok = prog.eval_loss(ds, K.LOSS["L2"])
    assert w == n and 0.05 < 1 - ok.mean() < 0.6
    del ds

    # (1) the oracle on every row, for a sample of trees
    sub = np.sort(rng.choice(NT, 384, replace=False))
    st = [trees[i] for i in sub]
    _, ref_l, ref_ok = oracle.eval_loss_batch(srhip.flatten(st, o, dtype=np.float32), X, y, dtype=np.float32,
                                              nthreads=16)
    losses = (s[sub] / n).astype(np.float32)
    nchk, _ = _check_losses(st, o, X, y, np.float32, losses, ok[sub], ref_l, ref_ok, 1e-5, name="config5_sample",
                            strict=True)
    assert nchk > 150

    # (2) config #5's partition: 8 row shards of 1.25M rows
    tot = np.zeros(NT)
    okall = np.ones(NT, dtype=bool)
    for r in range(8):
        dsr = srhip.DeviceDataset(ctx, X, y, row_begin=r * n // 8, row_end=(r + 1) * n // 8)
        sr, wr, okr = prog.eval_loss(dsr, K.LOSS["L2"])
        assert wr == n // 8
        tot += np.where(okr, sr, 0.0)
        okall &= okr
        del dsr
    assert np.array_equal(okall, ok)
    # the shards regroup the rows into tiles: a guarded FAST tile of one
    # grouping may be redone precisely in the other, which moves an
    # ill-conditioned tree by its conditioning (tests/numerics.py)
    both_inf = np.isinf(tot) & (tot == s)  # Float32 squares past FLT_MAX: Inf loss in both groupings
    with np.errstate(invalid="ignore"):
        rel = np.abs(tot - s) / np.abs(s)
    out = np.flatnonzero(ok & ~both_inf & ~(rel <= 1e-6))
    assert out.size <= 0.01 * ok.sum()
    if out.size:
        sp = loss_spread([trees[i] for i in out], o, X, y, None, np.float32, nperturb=2)
        assert_close_conditioned(tot[out], s[out], sp, rtol=1e-6, msg="shard sums")

    # (3) ∂L/∂c over one shard, 48 trees with constants, against the oracle
    shard = srhip.DeviceDataset(ctx, X, y, row_begin=0, row_end=n // 8)
    Xs, ys = X[:, : n // 8], y[: n // 8].astype(np.float64)
    gt = [t for i, t in enumerate(trees) if ok[i] and srhip.get_constants(t)][:48]
    gflat = srhip.flatten(gt, o, dtype=np.float32)
    gp = srhip.Program(ctx, gflat, np.float32)
    gsum, grads, gw, gok = gp.eval_loss_grad(shard, K.LOSS["L2"])
    assert gok.all() and gw == n // 8
    ls, _, lok = gp.eval_loss(shard, K.LOSS["L2"])
    np.testing.assert_allclose(gsum, ls, rtol=1e-6)
    f64 = srhip.flatten(gt, o, dtype=np.float64)
    X64 = Xs.astype(np.float64)
    # reference ∂L/∂c in Float64, and its spread when X and the constants move
    # by one Float32 ulp (tests/numerics.py): near a pole of ŷ or of ∂ŷ/∂c one
    # row's rounding decides the sum, which Float32 rows cannot reproduce;
    # and directly against the oracle's Float32 evaluation (the reference's
    # precision) under a tight bound: 1e-5 of Σ|terms| plus what a 4-ulp
    # difference of ŷ moves the terms by (no perturbation allowance)
    prng = np.random.default_rng(53)
    eps = float(np.finfo(np.float32).eps)
    Xp = [X64 * (1 + eps * prng.uniform(-1, 1, X64.shape)) for _ in range(2)]
    nbad = nbad32 = 0
    for t in range(len(gt)):
        k, a, _ = f64.tree(t)
        c = gflat.consts[gflat.const_off[t]:gflat.const_off[t + 1]].astype(np.float64)

        def dl(cc, XX):
            out, g, rok = oracle.eval_grad_consts(k, a, cc, XX, len(cc))
            terms = 2.0 * (out - ys)[None, :] * g
            return terms.sum(axis=1), np.abs(terms).sum(axis=1), rok

        ref, mass, rok = dl(c, X64)
        assert rok
        spread = np.zeros_like(ref)
        for XX in Xp:
            r2, _, _ = dl(c * (1 + eps * prng.uniform(-1, 1, c.shape)), XX)
            spread = np.maximum(spread, np.abs(r2 - ref))
        mine = grads[gflat.const_off[t]:gflat.const_off[t + 1]]
        b = ~(np.abs(mine - ref) <= 1e-4 * mass + 4 * spread)
        if b.any():
            print("grad outlier:", gt[t], mine[b], ref[b], mass[b], spread[b])
        nbad += int(b.sum())
        o32, g32, ok32 = oracle.eval_grad_consts(k, a, c.astype(np.float32), Xs, len(c), dtype=np.float32)
        assert ok32
        o32, g32 = o32.astype(np.float64), g32.astype(np.float64)
        t32 = 2.0 * (o32 - ys)[None, :] * g32
        dv = (np.abs(2.0 * g32) * (4 * eps * (np.abs(o32) + np.abs(ys)))[None, :]).sum(axis=1)
        b32 = ~(np.abs(mine - t32.sum(axis=1)) <= 1e-5 * np.abs(t32).sum(axis=1) + dv)
        if b32.any():
            print("grad outlier vs the Float32 oracle:", gt[t], mine[b32], t32.sum(axis=1)[b32])
        nbad32 += int(b32.sum())
    assert nbad32 == 0
    assert nbad == 0


@pytest.mark.timeout(600)
def test_config4_64_islands_10feat_100k_rows(gpu_ctx):
    rng = np.random.default_rng(41)
    X = rng.standard_normal((10, 100_000)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    o = srhip.Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp"], npopulations=64,
                      ncycles_per_iteration=100)
    hof, stats = srhip.equation_search(X, y, o, niterations=2, seed=3)
    front = hof.dominating()
    assert front and stats["launches"] >= 200
    ref = oracle_scorer(o, X, y)([m.tree for m in front])
    np.testing.assert_allclose([m.loss for m in front], ref, rtol=1e-5)
    assert min(m.loss for m in front) < 0.75 * float(np.var(y))
