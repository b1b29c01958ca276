"""Condition-aware comparison helpers for the parity tests.

Two correct evaluations of the same tree can differ by far more than a few
ulp when the tree amplifies rounding differences (cos of a huge argument,
x/(c - x) near a pole, exp of a large value...). The bar the engine must meet
is per operator (bit-exact + - * /, ≤ 4 ulp transcendentals — checked
directly by test_each_unary_operator / test_each_binary_operator); for whole
trees the tests allow, per row, the spread the oracle itself shows when X and
the constants are perturbed at the ulp scale of T and every transcendental
value carries rounding noise of the per-operator bar (oracle.set_noise).
"""
import numpy as np

import oracle
import srhip

# perturbation size: 4 ulp of T (a perturbation below 1 ulp of float64 would
# round away when applied in float64)
EPS = {np.dtype(np.float32): 4 * 2.0 ** -23, np.dtype(np.float64): 4 * 2.0 ** -52}
# rounding noise on every transcendental value (oracle.set_noise): the engine's
# per-operator bar is <= 4 ulp, so two correct evaluations of one tree may
# differ by what noise of that size does to it (rounding INSIDE the tree,
# which input perturbations do not model: cos of a cancellation, exp chains)
OP_EPS = {np.dtype(np.float32): 4 * 2.0 ** -24, np.dtype(np.float64): 4 * 2.0 ** -53}


def _perturbed(flat, X, T, k, rng):
    eps = EPS[np.dtype(T)]
    Xp = X.astype(np.float64) * (1 + eps * rng.uniform(-1, 1, X.shape))
    fp = srhip.node.FlatTrees(flat.node_off, flat.kind, flat.arg, flat.const_off,
                              flat.consts.astype(np.float64) * (1 + eps * rng.uniform(-1, 1, flat.consts.shape)),
                              flat.nodes)
    return fp, Xp


def output_spread(trees, options, X, T, nperturb=3, seed=0):
    """Per (tree, row): max |f(X', c') - f(X, c)| over ulp-scale perturbations,
    evaluated in float64 by the oracle."""
    flat = srhip.flatten(trees, options, dtype=np.float64)
    flat.consts = srhip.flatten(trees, options, dtype=T).consts.astype(np.float64)
    return output_spread_flat(flat, X, T, nperturb, seed)


def output_spread_flat(flat, X, T, nperturb=3, seed=0):
    """output_spread for an already flattened batch (constants rounded to T)."""
    rng = np.random.default_rng(seed)
    flat = srhip.node.FlatTrees(flat.node_off, flat.kind, flat.arg, flat.const_off,
                                np.asarray(flat.consts, dtype=np.float64), flat.nodes)
    base, _ = oracle.eval_trees(flat, X.astype(np.float64), dtype=np.float64)
    spread = np.zeros_like(base)
    with np.errstate(invalid="ignore", over="ignore"):
        for k in range(nperturb):
            fp, Xp = _perturbed(flat, X, T, 1, rng)
            oracle.set_noise(OP_EPS[np.dtype(T)], seed * 1000 + k + 1)
            try:
                pert, _ = oracle.eval_trees(fp, Xp, dtype=np.float64)
            finally:
                oracle.set_noise(0.0)
            d = np.abs(pert - base)
            spread = np.where(np.isfinite(d), np.maximum(spread, d), np.inf)
    return spread


def loss_spread(trees, options, X, y, w, T, nperturb=3, seed=0, loss=None):
    """Per tree: max |Σ w ℓ (perturbed) - Σ w ℓ| (float64 oracle)."""
    loss = loss or options.elementwise_loss
    flat = srhip.flatten(trees, options, dtype=np.float64)
    flat.consts = srhip.flatten(trees, options, dtype=T).consts.astype(np.float64)
    return loss_spread_flat(flat, X, y, w, T, loss, nperturb, seed)


def loss_spread_flat(flat, X, y, w, T, loss, nperturb=3, seed=0):
    """loss_spread for an already flattened batch (constants rounded to T)."""
    rng = np.random.default_rng(seed)
    flat = srhip.node.FlatTrees(flat.node_off, flat.kind, flat.arg, flat.const_off,
                                np.asarray(flat.consts, dtype=np.float64), flat.nodes)
    y64 = y.astype(np.float64)
    w64 = None if w is None else w.astype(np.float64)
    base, _, _ = oracle.eval_loss_batch(flat, X.astype(np.float64), y64, w64, loss.kind, loss.params,
                                        dtype=np.float64)
    spread = np.zeros_like(base)
    with np.errstate(invalid="ignore", over="ignore"):
        for k in range(nperturb):
            fp, Xp = _perturbed(flat, X, T, 1, rng)
            oracle.set_noise(OP_EPS[np.dtype(T)], seed * 1000 + k + 1)
            try:
                pert, _, _ = oracle.eval_loss_batch(fp, Xp, y64, w64, loss.kind, loss.params, dtype=np.float64)
            finally:
                oracle.set_noise(0.0)
            d = np.abs(pert - base)
            spread = np.where(np.isfinite(d), np.maximum(spread, d), np.inf)
    return spread


def assert_close_conditioned(actual, desired, spread, rtol, atol=0.0, factor=4.0, msg="", max_bad_frac=0.0):
    """|actual - desired| <= atol + rtol |desired| + factor * spread, elementwise
    (factor 4: an evaluation within the per-operator bar lands within the
    spread of the oracle's own perturbed evaluations, up to sampling: the
    FAST path's outliers at full size measure <= 0.85 x spread,
    profiles/r03_fast_parity.json)
    (a fraction max_bad_frac of the elements may exceed it: the input
    perturbation does not model rounding inside the tree, which matters for
    f32 derivatives near cancellations)."""
    actual = np.asarray(actual, dtype=np.float64)
    desired = np.asarray(desired, dtype=np.float64)
    tol = atol + rtol * np.abs(desired) + factor * spread
    with np.errstate(invalid="ignore"):
        bad = ~(np.abs(actual - desired) <= tol)
    bad &= ~(np.isnan(actual) & np.isnan(desired)) & ~(actual == desired)  # equal infinities agree
    if bad.sum() > max_bad_frac * bad.size:
        i = np.flatnonzero(bad.ravel())[:5]
        raise AssertionError(f"{msg}: {bad.sum()} of {bad.size} beyond the conditioned bound; "
                             f"actual={actual.ravel()[i]} desired={desired.ravel()[i]} "
                             f"spread={np.asarray(spread).ravel()[i]}")


def record_tail(name, rec):
    """Append one tail record (worst error / spread ratios of a parity test) to
    gpurun_out/parity_tails.jsonl (copied to profiles/ after a GPU run)."""
    import json
    from pathlib import Path

    out = Path(__file__).resolve().parent.parent / "gpurun_out"
    out.mkdir(exist_ok=True)
    with open(out / "parity_tails.jsonl", "a") as f:
        f.write(json.dumps(dict(test=name, **rec)) + "\n")


def assert_loss_tail(name, actual, desired, mask, flat, X, y, w, T, kind, params, rtol, bar=1e-5):
    """Every tree of `mask` within `rtol` of the oracle's mean loss, or — for the
    ill-conditioned tail — within 4x the oracle's own perturbation spread
    (loss_spread_flat: ulp-scale moves of X and the constants plus
    per-operator rounding noise), no fraction of trees left unchecked.
    Records the tail (count outside rtol, outside `bar` = north_star's 1e-5,
    worst error / spread) under gpurun_out/parity_tails.jsonl."""
    actual = np.asarray(actual, dtype=np.float64)
    desired = np.asarray(desired, dtype=np.float64)
    with np.errstate(invalid="ignore", divide="ignore"):
        rel = np.abs(actual - desired) / np.abs(desired)
    out = np.flatnonzero(mask & ~(rel <= rtol))
    rec = dict(checked=int(mask.sum()), rtol=rtol, outside_rtol=int(out.size),
               outside_bar=int(np.sum(mask & ~(rel <= bar))), bar=bar,
               max_rel=float(np.max(rel[mask])) if mask.any() else 0.0, max_err_over_spread=0.0)
    if out.size:
        from types import SimpleNamespace

        wsum = float(len(y)) if w is None else float(np.sum(w, dtype=np.float64))
        sp = loss_spread_flat(flat.take(out), X, y, w, T, SimpleNamespace(kind=kind, params=tuple(params)),
                              nperturb=3) / wsum
        err = np.abs(actual[out] - desired[out]) - rtol * np.abs(desired[out])
        with np.errstate(invalid="ignore", divide="ignore"):
            rec["max_err_over_spread"] = float(np.nanmax(err / sp))
        record_tail(name, rec)
        assert_close_conditioned(actual[out], desired[out], sp, rtol=rtol, factor=4.0, msg=f"{name} tail")
    else:
        record_tail(name, rec)
    return rec
