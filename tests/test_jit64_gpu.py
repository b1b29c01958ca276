"""Float64 tree code (csrc/jit64.cpp; VERDICT r03 missing 3): the shallow
trees of a Float64 program as straight-line code with the Float64
interpreter's operator routines (gen_jit64.py), L2 loss, weighted or not.
Config #3's operator set (safe_log / safe_sqrt / safe_pow / div on mixed-sign
data: NaN-heavy). Checks: the tree code ran (srhip_last_tree_code),
did_succeed identical to the interpreter's and the oracle's on every tree,
losses equal to the interpreter's up to the summation order and to the
oracle's Float64 losses; after set_constants the program runs interpreted
(the constants are literals of the code) with correct results."""
import os

import numpy as np
import pytest

import oracle
import srhip
from numerics import assert_close_conditioned, assert_loss_tail, output_spread_flat, record_tail
from srhip import constants as K

pytestmark = pytest.mark.gpu

CFG3 = dict(binary_operators=["+", "-", "*", "/", "^"], unary_operators=["safe_log", "safe_sqrt", "cos", "exp"])


def _progs(ctx, flat):
    progs = {}
    for mode in ("1", "0"):
        os.environ["SRHIP_JIT"] = mode
        try:
            progs[mode] = srhip.Program(ctx, flat, np.float64)
        finally:
            del os.environ["SRHIP_JIT"]
    return progs


@pytest.mark.parametrize("weighted", [False, True])
def test_float64_tree_code_matches_interpreter_and_oracle(gpu_ctx, weighted):
    o = srhip.Options(**CFG3)
    rng = np.random.default_rng(31 + weighted)
    n = 20_001  # a partial last tile
    X = rng.uniform(-3, 3, (5, n))
    y = rng.standard_normal(n)
    w = rng.uniform(0.5, 2.0, n) if weighted else None
    trees = srhip.random_population(1024, o, 5, np.float64, seed=32)
    flat = srhip.flatten(trees, o, dtype=np.float64)
    ctx = gpu_ctx
    ds = srhip.DeviceDataset(ctx, X, y, w)
    progs = _progs(ctx, flat)
    assert progs["1"].jit_info()["ntrees"] > 500, progs["1"].jit_info()
    s1, w1, ok1 = progs["1"].eval_loss(ds, K.LOSS["L2"])
    assert ctx.last_tree_code() > 500
    s0, w0, ok0 = progs["0"].eval_loss(ds, K.LOSS["L2"])
    assert ctx.last_tree_code() == 0 and w1 == w0
    assert np.array_equal(ok1, ok0)
    with np.errstate(invalid="ignore", divide="ignore"):
        rel = np.abs(s1 - s0) / np.abs(s0)
    m = ok1 & (s0 != 0)
    assert np.all(rel[m] <= 1e-11), float(np.nanmax(rel[m]))
    _, rl, rok = oracle.eval_loss_batch(flat, X, y, w, 0, (0.0,), dtype=np.float64, nthreads=16)
    assert np.array_equal(ok1, rok)
    with np.errstate(invalid="ignore", divide="ignore"):
        relo = np.abs(s1 / w1 - rl) / np.abs(rl)
    mo = ok1 & np.isfinite(rl) & (rl != 0)
    assert np.all(relo[mo] <= 1e-9), float(np.nanmax(relo[mo]))
    assert 0.05 < ok1.mean() < 0.95


def test_float64_tree_code_new_constants_run_interpreted(gpu_ctx):
    o = srhip.Options(**CFG3)
    rng = np.random.default_rng(33)
    n = 5000
    X = rng.uniform(-3, 3, (5, n))
    y = rng.standard_normal(n)
    trees = srhip.random_population(600, o, 5, np.float64, seed=34)
    flat = srhip.flatten(trees, o, dtype=np.float64)
    ctx = gpu_ctx
    ds = srhip.DeviceDataset(ctx, X, y)
    progs = _progs(ctx, flat)
    progs["1"].eval_loss(ds, K.LOSS["L2"])
    assert ctx.last_tree_code() > 300
    newc = flat.consts * 1.5 - 0.25
    for p in progs.values():
        p.set_constants(newc)
    s1, _, ok1 = progs["1"].eval_loss(ds, K.LOSS["L2"])
    assert ctx.last_tree_code() == 0
    s0, _, ok0 = progs["0"].eval_loss(ds, K.LOSS["L2"])
    assert np.array_equal(ok1, ok0)
    np.testing.assert_array_equal(s1[ok1], s0[ok0])


def test_float64_output_tree_code_equals_interpreter(gpu_ctx):
    """eval_tree_array of a Float64 program (config #3, InterfaceDynamicExpressions.jl:50-52)
    through its per-row output tree code (jit64.cpp emit_store_out): every
    tree's outputs identical to the interpreter's MODE_OUT (NaN where NaN),
    did_succeed = interpreter = oracle."""
    o = srhip.Options(**CFG3)
    rng = np.random.default_rng(35)
    n = 20_001
    X = rng.uniform(-3, 3, (5, n))
    y = np.zeros(n)
    trees = srhip.random_population(1024, o, 5, np.float64, seed=36)
    flat = srhip.flatten(trees, o, dtype=np.float64)
    ctx = gpu_ctx
    ds = srhip.DeviceDataset(ctx, X, y)
    progs = _progs(ctx, flat)
    out1, ok1 = progs["1"].eval_tree_array(ds)
    assert ctx.last_tree_code() > 500 and ctx.last_kernel_name() == "sr_jit64_out"
    out0, ok0 = progs["0"].eval_tree_array(ds)
    assert ctx.last_tree_code() == 0
    assert np.array_equal(ok1, ok0)
    assert np.array_equal(out1, out0, equal_nan=True)
    _, _, rok = oracle.eval_loss_batch(flat, X, y, dtype=np.float64, nthreads=16)
    assert np.array_equal(ok1, rok)
    # the values of succeeding trees against the oracle's Float64 evaluation
    # (device vs host libm: ulp-level differences, amplified by cancellations)
    ref = oracle.eval_trees(flat, X[:, :2000], dtype=np.float64)[0]
    sel = np.flatnonzero(ok1)[:200]
    with np.errstate(invalid="ignore", divide="ignore"):
        rel = np.abs(out1[sel, :2000] - ref[sel]) / np.maximum(np.abs(ref[sel]), 1e-300)
    # every row within 1e-9, or (the ill-conditioned rows) within 4x the
    # oracle's own spread under ulp-scale perturbations: no row unchecked
    bad = ~(rel <= 1e-9) & ~(np.isnan(out1[sel, :2000]) & np.isnan(ref[sel]))
    rows = np.flatnonzero(bad.any(axis=0))
    tr = np.flatnonzero(bad.any(axis=1))
    rec = dict(checked=int(rel.size), rtol=1e-9, outside_rtol=int(bad.sum()), max_err_over_spread=0.0)
    if tr.size:
        sp = output_spread_flat(flat.take(sel[tr]), X[:, rows], np.float64)
        a, d = out1[sel[tr]][:, rows], ref[sel[tr]][:, rows]
        with np.errstate(invalid="ignore", divide="ignore"):
            rec["max_err_over_spread"] = float(np.nanmax(np.where(bad[np.ix_(tr, rows)],
                                                                  (np.abs(a - d) - 1e-9 * np.abs(d)) / sp, 0)))
        assert_close_conditioned(a, d, sp, rtol=1e-9, factor=4.0, msg="Float64 per-row outputs")
    record_tail("float64_output_tree_code_rows", rec)


LOSS_CASES = [("L1", 0.0), ("LP", 2.5), ("HUBER", 1.0), ("LOGCOSH", 0.0), ("L1EPSINS", 0.3), ("L2EPSINS", 0.3),
              ("QUANTILE", 0.3), ("PERIODIC", 2.0), ("LOGITDIST", 0.0)]


@pytest.mark.parametrize("loss,param", LOSS_CASES, ids=[c[0] for c in LOSS_CASES])
def test_float64_loss_tree_code_other_losses(gpu_ctx, loss, param):
    """Float64 tree code with another elementwise loss in the tile tail
    (jit64.cpp emit_tail_loss: the Float64 interpreter's elem_loss as a
    routine), weighted for half of the losses: tree code ran, did_succeed =
    interpreter = oracle, losses within 1e-11 of the interpreter's (row-sum
    order) and 1e-9 of the oracle's (but for ill-conditioned trees)."""
    o = srhip.Options(**CFG3)
    k = [c[0] for c in LOSS_CASES].index(loss)
    rng = np.random.default_rng(37 + k)
    n = 10_001
    X = rng.uniform(-3, 3, (5, n))
    y = rng.standard_normal(n)
    w = rng.uniform(0.5, 2.0, n) if k % 2 else None
    trees = srhip.random_population(600, o, 5, np.float64, seed=38)
    flat = srhip.flatten(trees, o, dtype=np.float64)
    ctx = gpu_ctx
    ds = srhip.DeviceDataset(ctx, X, y, w)
    progs = _progs(ctx, flat)
    s1, w1, ok1 = progs["1"].eval_loss(ds, K.LOSS[loss], [param])
    # every loss has a Float64 routine (LogCosh / LogitDist since round 5: the
    # SGPRs above the routine temporaries are held live, gen_jit64.py)
    assert ctx.last_tree_code() > 300
    s0, w0, ok0 = progs["0"].eval_loss(ds, K.LOSS[loss], [param])
    assert ctx.last_tree_code() == 0 and w1 == w0
    assert np.array_equal(ok1, ok0)
    with np.errstate(invalid="ignore", divide="ignore"):
        rel = np.abs(s1 - s0) / np.abs(s0)
    m = ok1 & (s0 != 0) & np.isfinite(s0)
    assert np.all(rel[m] <= 1e-11), float(np.nanmax(rel[m]))
    _, rl, rok = oracle.eval_loss_batch(flat, X, y, w, K.LOSS[loss], (param,), dtype=np.float64, nthreads=16)
    assert np.array_equal(ok1, rok)
    with np.errstate(invalid="ignore", divide="ignore"):
        relo = np.abs(s1 / w1 - rl) / np.abs(rl)
    mo = ok1 & np.isfinite(rl) & (rl != 0)
    # one tree of this population, cos(exp(cos(c)^x5)·(c - x2)), takes cos of
    # arguments up to 1e20: a 1-ulp difference of device and host pow / exp
    # moves that cos anywhere (1e-4 .. 1e-3 here, interpreter and tree code
    # alike): such trees are held to the oracle's perturbation spread below
    # every tree within 1e-9 of the oracle, or within 4x the oracle's own
    # perturbation spread (Periodic: 1 - cos(2πr/c) of |ŷ| up to 1e10 moves by
    # (2π/c)·|Δr|, which the perturbed oracle runs show), no tree unchecked
    assert_loss_tail(f"float64_loss_tree_code_{loss}", s1 / w1, rl, mo, flat, X, y, w, np.float64,
                     K.LOSS[loss], (param,), rtol=1e-9)
    assert np.median(relo[mo]) <= 1e-13
