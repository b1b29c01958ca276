"""Config #2 at full size (4096 trees × 1M rows × 5 features, Float32) with
losses other than L2 (round 6): the loss tree code's tile tails for L1,
Huber and LogCosh (jit.cpp, the PRECISE-region loss routines after the FAST
or PRECISE tree body; the FAST path's loss-parity guards were tuned on L2)
against the oracle (LossFunctions.jl's distance losses,
src/LossFunctions.jl:11-31): did_succeed identical on every tree, and every
succeeding tree's mean loss within the north_star's 1e-5 of the oracle's."""
import json
from pathlib import Path

import numpy as np
import pytest

import oracle
import srhip

pytestmark = pytest.mark.gpu

LOSSES = [srhip.L1DistLoss(), srhip.HuberLoss(1.0), srhip.LogCoshLoss(), srhip.L2DistLoss()]


@pytest.mark.parametrize("loss", LOSSES, ids=lambda l: f"kind{l.kind}")
def test_config2_full_size_other_losses(gpu_ctx, loss):
    """(L2 here with row weights: the weighted loops, sr_jit_eval_dlpw)"""
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(4096, o, 5, np.float32, seed=0)
    rng = np.random.default_rng(1)
    X = rng.standard_normal((5, 1_000_000)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    prog = srhip.Program(gpu_ctx, flat, np.float32)
    w = None
    if loss.kind == 0:  # L2: the weighted tree loops
        w = np.abs(rng.standard_normal(1_000_000)).astype(np.float32) + np.float32(0.1)
    ds = srhip.DeviceDataset(gpu_ctx, X, y, w)
    s, wsum, ok = prog.eval_loss(ds, loss.kind, loss.params)
    assert gpu_ctx.last_tree_code() > 4000
    ok = np.asarray(ok, dtype=bool)
    _, ref_l, ref_ok = oracle.eval_loss_batch(flat, X, y, w, loss.kind, loss.params, dtype=np.float32,
                                              nthreads=16)
    bad = np.flatnonzero(ok != ref_ok.astype(bool))
    assert bad.size == 0, f"did_succeed differs on {bad[:20]}"
    m = ok & np.isfinite(ref_l) & (ref_l != 0)
    with np.errstate(invalid="ignore", divide="ignore"):
        rel = np.abs(np.asarray(s, dtype=np.float64) / wsum - ref_l) / np.abs(ref_l)
    out = np.flatnonzero(m & ~(rel <= 1e-5))
    rec = {"test": f"config2_full_loss_kind{loss.kind}" + ("_weighted" if w is not None else ""), "succeeding": int(m.sum()), "outside_1e-5": int(out.size),
           "max_rel": float(np.max(rel[m])), "median_rel": float(np.median(rel[m]))}
    d = Path(__file__).resolve().parent.parent / "gpurun_out"
    d.mkdir(exist_ok=True)
    with open(d / "parity_counts.jsonl", "a") as f:
        f.write(json.dumps(rec) + "\n")
    assert m.sum() > 3000
    assert out.size == 0, (out[:20].tolist(), rel[out[:20]].tolist())
