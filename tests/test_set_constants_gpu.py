"""srhip_program_set_constants on a VARYING_CONSTANTS program (the constant
optimiser's candidates) against a program created fresh with the same
constants: constants that make trees fail statically (an overflowing folded
subtree, a NaN constant) and then finite again are patched in place
(compile_batch keep_layout: no full rebuild), and every step's losses,
did_succeed and ∂L/∂c equal the fresh program's. Reference: the constant
optimiser's set_constants! between evaluations, ConstantOptimization.jl:12-19."""
import numpy as np
import pytest

import srhip
from srhip import constants as K
from srhip.node import FlatTrees

pytestmark = pytest.mark.gpu


def _with_consts(flat, c):
    return FlatTrees(flat.node_off, flat.kind, flat.arg, flat.const_off, np.asarray(c, dtype=flat.consts.dtype),
                     flat.nodes)


def _steps(c0, rng):
    n = len(c0)
    big = c0.copy()
    big[rng.choice(n, n // 8, replace=False)] = np.float32(1e30)  # exp / products overflow: folds fail
    nan = c0.copy()
    nan[rng.choice(n, n // 10, replace=False)] = np.nan
    return [("x0", c0), ("big", big), ("scaled", (c0 * np.float32(1.1)).astype(np.float32)), ("nan", nan),
            ("x0 again", c0), ("big again", big),
            ("noise", (c0 * (1 + rng.standard_normal(n).astype(np.float32) / 2)).astype(np.float32))]


@pytest.mark.parametrize("ntrees", [300, 1200])
def test_set_constants_in_place_equals_fresh_program(gpu_ctx, ntrees):
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(5 + ntrees)
    n = 3001
    X = rng.standard_normal((5, n)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0]).astype(np.float32)
    trees = srhip.random_population(ntrees, o, 5, np.float32, seed=6 + ntrees)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    ctx = gpu_ctx
    ds = srhip.DeviceDataset(ctx, X, y)
    prog = srhip.Program(ctx, flat, np.float32, varying_constants=True)
    for name, c in _steps(np.asarray(flat.consts, dtype=np.float32), rng):
        prog.set_constants(c)
        s, w, ok = prog.eval_loss(ds, K.LOSS["L2"])
        s, ok = s.copy(), ok.copy()
        gs, gg, gw, gok = prog.eval_loss_grad(ds, K.LOSS["L2"])
        fresh = srhip.Program(ctx, _with_consts(flat, c), np.float32)
        fs, fw, fok = fresh.eval_loss(ds, K.LOSS["L2"])
        fgs, fgg, fgw, fgok = fresh.eval_loss_grad(ds, K.LOSS["L2"])
        assert np.array_equal(ok, fok), (name, np.flatnonzero(ok != fok)[:10])
        assert np.array_equal(gok, fgok), (name, np.flatnonzero(gok != fgok)[:10])
        m = ok & np.isfinite(fs)
        with np.errstate(all="ignore"):
            rel = np.abs(s[m] - fs[m]) / np.maximum(np.abs(fs[m]), 1e-30)
        # memory-constant and literal-constant tree code may take different
        # (equally accurate) routes, e.g. the constant-divisor reciprocal: the
        # loss parity bar of the rest of the suite
        assert np.all(rel <= 1e-5), (name, float(rel.max()))
        # ∂L/∂c of the succeeding trees
        co = flat.const_off
        for t in np.flatnonzero(gok)[:200]:
            a, b = co[t], co[t + 1]
            if b > a:
                np.testing.assert_allclose(gg[a:b], fgg[a:b], rtol=1e-4, atol=1e-6 * max(1.0, float(np.abs(fgg[a:b]).max())),
                                           err_msg=f"{name} tree {t}")
    assert prog.update_stats()["rebuilt"] == 0, prog.update_stats()
