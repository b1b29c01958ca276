"""Gradient tree code (SRHIP_GJIT=1) against the forward-mode interpreter
(SRHIP_GJIT=0) and float64 numpy on one-operator trees of config #3's
operators: ∂L/∂c of each constant, side by side, at several row counts.
Usage: python tools/debug_grad_ops.py (GPU box)."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

import srhip  # noqa: E402
from srhip import Node  # noqa: E402
from srhip import constants as K  # noqa: E402


def main():
    o = srhip.Options(binary_operators=["+", "-", "*", "/", "^"], unary_operators=["safe_log", "safe_sqrt", "cos", "exp"])
    B, U = o.make_binary, o.make_unary

    def x(i):
        return Node(feature=i)

    def c(v):
        return Node(val=v)

    cases = [
        ("exp(0.3x)", U("exp", B("*", c(0.3), x(1))), lambda x: np.exp(0.3 * x), lambda x: x * np.exp(0.3 * x)),
        ("sqrt(1.3x)", U("safe_sqrt", B("*", c(1.3), x(1))), lambda x: np.sqrt(1.3 * x), lambda x: 0.5 * x / np.sqrt(1.3 * x)),
        ("log(1.3x)", U("safe_log", B("*", c(1.3), x(1))), lambda x: np.log(1.3 * x), lambda x: 1 / 1.3 + 0 * x),
        ("sqrt(1.3+x)", U("safe_sqrt", B("+", c(1.3), x(1))), lambda x: np.sqrt(1.3 + x), lambda x: 0.5 / np.sqrt(1.3 + x)),
        ("1.3*sqrt(x)", B("*", c(1.3), U("safe_sqrt", x(1))), lambda x: 1.3 * np.sqrt(x), lambda x: np.sqrt(x)),
    ]
    rng = np.random.default_rng(1)
    ctx = srhip.get_context(0)
    for n in (256, 512, 3001):
        X = (np.abs(rng.standard_normal((5, n))) + 0.1).astype(np.float32)
        y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
        x0, y0 = X[0].astype(np.float64), y.astype(np.float64)
        ds = srhip.DeviceDataset(ctx, X, y)
        for name, t, f, df in cases:
            out = {}
            for gj in ("1", "0"):
                os.environ["SRHIP_GJIT"] = gj
                prog = srhip.Program(ctx, srhip.flatten([t] * 300, o, dtype=np.float32), np.float32)
                s, g, w, ok = prog.eval_loss_grad(ds, K.LOSS["L2"])
                out[gj] = (float(s[0]), float(g[0]), prog.grad_jit_info()["ntrees"])
                del os.environ["SRHIP_GJIT"]
            r = f(x0) - y0
            print(f"n={n} {name:12s} jit {out['1']}  interp {out['0']}  numpy ({np.sum(r * r):.7g}, {np.sum(2 * r * df(x0)):.7g})",
                  flush=True)


if __name__ == "__main__":
    main()
