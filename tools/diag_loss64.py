"""Float64 losses other than L2 on the device vs the same losses computed on
the host from the device's own per-row outputs (Program.eval_tree_array):
which trees does the device fail, and with what loss, that the host does not?
Prints one JSON line per (loss, weighted) case. Run on the GPU box."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402

CFG3 = dict(binary_operators=["+", "-", "*", "/", "^"], unary_operators=["safe_log", "safe_sqrt", "cos", "exp"])


def host_loss(kind, p, r):
    ar = np.abs(r)
    if kind == "L1":
        return ar
    if kind == "LOGCOSH":
        return ar + np.log1p(np.exp(-2.0 * ar)) - np.log(2.0)
    if kind == "LOGITDIST":
        return ar + 2.0 * np.log1p(np.exp(-ar)) - np.log(4.0)
    if kind == "HUBER":
        return np.where(ar <= p, 0.5 * r * r, p * (ar - 0.5 * p))
    raise ValueError(kind)


def main():
    o = srhip.Options(**CFG3)
    ctx = srhip.get_context(0)
    for k, (loss, par) in enumerate([("LOGCOSH", 0.0), ("L1", 0.0), ("LOGITDIST", 0.0), ("HUBER", 1.0)]):
        rng = np.random.default_rng(40)
        n = 10_001
        X = rng.uniform(-3, 3, (5, n))
        y = rng.standard_normal(n)
        wts = rng.uniform(0.5, 2.0, n)
        trees = srhip.random_population(600, o, 5, np.float64, seed=38)
        flat = srhip.flatten(trees, o, dtype=np.float64)
        for weighted in (False, True):
            w = wts if weighted else None
            ds = srhip.DeviceDataset(ctx, X, y, w)
            for jit in ("0", "1"):
                os.environ["SRHIP_JIT"] = jit
                try:
                    prog = srhip.Program(ctx, flat, np.float64)
                finally:
                    del os.environ["SRHIP_JIT"]
                s, ws, ok = prog.eval_loss(ds, K.LOSS[loss], [par])
                out, ook = prog.eval_tree_array(ds)
                out = np.asarray(out)[:, :n]
                with np.errstate(all="ignore"):
                    lh = host_loss(loss, par, out - y)
                    sh = (lh * (w if w is not None else 1.0)).sum(axis=1)
                hok = np.asarray(ook, bool) & np.isfinite(sh)
                bad = np.flatnonzero(np.asarray(ok, bool) != hok)
                rec = dict(loss=loss, weighted=weighted, jit=jit, tree_code=int(ctx.last_tree_code()),
                           n_ok=int(np.sum(ok)), n_hok=int(hok.sum()), mismatch=bad[:12].tolist(),
                           examples=[dict(i=int(i), tree=str(trees[i]), dev_s=float(s[i]), host_s=float(sh[i]),
                                          dev_ok=bool(ok[i]), out_ok=bool(ook[i])) for i in bad[:3]])
                print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
