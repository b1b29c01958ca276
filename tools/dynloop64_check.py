"""Float64 hand-written tree loop (sr_jit64_eval_dl, default) against the
compiled one (SRHIP_JIT_DYNLOOP=0): config #3's operator set on NaN-heavy
data, weighted and not, partial last tile; sums and did_succeed bit for bit;
then config #3 (4096 trees x 100k rows) timed interleaved."""
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


def main():
    o = srhip.Options(**CFG3)
    ctx = srhip.get_context(0)
    rng = np.random.default_rng(3)
    for name, nt, n, weighted in (("small", 700, 20_001, False), ("small_w", 700, 20_001, True),
                                  ("cfg3", 4096, 100_000, False)):
        X = rng.uniform(-3, 3, (5, n))
        y = np.cos(X[3]) * 2 + X[0] ** 2 - 2
        w = rng.uniform(0.5, 2, n) if weighted else None
        trees = srhip.random_population(nt, o, 5, np.float64, seed=3)
        ds = srhip.DeviceDataset(ctx, X, y, w)
        os.environ["SRHIP_JIT"] = "1"
        try:
            prog = srhip.Program(ctx, srhip.flatten(trees, o, dtype=np.float64), np.float64)
        finally:
            del os.environ["SRHIP_JIT"]
        res, ks = {}, {"0": [], "1": []}
        for r in range(6):
            for m in (("0", "1") if r % 2 == 0 else ("1", "0")):
                os.environ["SRHIP_JIT_DYNLOOP"] = m
                for _ in range(3):
                    res[m] = prog.eval_loss(ds, K.LOSS["L2"])
                    ks[m].append(ctx.last_kernel_time()[0])
        del os.environ["SRHIP_JIT_DYNLOOP"]
        (s0, w0, ok0), (s1, w1, ok1) = res["0"], res["1"]
        same = bool(np.array_equal(ok0, ok1) and np.array_equal(s0[ok0], s1[ok1]) and w0 == w1)
        print(json.dumps(dict(case=name, identical=same, tree_code=prog.jit_info()["ntrees"],
                              static_ms=round(float(np.median(ks["0"])), 4),
                              dynloop_ms=round(float(np.median(ks["1"])), 4), ok=int(ok0.sum()))), flush=True)
        if not same:
            sys.exit(1)


if __name__ == "__main__":
    main()
