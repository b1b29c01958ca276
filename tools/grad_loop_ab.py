"""Interleaved A/B of the gradient tree loops on config #5's gradient
workload (16384 trees x 20 features x the 1.25M-row shard): compiled static
(SRHIP_JIT_DYNLOOP=0) against the hand-written one (default); after a
warm-up, rounds of 2 calls per mode in alternating order; median kernel ms."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402


def main():
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    ctx = srhip.get_context(0)
    n = 1_250_000
    X = np.random.default_rng(5).standard_normal((20, n), dtype=np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    trees = srhip.random_population(16384, o, 20, np.float32, seed=5)
    ds = srhip.DeviceDataset(ctx, X, y)
    prog = srhip.Program(ctx, srhip.flatten(trees, o, dtype=np.float32), np.float32)
    for _ in range(3):
        prog.eval_loss_grad(ds, K.LOSS["L2"])
    ks = {"static": [], "dynloop": []}
    for r in range(5):
        for m in (["static", "dynloop"] if r % 2 == 0 else ["dynloop", "static"]):
            os.environ["SRHIP_JIT_DYNLOOP"] = "0" if m == "static" else "1"
            for _ in range(2):
                prog.eval_loss_grad(ds, K.LOSS["L2"])
                ks[m].append(ctx.last_kernel_time()[0])
    print(json.dumps(dict(case="cfg5_grad_shard", **{m: round(float(np.median(v)), 3) for m, v in ks.items()})))


if __name__ == "__main__":
    main()
