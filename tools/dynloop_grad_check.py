"""Hand-written gradient tree loop (sr_jit_grad_dl, default) against the
compiled one (SRHIP_JIT_DYNLOOP=0): losses, ∂L/∂c and did_succeed identical;
kernel times. Small (600 trees x 30001 rows, weighted and not), then with
`full` config #5's gradient workload (16384 trees x 20 features x the
1.25M-row shard). One JSON line per case."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402


def run(ctx, prog, ds, mode, reps):
    os.environ["SRHIP_JIT_DYNLOOP"] = mode
    try:
        ks = []
        for i in range(reps + 1):
            r = prog.eval_loss_grad(ds, K.LOSS["L2"])
            if i:
                ks.append(ctx.last_kernel_time()[0])
        return r, float(np.median(ks)), ctx.last_tree_code()
    finally:
        del os.environ["SRHIP_JIT_DYNLOOP"]


def main():
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    ctx = srhip.get_context(0)
    rng = np.random.default_rng(7)
    X = rng.standard_normal((5, 30_001)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    w = rng.uniform(0.5, 2, 30_001).astype(np.float32)
    small = srhip.random_population(600, o, 5, np.float32, seed=8)
    cases = [("small", small, X, y, None, 2), ("small_w", small, X, y, w, 2)]
    if len(sys.argv) > 1 and sys.argv[1] == "full":
        n = 1_250_000
        X5 = np.random.default_rng(5).standard_normal((20, n), dtype=np.float32)
        y5 = (np.float32(2) * np.cos(X5[3]) + X5[0] * X5[0] - np.float32(2)).astype(np.float32)
        t5 = srhip.random_population(16384, o, 20, np.float32, seed=5)
        cases.append(("cfg5_shard", t5, X5, y5, None, 3))
    for name, trees, Xc, yc, wc, reps in cases:
        ds = srhip.DeviceDataset(ctx, Xc, yc, wc)
        prog = srhip.Program(ctx, srhip.flatten(trees, o, dtype=np.float32), np.float32)
        r0, k0, n0 = run(ctx, prog, ds, "0", reps)
        r1, k1, n1 = run(ctx, prog, ds, "1", reps)
        same = all(np.array_equal(np.asarray(a), np.asarray(b), equal_nan=True) for a, b in zip(r0, r1))
        print(json.dumps(dict(case=name, trees=len(trees), identical=bool(same), static_ms=round(k0, 3),
                              dynloop_ms=round(k1, 3), tree_code=[n0, n1])), flush=True)
        if not same:
            sys.exit(1)


if __name__ == "__main__":
    main()
