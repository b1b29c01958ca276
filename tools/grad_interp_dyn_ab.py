"""Forward-mode gradient interpreter (grad_kernels.hip): items dealt from an
LDS counter (default) against round-robin (SRHIP_INTERP_DYN=0), interleaved;
losses, ∂L/∂c and did_succeed bit for bit. SRHIP_GJIT=0 keeps every tree in
the interpreter. Float32 (1024 trees x 100k rows) and Float64 (config #3's
operator set, 1024 trees x 100k rows)."""
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
    os.environ["SRHIP_GJIT"] = "0"
    ctx = srhip.get_context(0)
    o2 = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    o3 = srhip.Options(binary_operators=["+", "-", "*", "/", "^"], unary_operators=["safe_log", "safe_sqrt", "cos", "exp"])
    rng = np.random.default_rng(4)
    X = rng.uniform(-3, 3, (5, 100_000))
    y = np.cos(X[3]) * 2 + X[0] ** 2 - 2
    for name, o, T in (("f32", o2, np.float32), ("f64", o3, np.float64)):
        trees = srhip.random_population(1024, o, 5, T, seed=11)
        ds = srhip.DeviceDataset(ctx, X.astype(T), y.astype(T))
        prog = srhip.Program(ctx, srhip.flatten(trees, o, dtype=T), T)
        prog.eval_loss_grad(ds, K.LOSS["L2"])
        ks, res = {"0": [], "1": []}, {}
        for r in range(4):
            for m in (("0", "1") if r % 2 == 0 else ("1", "0")):
                os.environ["SRHIP_INTERP_DYN"] = m
                for _ in range(2):
                    res[m] = prog.eval_loss_grad(ds, K.LOSS["L2"])
                    ks[m].append(ctx.last_kernel_time()[0])
        same = all(np.array_equal(np.asarray(a), np.asarray(b), equal_nan=True) for a, b in zip(res["0"], res["1"]))
        print(json.dumps(dict(case=name, identical=bool(same), tree_code=ctx.last_tree_code(),
                              static_ms=round(float(np.median(ks["0"])), 3),
                              dyn_ms=round(float(np.median(ks["1"])), 3))), flush=True)
        if not same:
            sys.exit(1)


if __name__ == "__main__":
    main()
