"""Interpreter kernels: trees dealt from an LDS counter (SRHIP_INTERP_DYN=1)
against round-robin (0), interleaved in one process; sums and did_succeed
bit for bit. Workloads (all interpreted, SRHIP_JIT=0): config #2's 4096 trees
x 1M rows (Float32), config #3's 4096 NaN-heavy trees x 100k rows (Float64),
and a search-sized batch (300 trees x 100k rows). One JSON line each, with
the library path (SRHIP_LIB) so runs of two builds can be compared."""
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
    ctx = srhip.get_context(0)
    o2 = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    o3 = srhip.Options(binary_operators=["+", "-", "*", "/", "^"], unary_operators=["safe_log", "safe_sqrt", "cos", "exp"])
    rng = np.random.default_rng(1)
    X2 = rng.standard_normal((5, 1_000_000)).astype(np.float32)
    y2 = (np.float32(2) * np.cos(X2[3]) + X2[0] * X2[0] - np.float32(2)).astype(np.float32)
    X3 = rng.uniform(-3, 3, (5, 100_000))
    y3 = np.cos(X3[3]) * 2 + X3[0] ** 2 - 2
    cases = [("cfg2_interp", srhip.random_population(4096, o2, 5, np.float32, seed=1000, maxsize=30), o2, X2, y2, np.float32),
             ("cfg3_interp", srhip.random_population(4096, o3, 5, np.float64, seed=3), o3, X3, y3, np.float64),
             ("batch300", srhip.random_population(300, o2, 5, np.float32, seed=7), o2,
              np.ascontiguousarray(X2[:, :100_000]), y2[:100_000].copy(), np.float32)]
    mode = os.environ.get("AB_MODES", "01")
    for name, trees, o, X, y, T in cases:
        ds = srhip.DeviceDataset(ctx, X, y)
        os.environ["SRHIP_JIT"] = "0"
        prog = srhip.Program(ctx, srhip.flatten(trees, o, dtype=T), T)
        del os.environ["SRHIP_JIT"]
        for _ in range(5):
            prog.eval_loss(ds, K.LOSS["L2"])
        ks = {m: [] for m in mode}
        res = {}
        for r in range(6):
            for m in (mode if r % 2 == 0 else mode[::-1]):
                os.environ["SRHIP_INTERP_DYN"] = m
                for _ in range(4):
                    res[m] = prog.eval_loss(ds, K.LOSS["L2"])
                    ks[m].append(ctx.last_kernel_time()[0])
        ok = all(np.array_equal(res[m][2], res[mode[0]][2]) and
                 np.array_equal(res[m][0][res[m][2]], res[mode[0]][0][res[mode[0]][2]]) for m in mode)
        print(json.dumps(dict(case=name, lib=os.environ.get("SRHIP_LIB", "default"), identical=bool(ok),
                              **{"dyn" + m: round(float(np.median(v)), 4) for m, v in ks.items()})), flush=True)
        if not ok:
            sys.exit(1)


if __name__ == "__main__":
    main()
