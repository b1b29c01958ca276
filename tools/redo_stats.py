"""Config #2 (bench.py's batch): tiles the tree code redid with the PRECISE
routines, trees that failed, and the kernel time with the FAST path on / off."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "symbolicregression.jl_amd"))
import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402

o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
rng = np.random.default_rng(1)
n = 1_000_000
X = rng.standard_normal((5, n)).astype(np.float32)
y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
trees = srhip.random_population(4096, o, 5, np.float32, seed=1000, maxsize=30)
ctx = srhip.get_context(0)
ds = srhip.DeviceDataset(ctx, X, y)
flat = srhip.flatten(trees, o, dtype=np.float32)
for fast in ("1", "0"):
    os.environ["SRHIP_JIT_FAST"] = fast
    p = srhip.Program(ctx, flat, np.float32)
    for _ in range(3):
        s, w, ok = p.eval_loss(ds, K.LOSS["L2"])
    ms = []
    for _ in range(10):
        p.eval_loss(ds, K.LOSS["L2"])
        ms.append(ctx.last_kernel_time()[0])
    bailed, redone = ctx.last_jit_events()
    info = p.jit_info()
    print(f"FAST={fast}: kernel {np.median(ms):.3f} ms, trees ok {int(ok.sum())}/{len(ok)}, "
          f"tiles redone {redone} of {info['ntrees'] * (n // 256)} tree-tiles, bailed {bailed}, nfast {info['nfast']}")
