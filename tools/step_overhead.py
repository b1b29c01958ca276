"""Per-call host overhead of eval_loss: wall time per call vs the kernel time,
for the strong-scaling shard sizes of config #2 (4096/N trees x 1M rows) and a
tiny problem (pure overhead)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "symbolicregression.jl_amd"))
import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402

o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
ctx = srhip.get_context(0)
for nt, n in ((4096, 1_000_000), (2048, 1_000_000), (1024, 1_000_000), (512, 1_000_000), (512, 2048)):
    rng = np.random.default_rng(1)
    X = rng.standard_normal((5, n)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    trees = srhip.random_population(4096, o, 5, np.float32, seed=1000, maxsize=30)[: nt * (4096 // nt):(4096 // nt)]
    ds = srhip.DeviceDataset(ctx, X, y)
    p = srhip.Program(ctx, srhip.flatten(trees, o, dtype=np.float32), np.float32)
    for _ in range(10):
        p.eval_loss(ds, K.LOSS["L2"])
    ctx.sync()
    ks = []
    t = time.perf_counter()
    for _ in range(50):
        p.eval_loss(ds, K.LOSS["L2"])
        ks.append(ctx.last_kernel_time()[0])
    wall = (time.perf_counter() - t) / 50 * 1e3
    print(f"{nt:5d} trees x {n:8d} rows: {wall:.3f} ms per call, kernel {np.mean(ks):.3f} ms, host+other {wall - np.mean(ks):.3f} ms")
