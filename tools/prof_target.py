#!/usr/bin/env python3
"""Profiling target: config #2 (4096 trees x 1M rows) evaluated K times with
tree code (MODE=jit, default) or the interpreter (MODE=interp); NTREES=512
(1024, 2048) takes every 4096/NTREES-th tree (the strong-scaling shards)."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "symbolicregression.jl_amd"))
import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402

mode = os.environ.get("MODE", "jit")
os.environ["SRHIP_JIT"] = "0" if mode == "interp" else "1"
if mode == "jit-precise":
    os.environ["SRHIP_JIT_FAST"] = "0"
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
rng = np.random.default_rng(1)
X = rng.standard_normal((5, 1_000_000)).astype(np.float32)
y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
trees = srhip.random_population(4096, o, 5, np.float32, seed=1000)
trees = trees[::4096 // int(os.environ.get("NTREES", "4096"))]
ctx = srhip.get_context(0)
ds = srhip.DeviceDataset(ctx, X, y)
prog = srhip.Program(ctx, srhip.flatten(trees, o, dtype=np.float32), np.float32)
for _ in range(steps):
    prog.eval_loss(ds, K.LOSS["L2"])
print(mode, "kernel ms (last):", ctx.last_kernel_time())
