#!/usr/bin/env python3
"""Config #2 through the tree compiler: code size, build time, per-pass
kernel times (SRHIP_DEBUG_PASSES), trees handed back, tiles redone with the
PRECISE routines. Usage: python3 tools/jit_diag.py [ntrees] [rows]"""
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "symbolicregression.jl_amd"))
os.environ.setdefault("SRHIP_DEBUG_PASSES", "1")
import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402

nt = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
rng = np.random.default_rng(1)
X = rng.standard_normal((5, n)).astype(np.float32)
y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
trees = srhip.random_population(nt, o, 5, np.float32, seed=1000)
ctx = srhip.get_context(0)
ds = srhip.DeviceDataset(ctx, X, y)
flat = srhip.flatten(trees, o, dtype=np.float32)
for mode in (os.environ.get("MODES", "jit,jit-precise,interp")).split(","):
    os.environ["SRHIP_JIT"] = "0" if mode == "interp" else "1"
    os.environ["SRHIP_JIT_FAST"] = "0" if mode == "jit-precise" else "1"
    t0 = time.perf_counter()
    prog = srhip.Program(ctx, flat, np.float32)
    t1 = time.perf_counter()
    print(f"== {mode}: program create {1e3 * (t1 - t0):.1f} ms, jit {prog.jit_info()}", flush=True)
    for it in range(3):
        prog.eval_loss(ds, K.LOSS["L2"])
        ms, nl = ctx.last_kernel_time()
        print(f"   eval {it}: kernels {ms:.3f} ms in {nl} launches, handed back / redone tiles "
              f"{ctx.last_jit_events()}", flush=True)
    del prog
