#!/usr/bin/env python3
"""Profiling target: config #5's gradient workload — eval_loss_grad (∂L/∂c of
every constant) of 16384 trees (20 features) over the 1.25M-row shard one of
8 GPUs holds, K times; prints node·row/s from the HIP-event kernel times."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "symbolicregression.jl_amd"))
import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
nt = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
rows = 1_250_000
o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
rng = np.random.default_rng(5)
X = rng.standard_normal((20, rows), dtype=np.float32)
y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
trees = srhip.random_population(nt, o, 20, np.float32, seed=5)
ctx = srhip.get_context(0)
prog = srhip.Program(ctx, srhip.flatten(trees, o, np.float32), np.float32)
_, nodes, _ = prog.info()
ds = srhip.DeviceDataset(ctx, X, y)
prog.eval_loss_grad(ds, K.LOSS["L2"])
ks = []
for _ in range(steps):
    prog.eval_loss_grad(ds, K.LOSS["L2"])
    ks.append(ctx.last_kernel_time())
k_ms = float(np.median([k[0] for k in ks]))
print(json.dumps({"tool": "prof_grad", "trees": nt, "rows": rows, "nodes": int(nodes), "grad_jit": prog.grad_jit_info(),
                  "constants": int(prog.flat.const_off[-1]), "kernel_ms": k_ms, "launches": ks[-1][1],
                  "node_rows_per_s": nodes * rows / (k_ms * 1e-3)}))
