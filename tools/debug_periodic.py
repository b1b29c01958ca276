"""Float32 Periodic loss inside the gradient tree code vs the forward-mode
interpreter (GPU box): the worst trees' loss sums, with a host check of a
few rows (one-off debugging aid for device_ops.h periodic_g_f32)."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

import srhip  # noqa: E402

o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
rng = np.random.default_rng(71)
n = 4001
X = rng.standard_normal((5, n)).astype(np.float32)
y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
trees = [srhip.Node("x1"), o.make_binary("-", srhip.Node("x2"), srhip.Node(val=np.float32(0.5)))]
trees += srhip.random_population(300, o, 5, np.float32, seed=72)
flat = srhip.flatten(trees, o, dtype=np.float32)
loss = srhip.PeriodicLoss(2.0)
ctx = srhip.get_context(0)
ds = srhip.DeviceDataset(ctx, X, y)
res = {}
for mode in ("1", "0"):
    os.environ["SRHIP_GJIT"] = mode
    prog = srhip.Program(ctx, flat, np.float32)
    res[mode] = [np.array(v, copy=True) for v in prog.eval_loss_grad(ds, loss.kind, loss.params)]
    print(mode, "tree code", ctx.last_tree_code())
s1, g1, _, ok1 = res["1"]
s0, g0, _, ok0 = res["0"]
r = (X[1] - y).astype(np.float64)
k = 2 * np.pi / 2.0
print("tree x1: host", float(np.sum(1 - np.cos(k * r))), "code", s1[0], "interp", s0[0])
print("grad of x2-0.5: code", g1[0:2], "interp", g0[0:2])
rel = np.abs(s1 - s0) / np.abs(s0)
for t in np.argsort(-np.nan_to_num(rel))[:5]:
    print(t, rel[t], s1[t], s0[t], srhip.string_tree(trees[t], o))
