"""The README usage example, run as-is (GPU)."""
import sys; sys.path.insert(0, "symbolicregression.jl_amd")
import numpy as np, srhip
o = srhip.Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp"])
X = np.random.randn(5, 100).astype(np.float32); y = 2 * np.cos(X[3]) + X[0] ** 2 - 2
ds = srhip.Dataset(X, y)
trees = srhip.random_population(1000, o, 5, np.float32)
losses, ok = srhip.eval_loss_batch_ok(trees, ds, o)          # one launch, fused L2
out, ok1 = srhip.eval_tree_array(trees[0], X, o)              # per-row outputs
val, dydx, ok2 = srhip.eval_grad_tree_array(trees[0], X, o, variable=True)
res = srhip.optimize_constants_batch(ds, trees[:100], o)      # batched BFGS on the device
hof, stats = srhip.equation_search(X, y, o, niterations=5)    # lockstep islands
print("losses", losses[:3], "ok", ok.mean(), "hof", len(hof.dominating()), stats["seconds"])
