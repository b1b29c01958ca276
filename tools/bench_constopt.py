"""Batched constant optimisation throughput: one
optimize_constants_batch call over a random population, 8 BFGS iterations,
1 + 2 starts per tree (the reference defaults). Prints one JSON line.
Usage: bench_constopt.py [ntrees] [rows] [f32|f64] [cfg2|cfg3] (cfg3: config
#3's operators on X ~ U(-3, 3), NaN-heavy)."""
import json, sys, time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "symbolicregression.jl_amd"))
import srhip  # noqa: E402

ntrees = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
dt_ = np.float64 if (len(sys.argv) > 3 and sys.argv[3] == "f64") else np.float32
cfg = sys.argv[4] if len(sys.argv) > 4 else "cfg2"
nfeat = 10
if cfg == "cfg3":
    o = srhip.Options(binary_operators=["+", "-", "*", "/", "^"], unary_operators=["safe_log", "safe_sqrt", "cos", "exp"])
else:
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
rng = np.random.default_rng(1)
X = (rng.uniform(-3, 3, (nfeat, rows)) if cfg == "cfg3" else rng.standard_normal((nfeat, rows))).astype(dt_)
y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(dt_)
ds = srhip.Dataset(X, y)
trees = srhip.random_population(ntrees, o, nfeat, dt_, seed=0)
srhip.optimize_constants_batch(ds, trees[:64], o, rng=np.random.default_rng(0))  # warm-up
trees = srhip.random_population(ntrees, o, nfeat, dt_, seed=0)
before = srhip.eval_loss_batch(trees, ds, o)
t0 = time.perf_counter()
res = srhip.optimize_constants_batch(ds, trees, o, rng=np.random.default_rng(0))
dt = time.perf_counter() - t0
from srhip.constant_optimization import last_profile  # noqa: E402
prof = last_profile()
m = np.isfinite(before)
print(json.dumps({
    "tool": "bench_constopt", "ntrees": ntrees, "rows": rows, "nfeat": nfeat, "dtype": np.dtype(dt_).name,
    "ops": cfg, "seconds": dt,
    "trees_per_s": ntrees / dt, "loss_evals": float(res.num_evals.sum()),
    "loss_evals_x_rows_per_s": float(res.num_evals.sum()) * rows / dt,
    "converged": int(res.converged.sum()),
    "improved": int((res.losses[m] < before[m]).sum()), "finite_before": int(m.sum()),
    "profile": prof,
}))
