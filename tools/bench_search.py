"""Config #4 shape: equation_search with islands in lockstep,
10 features x 100k rows F32. Args: islands, cycles per iteration, iterations.
Prints one JSON line: evals/s, s/iteration, and the share of wall time spent
inside engine calls (the rest is host-side mutation bookkeeping)."""
import json, sys, time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "symbolicregression.jl_amd"))
import srhip  # noqa: E402

islands = int(sys.argv[1]) if len(sys.argv) > 1 else 64
cycles = int(sys.argv[2]) if len(sys.argv) > 2 else 100
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 1
rows, nfeat = 100_000, 10
rng = np.random.default_rng(0)
X = rng.standard_normal((nfeat, rows)).astype(np.float32)
y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
o = srhip.Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp"], npopulations=islands)
o.ncycles_per_iteration = cycles
ds = srhip.Dataset(X, y)
engine_s = [0.0]


def scorer(trees):
    t0 = time.perf_counter()
    out = srhip.eval_loss_batch(trees, ds, o)
    engine_s[0] += time.perf_counter() - t0
    return out


srhip.equation_search(X, y, o, niterations=1, seed=0, scorer=scorer)  # warm-up (engine init, kernels)
engine_s[0] = 0.0
hof, st = srhip.equation_search(X, y, o, niterations=iters, seed=1, scorer=scorer)
best = min(m.loss for m in hof.dominating())
print(json.dumps({"tool": "bench_search", "islands": islands, "cycles_per_iteration": cycles, "iterations": iters,
                  "rows": rows, "nfeat": nfeat, "seconds": st["seconds"], "evals": st["evals"],
                  "evals_per_s": st["evals_per_s"], "seconds_per_iteration": st["seconds_per_iteration"],
                  "launches": st["launches"], "engine_share": engine_s[0] / st["seconds"], "best_loss": best}))
