"""Float64 ∂L/∂c today (forward-mode interpreter) on config #3's trees: the
4096-tree batch over 100k rows, eval_loss_grad kernel time, and the same trees
as Float32 (gradient tree code where it compiles) for scale. One JSON line."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402

CFG3 = dict(binary_operators=["+", "-", "*", "/", "^"], unary_operators=["safe_log", "safe_sqrt", "cos", "exp"])
CFG2 = dict(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])


def run(cfg, T, n=100_000, nt=4096):
    o = srhip.Options(**cfg)
    rng = np.random.default_rng(3)
    X = rng.uniform(-3, 3, (5, n)).astype(T)
    y = rng.standard_normal(n).astype(T)
    trees = srhip.random_population(nt, o, 5, T, seed=33)
    ctx = srhip.get_context(0)
    ds = srhip.DeviceDataset(ctx, X, y)
    prog = srhip.Program(ctx, srhip.flatten(trees, o, dtype=T), T)
    _, nodes, _ = prog.info()
    prog.eval_loss_grad(ds, K.LOSS["L2"])
    ks = []
    for _ in range(5):
        _, _, _, ok = prog.eval_loss_grad(ds, K.LOSS["L2"])
        ks.append(ctx.last_kernel_time()[0])
    gj = prog.grad_jit_info()
    return dict(dtype=np.dtype(T).name, ops=cfg["binary_operators"] + cfg["unary_operators"], trees=nt, rows=n,
                nodes=int(nodes), kernel_ms=float(np.median(ks)), ok=int(np.sum(ok)), grad_jit_trees=gj["ntrees"],
                node_rows_per_s=float(nodes) * n / (float(np.median(ks)) * 1e-3))


print(json.dumps([run(CFG3, np.float64), run(CFG3, np.float32), run(CFG2, np.float64), run(CFG2, np.float32)]))
