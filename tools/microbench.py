"""Per-operator cost attribution: eval_loss kernel time for 4096 random trees
over the given rows with different operator sets."""
import sys, time, json
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd")]
import numpy as np
import srhip
from srhip import constants as K

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
only = sys.argv[2] if len(sys.argv) > 2 else None  # run one config (for PMC passes)
ctx = srhip.get_context(0)
X = np.random.default_rng(1).standard_normal((5, rows)).astype(np.float32)
y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
ds = srhip.DeviceDataset(ctx, X, y)
configs = {
    "+-*": (["+", "-", "*"], []),
    "+-*/": (["+", "-", "*", "/"], []),
    "+-*|neg": (["+", "-", "*"], ["neg"]),
    "+-*|cos": (["+", "-", "*"], ["cos"]),
    "+-*|exp": (["+", "-", "*"], ["exp"]),
    "cfg2 +-*/|cos,exp": (["+", "-", "*", "/"], ["cos", "exp"]),
    "full +-*/|cos,exp,tanh": (["+", "-", "*", "/"], ["cos", "exp", "tanh"]),
}
res = {}
for name, (b, u) in configs.items():
    if only and name != only:
        continue
    o = srhip.Options(binary_operators=b, unary_operators=u)
    trees = srhip.random_population(4096, o, 5, np.float32, seed=1000)
    prog = srhip.Program(ctx, srhip.flatten(trees, o, np.float32), np.float32)
    _, nodes, _ = prog.info()
    prog.eval_loss(ds, K.LOSS["L2"])
    ms = []
    for _ in range(3):
        s, w, ok = prog.eval_loss(ds, K.LOSS["L2"])
        ms.append(ctx.last_kernel_time()[0])
    kms = float(np.median(ms))
    res[name] = dict(kernel_ms=kms, nodes=int(nodes), node_rows_per_s=nodes * rows / (kms * 1e-3), ok=float(ok.mean()))
    print(name, json.dumps(res[name]), flush=True)
json.dump(res, open(ROOT / "gpurun_out" / "microbench.json", "w"), indent=1)
