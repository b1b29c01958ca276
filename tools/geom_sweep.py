"""Tree-code launch geometry at shard sizes: the config
#2 trees on a row shard (rows = 1M / N) or a tree shard (every N-th tree on
1M rows), timed under the geometry knobs of the environment (SRHIP_TARGET_WG,
SRHIP_MIN_PER_GROUP, SRHIP_TREE_NT, SRHIP_EVAL_LDS, SRHIP_JIT_TAIL; read once
per process, so tools/gpu_geom.sh runs one process per setting). Prints one
JSON line: kernel and wall ms (medians) and the grid (SRHIP_DEBUG_PASSES)."""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402
from srhip.distributed import shard_trees  # noqa: E402


def main():
    kind, N, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(1)
    n = 1_000_000
    X = rng.standard_normal((5, n)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    trees = srhip.random_population(4096, o, 5, np.float32, seed=1000, maxsize=30)
    if kind == "rows":
        X, y = np.ascontiguousarray(X[:, : n // N]), np.ascontiguousarray(y[: n // N])
    else:
        trees = [trees[i] for i in shard_trees(len(trees), 0, N)]
    ctx = srhip.get_context(0)
    ds = srhip.DeviceDataset(ctx, X, y)
    prog = srhip.Program(ctx, srhip.flatten(trees, o, dtype=np.float32), np.float32)
    ks, walls = [], []
    for i in range(steps + 3):
        t0 = time.perf_counter()
        prog.eval_loss(ds, K.LOSS["L2"])
        w = (time.perf_counter() - t0) * 1e3
        if i >= 3:
            ks.append(ctx.last_kernel_time()[0])
            walls.append(w)
    knobs = {k: v for k, v in os.environ.items() if k.startswith("SRHIP_") and k != "SRHIP_DEBUG_PASSES"}
    print(json.dumps(dict(kind=kind, N=N, knobs=knobs, kernel_ms=round(float(np.median(ks)), 4),
                          wall_ms=round(float(np.median(walls)), 4))), flush=True)


if __name__ == "__main__":
    main()
