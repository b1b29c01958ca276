"""Why some 512-tree shards of config #2 run at their all-PRECISE speed
(profiles/r04_shard_probe_b.json: shards 2, 3, 5 report 0 redone tiles):
per strided shard, the tree code's FAST count (jit_info nfast), the last
call's tree-code events (bailed trees, redone tiles) and the kernel time with
the FAST path on and off. One JSON line per shard."""
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
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(1)
    X = rng.standard_normal((5, 1_000_000)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    trees = srhip.random_population(4096, o, 5, np.float32, seed=1000, maxsize=30)
    ctx = srhip.get_context(0)
    ds = srhip.DeviceDataset(ctx, X, y)
    for r in list(range(8)) + ["full"]:
        sub = trees if r == "full" else [trees[i] for i in shard_trees(len(trees), r, 8)]
        prog = srhip.Program(ctx, srhip.flatten(sub, o, dtype=np.float32), np.float32)
        rec = dict(shard=r, jit=prog.jit_info())
        for fast in ("1", "0"):
            os.environ["SRHIP_JIT_FAST"] = fast
            ks = []
            for i in range(8):
                prog.eval_loss(ds, K.LOSS["L2"])
                if i >= 2:
                    ks.append(ctx.last_kernel_time()[0])
            rec["fast" + fast] = dict(kernel_ms=round(float(np.median(ks)), 4), events=list(ctx.last_jit_events()),
                                      tree_code=ctx.last_tree_code())
        del os.environ["SRHIP_JIT_FAST"]
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
