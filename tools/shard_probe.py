"""Strong scaling at N = 8 from one GPU: the
config #2 batch (bench.py's 4096 trees, 1M rows) against its eight 512-tree
shards, under two partitions:
  strided  rank r takes trees r, r+8, ... (srhip.distributed.shard_trees,
           what bench.py --gpus 8 runs);
  balanced trees dealt to the shard with the least estimated cost so far,
           most expensive first (LPT), cost = the tree's VALU estimate
           (nodes weighted by operator: srhip.distributed.tree_cost).
Per shard: kernel time (HIP events, median of K calls) and node count. The
N = 8 step is the slowest shard, so the projected speedup is
t(4096) / max_r t(shard r). Row shards (every tree on n/N rows, N = 2, 4,
8; the N > 1 step adds an all-reduce of the per-tree partials) are timed too.
Prints one JSON line."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402
from srhip.distributed import shard_trees, shard_trees_balanced  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    world = 8
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(1)
    X = rng.standard_normal((5, 1_000_000)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    trees = srhip.random_population(4096, o, 5, np.float32, seed=1000, maxsize=30)
    ctx = srhip.get_context(0)
    ds = srhip.DeviceDataset(ctx, X, y)

    def timed(sub, ds=ds):
        prog = srhip.Program(ctx, srhip.flatten(sub, o, dtype=np.float32), np.float32)
        _, nodes, _ = prog.info()
        ks, walls = [], []
        import time
        for i in range(steps + 2):
            t0 = time.perf_counter()
            prog.eval_loss(ds, K.LOSS["L2"])
            w = (time.perf_counter() - t0) * 1e3
            if i >= 2:
                ks.append(ctx.last_kernel_time()[0])
                walls.append(w)
        redone = ctx.last_jit_events()[1]
        return dict(trees=len(sub), nodes=int(nodes), kernel_ms=float(np.median(ks)), wall_ms=float(np.median(walls)),
                    redone_tiles=int(redone))

    full = timed(trees)
    out = dict(tool="shard_probe", full=full)
    for name, part in (("strided", lambda r: shard_trees(len(trees), r, world)),
                       ("balanced", lambda r: shard_trees_balanced(trees, o, r, world))):
        shards = [timed([trees[i] for i in part(r)]) for r in range(world)]
        mx = max(s["wall_ms"] for s in shards)
        out[name] = dict(shards=shards, max_wall_ms=mx, max_kernel_ms=max(s["kernel_ms"] for s in shards),
                         projected_speedup_wall=full["wall_ms"] / mx)
    # the same strided shards with every tile PRECISE (SRHIP_JIT_FAST=0, read
    # per call): if their spread goes, it came from the tiles redone PRECISE
    import os
    os.environ["SRHIP_JIT_FAST"] = "0"
    try:
        full_p = timed(trees)
        shards = [timed([trees[i] for i in shard_trees(len(trees), r, world)]) for r in range(world)]
    finally:
        del os.environ["SRHIP_JIT_FAST"]
    mx = max(s["wall_ms"] for s in shards)
    out["strided_precise"] = dict(full=full_p, shards=shards, max_wall_ms=mx,
                                  min_wall_ms=min(s["wall_ms"] for s in shards),
                                  projected_speedup_wall=full_p["wall_ms"] / mx)
    # row shards: every tree on rows [r n/N, (r+1) n/N) (the partials then
    # all-reduced: one [Σ, failed] pair per tree + Σw, 64 KiB at 4096 trees)
    n = X.shape[1]
    rows_out = {}
    for N in (2, 4, 8):
        rs = range(N) if N == 8 else (0,)
        sh = []
        for r in rs:
            rb, re = r * n // N, (r + 1) * n // N
            dsr = srhip.DeviceDataset(ctx, np.ascontiguousarray(X[:, rb:re]), np.ascontiguousarray(y[rb:re]))
            sh.append(timed(trees, dsr))
            del dsr
        mx = max(s["wall_ms"] for s in sh)
        rows_out[str(N)] = dict(shards=sh, max_wall_ms=mx, max_kernel_ms=max(s["kernel_ms"] for s in sh),
                                projected_speedup_wall_no_allreduce=full["wall_ms"] / mx)
    out["rows"] = rows_out
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
