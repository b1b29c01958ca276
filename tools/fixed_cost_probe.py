"""Where the fixed per-call cost of the shard sizes comes from (VERDICT r04
next 4): the config #2 batch (4096 trees, seed 1000, as bench.py) and a 512-tree
strided shard, over 1M / 500k / 250k / 125k rows, each timed
  default   the product path
  ok_only   the trees that succeed on the 1M rows only (the failing trees'
            work until their row groups skip them is per launch, not per row)
  precise   every tile PRECISE (SRHIP_JIT_FAST=0: no redone tiles)
  gcols0    no shared-subtree columns (SRHIP_JIT_GCOLS=0: no derive pass)
Kernel time = median HIP-event time of K calls. One JSON line per case plus
the least-squares fit kernel_ms = a + b·rows per (set, variant)."""
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
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(1)
    X = rng.standard_normal((5, 1_000_000)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    trees = srhip.random_population(4096, o, 5, np.float32, seed=1000, maxsize=30)
    ctx = srhip.get_context(0)
    dss = {n: srhip.DeviceDataset(ctx, np.ascontiguousarray(X[:, :n]), y[:n]) for n in
           (1_000_000, 500_000, 250_000, 125_000, 62_500)}

    def timed(sub, ds):
        prog = srhip.Program(ctx, srhip.flatten(sub, o, dtype=np.float32), np.float32)
        ks = []
        ok = None
        for i in range(steps + 2):
            _, _, ok = prog.eval_loss(ds, K.LOSS["L2"])
            if i >= 2:
                ks.append(ctx.last_kernel_time()[0])
        return float(np.median(ks)), int(ctx.last_jit_events()[1]), np.asarray(ok, dtype=bool), ctx.last_kernel_name()

    _, _, ok_full, _ = timed(trees, dss[1_000_000])
    shard = [trees[i] for i in shard_trees(len(trees), 0, 8)]
    sets = {"4096": trees, "4096_ok": [t for t, k in zip(trees, ok_full) if k],
            "512": shard, "512_ok": [trees[i] for i in shard_trees(len(trees), 0, 8) if ok_full[i]]}
    only = os.environ.get("FIXED_SETS")  # e.g. "4096,4096_ok"
    if only:
        sets = {k: v for k, v in sets.items() if k in only.split(",")}
    fits = {}
    for name, sub in sets.items():
        for variant in ("default", "precise", "gcols0"):
            if variant == "precise":
                os.environ["SRHIP_JIT_FAST"] = "0"
            if variant == "gcols0":  # no shared-subtree columns (read per build)
                os.environ["SRHIP_JIT_GCOLS"] = "0"
            pts = []
            try:
                for n, ds in dss.items():
                    t0 = time.perf_counter()
                    ms, redone, _, kern = timed(sub, ds)
                    rec = dict(tool="fixed_cost_probe", set=name, variant=variant, trees=len(sub), rows=n,
                               kernel_ms=ms, redone_tiles=redone, kernel=kern,
                               wall_s=time.perf_counter() - t0)
                    print(json.dumps(rec), flush=True)
                    pts.append((n, ms))
            finally:
                os.environ.pop("SRHIP_JIT_FAST", None)
                os.environ.pop("SRHIP_JIT_GCOLS", None)
            r = np.asarray([p[0] for p in pts], dtype=float)
            t = np.asarray([p[1] for p in pts])
            b, a = np.polyfit(r, t, 1)
            fits[f"{name}/{variant}"] = dict(a_ms=float(a), b_ms_per_Mrow=float(b * 1e6),
                                             share_fixed_at_125k=float(a / (a + b * 125_000)),
                                             share_fixed_at_1M=float(a / (a + b * 1e6)))
    print(json.dumps(dict(tool="fixed_cost_probe", fits=fits)), flush=True)


if __name__ == "__main__":
    main()
