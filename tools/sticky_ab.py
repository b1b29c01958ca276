"""Interleaved A/B of sticky PRECISE per tree (SRHIP_JIT_STICKY_TREE=1: a
tree redone PRECISE in one row group runs PRECISE in the later ones) on
config #2 and its N = 8 shards; did_succeed identical and losses within 1e-6
of each other across the modes (PRECISE is the reference's value). After a
warm-up, rounds of 5 calls per mode; median kernel ms, redone tiles."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402
from srhip.distributed import shard_trees  # noqa: E402

MODES = {"sticky0": "0", "sticky1": "1"}


def main():
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    ctx = srhip.get_context(0)
    rng = np.random.default_rng(1)
    X = rng.standard_normal((5, 1_000_000)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    trees = srhip.random_population(4096, o, 5, np.float32, seed=1000, maxsize=30)
    if len(sys.argv) > 2 and sys.argv[2] == "sizes":  # the row-count crossover
        cases = [(f"rows{n}", trees, np.ascontiguousarray(X[:, :n]), y[:n].copy())
                 for n in (30_000, 100_000, 250_000, 500_000)]
    else:
        cases = [("cfg2", trees, X, y), ("shard0of8", [trees[i] for i in shard_trees(4096, 0, 8)], X, y),
                 ("rows8", trees, np.ascontiguousarray(X[:, :125_000]), y[:125_000].copy())]
    for name, tr, Xc, yc in cases:
        ds = srhip.DeviceDataset(ctx, Xc, yc)
        prog = srhip.Program(ctx, srhip.flatten(tr, o, dtype=np.float32), np.float32)
        for _ in range(20):
            prog.eval_loss(ds, K.LOSS["L2"])
        ks = {m: [] for m in MODES}
        ref, red = None, {}
        order = list(MODES)
        for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
            for m in order[r % 3:] + order[:r % 3]:
                os.environ["SRHIP_JIT_STICKY_TREE"] = MODES[m]
                for _ in range(5):
                    s_, w_, ok_ = prog.eval_loss(ds, K.LOSS["L2"])
                    ks[m].append(ctx.last_kernel_time()[0])
                    red[m] = ctx.last_jit_events()[1]
                    if ref is None:
                        ref = (s_, ok_)
                    else:
                        with np.errstate(invalid="ignore", divide="ignore"):
                            rel = np.abs(s_[ok_] - ref[0][ok_]) / np.abs(ref[0][ok_])
                        if not np.array_equal(ok_, ref[1]) or np.nanmax(rel, initial=0) > 1e-5:
                            print(json.dumps(dict(case=name, mode=m, mismatch=float(np.nanmax(rel, initial=0)))))
                            sys.exit(1)
        print(json.dumps(dict(case=name, redone=red, **{m: round(float(np.median(v)), 4) for m, v in ks.items()},
                              spread={m: round(float(np.percentile(v, 90) - np.percentile(v, 10)), 4)
                                      for m, v in ks.items()})), flush=True)


if __name__ == "__main__":
    main()
