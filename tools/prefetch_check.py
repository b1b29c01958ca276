"""[prefetch_check: the same cases, three loops: compiled static (DYNLOOP=0),
hand-written (DYNLOOP=1), hand-written with the next tree's flag and code
offset prefetched (SRHIP_JIT_PREFETCH=1, sr_jit_eval_dlp).]
Hand-written tree loop (SRHIP_JIT_DYNLOOP=1, sr_jit_eval_dl) against the
compiled static loop on the same programs: losses, did_succeed and the
tree-code events must be identical (the loop sums each tree's wave in
wave_sum's order). Small first (600 trees x 30001 rows, weighted and not),
then config #2's 4096 trees x 1M rows and a 512-tree shard, with kernel times.
One JSON line per case."""
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


def run(ctx, prog, ds, mode, reps):
    os.environ["SRHIP_JIT_DYNLOOP"] = mode[0]  # "0": the static loop
    os.environ["SRHIP_JIT_PREFETCH"] = mode[1:] or "0"
    try:
        ks = []
        for i in range(reps + 1):
            s, w, ok = prog.eval_loss(ds, K.LOSS["L2"])
            if i:
                ks.append(ctx.last_kernel_time()[0])
        return s, w, ok, float(np.median(ks)), list(ctx.last_jit_events())
    finally:
        del os.environ["SRHIP_JIT_DYNLOOP"]
        del os.environ["SRHIP_JIT_PREFETCH"]


def main():
    os.environ["SRHIP_JIT_STICKY_TREE"] = "0"  # bit-identity needs the same FAST / PRECISE choices per tile
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    ctx = srhip.get_context(0)
    rng = np.random.default_rng(5)
    cases = []
    X = rng.standard_normal((5, 30_001)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    w = rng.uniform(0.5, 2, 30_001).astype(np.float32)
    small = srhip.random_population(600, o, 5, np.float32, seed=4)
    cases.append(("small", small, X, y, None, 3))
    cases.append(("small_w", small, X, y, w, 3))
    cases.append(("small_memc", small, X, y, None, 3))
    cases.append(("small_memc_w", small, X, y, w, 3))
    if len(sys.argv) > 1 and sys.argv[1] == "full":
        rng = np.random.default_rng(1)
        Xf = rng.standard_normal((5, 1_000_000)).astype(np.float32)
        yf = (np.float32(2) * np.cos(Xf[3]) + Xf[0] * Xf[0] - np.float32(2)).astype(np.float32)
        trees = srhip.random_population(4096, o, 5, np.float32, seed=1000, maxsize=30)
        cases.append(("cfg2", trees, Xf, yf, None, 10))
        cases.append(("shard0of8", [trees[i] for i in shard_trees(4096, 0, 8)], Xf, yf, None, 10))
        cases.append(("rows8", trees, np.ascontiguousarray(Xf[:, :125_000]), yf[:125_000].copy(), None, 10))
    for name, trees, Xc, yc, wc, reps in cases:
        ds = srhip.DeviceDataset(ctx, Xc, yc, wc)
        os.environ["SRHIP_JIT"] = "1"
        try:  # *_memc: memory-constant tree code (sr_jit_eval_dlm), new constants set in place
            memc = "memc" in name
            prog = srhip.Program(ctx, srhip.flatten(trees, o, dtype=np.float32), np.float32, varying_constants=memc)
            if memc:
                c = prog.flat.consts.astype(np.float32)
                prog.set_constants((c * np.float32(1.01) + np.float32(0.002)).astype(np.float32))
        finally:
            del os.environ["SRHIP_JIT"]
        s0, w0, ok0, k0, e0 = run(ctx, prog, ds, "1", reps)
        s1, w1, ok1, k1, e1 = run(ctx, prog, ds, "11", reps)
        s2, w2, ok2, k2, e2 = run(ctx, prog, ds, "0", reps)
        same = bool(np.array_equal(ok0, ok1) and np.array_equal(s0[ok0], s1[ok1]) and w0 == w1 and
                    np.array_equal(ok0, ok2) and np.array_equal(s0[ok0], s2[ok2]))
        print(json.dumps(dict(case=name, trees=len(trees), identical=same, dynloop_ms=round(k0, 4),
                              prefetch_ms=round(k1, 4), static_ms=round(k2, 4),
                              ok=int(ok0.sum()), ntree_code=prog.jit_info()["ntrees"])), flush=True)
        if not same:
            d = np.flatnonzero((ok0 != ok1) | (ok0 & (s0 != s1)))
            print(json.dumps(dict(first_diff=d[:10].tolist(), s0=s0[d[:5]].tolist(), s1=s1[d[:5]].tolist())), flush=True)
            sys.exit(1)


if __name__ == "__main__":
    main()
