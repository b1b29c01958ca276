"""FAST-path loss parity at full size: for config #2
(4096 trees x 1M rows) and a config #5 sample (384 of 16384 trees over 10M
rows x 20 features), count the trees whose engine loss lies outside 1e-5
relative of the oracle, with the FAST path on and off, and price each outlier
against the oracle's perturbation spread (tests/numerics.py). Writes
gpurun_out/fast_parity.json and prints the worst trees.

Usage: python tools/fast_parity.py [cfg2|cfg5|both]
"""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402
from numerics import loss_spread  # noqa: E402

CFG = dict(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])


def workload(which):
    o = srhip.Options(**CFG)
    if which == "cfg2":
        trees = srhip.random_population(4096, o, 5, np.float32, seed=0)
        rng = np.random.default_rng(1)
        X = rng.standard_normal((5, 1_000_000)).astype(np.float32)
    else:
        rng = np.random.default_rng(51)
        X = rng.standard_normal((20, 10_000_000), dtype=np.float32)
        trees = srhip.random_population(16384, o, 20, np.float32, seed=52)
        sub = np.sort(rng.choice(16384, 384, replace=False))
        trees = [trees[i] for i in sub]
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    return o, trees, X, y


def run(which, out):
    o, trees, X, y = workload(which)
    n = X.shape[1]
    ctx = srhip.get_context(0)
    ds = srhip.DeviceDataset(ctx, X, y)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    t0 = time.time()
    _, ref_l, ref_ok = oracle.eval_loss_batch(flat, X, y, dtype=np.float32, nthreads=16)
    print(f"[{which}] oracle {time.time() - t0:.1f} s", flush=True)
    res = {}
    for mode in ("fast", "precise"):
        os.environ["SRHIP_JIT_FAST"] = "1" if mode == "fast" else "0"
        os.environ["SRHIP_JIT"] = "1"
        prog = srhip.Program(ctx, flat, np.float32)
        s, w, ok = prog.eval_loss(ds, K.LOSS["L2"])
        losses = s / n
        m = ok & ref_ok & np.isfinite(ref_l)
        with np.errstate(invalid="ignore", divide="ignore"):
            rel = np.abs(losses - ref_l.astype(np.float64)) / np.abs(ref_l.astype(np.float64))
        bad = np.flatnonzero(m & ~(rel <= 1e-5))
        r = dict(did_succeed_mismatch=int((ok != ref_ok).sum()), succeeding=int(m.sum()),
                 outside_1e5=int(bad.size), max_rel=float(np.nanmax(np.where(m, rel, 0))),
                 tree_code=prog.jit_info())
        if bad.size:
            sp = loss_spread([trees[i] for i in bad], o, X, y, None, np.float32, nperturb=3) / n
            err = np.abs(losses[bad] - ref_l[bad].astype(np.float64))
            ratio = err / np.maximum(sp, 1e-300)
            r["outliers"] = [dict(tree=int(t), rel=float(rel[t]), err_over_spread=float(q),
                                  expr=srhip.string_tree(trees[t], o))
                             for t, q in sorted(zip(bad, ratio), key=lambda z: -z[1])][:40]
            r["max_err_over_spread"] = float(ratio.max())
            r["outliers_beyond_4x_spread"] = int((ratio > 4).sum())
        res[mode] = r
        print(f"[{which}] {mode}: " + json.dumps({k: v for k, v in r.items() if k != "outliers"}), flush=True)
        for q in r.get("outliers", [])[:12]:
            print("   ", json.dumps(q), flush=True)
        del prog
    out[which] = res


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "both"
    out = {}
    for w in (["cfg2", "cfg5"] if which == "both" else [which]):
        run(w, out)
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "fast_parity.json").write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
