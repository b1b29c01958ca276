#!/usr/bin/env python3
"""Loss parity of the FAST path with and without sticky PRECISE per tree
(SRHIP_JIT_STICKY_TREE, read per launch) against the Float32 oracle on
config #2's batch at reduced row counts (GPU box; the oracle is the checker).

Prints per row count and mode: trees whose mean loss is outside 1e-5 of the
oracle's, the worst relative difference and the tiles redone.

Usage: python tools/sticky_parity.py [--rows 30000,125000] [--ntrees 4096]
       python tools/sticky_parity.py --tree 759 --rows 30000   (one tree: its
       256-row tiles against the oracle, the worst tile's rows one by one, and
       the oracle's perturbation spread of the tree's loss)
"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "symbolicregression.jl_amd"))
sys.path.insert(0, str(ROOT / "oracle"))

import oracle  # noqa: E402  (checker only)
import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="30000,47000,125000")
    ap.add_argument("--ntrees", type=int, default=4096)
    ap.add_argument("--tree", type=int, default=-1)
    ap.add_argument("--seeds", default="1000", help="batch seeds (random_population)")
    ap.add_argument("--modes", default="0,1", help="SRHIP_JIT_STICKY_TREE values; 'auto' = unset")
    a = ap.parse_args()
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(1)
    X = rng.standard_normal((5, 1_000_000)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    ctx = srhip.get_context(0)
    if a.tree >= 0:
        trees = srhip.random_population(4096, o, 5, np.float32, seed=int(a.seeds.split(",")[0]))
        return one_tree(ctx, o, trees[a.tree], X, y, int(a.rows.split(",")[0]))
    for seed, rows in [(int(sd), int(r)) for sd in a.seeds.split(",") for r in a.rows.split(",")]:
        trees = srhip.random_population(4096, o, 5, np.float32, seed=seed)[: a.ntrees]
        flat = srhip.flatten(trees, o, dtype=np.float32)
        prog = srhip.Program(ctx, flat, np.float32)
        Xr, yr = np.ascontiguousarray(X[:, :rows]), np.ascontiguousarray(y[:rows])
        ds = srhip.DeviceDataset(ctx, Xr, yr)
        _, ref_l, ref_ok = oracle.eval_loss_batch(flat, Xr, yr, None, K.LOSS["L2"], (0.0,), dtype=np.float32,
                                                  nthreads=16)
        ref_ok = ref_ok.astype(bool)
        for mode in a.modes.split(","):
            if mode == "auto":
                os.environ.pop("SRHIP_JIT_STICKY_TREE", None)
            else:
                os.environ["SRHIP_JIT_STICKY_TREE"] = mode
            s, wsum, ok = prog.eval_loss(ds, K.LOSS["L2"])
            redone = ctx.last_jit_events()[1]
            ok = np.asarray(ok, dtype=bool)
            m = ok & ref_ok & np.isfinite(ref_l) & (ref_l != 0)
            with np.errstate(invalid="ignore", divide="ignore"):
                rel = np.abs(np.asarray(s, np.float64) / wsum - ref_l) / np.abs(ref_l)
            out = np.flatnonzero(m & ~(rel <= 1e-5))
            spread = []
            if out.size:
                sys.path.insert(0, str(ROOT / "tests"))
                from numerics import loss_spread
                sp = loss_spread([trees[t] for t in out[:8]], o, Xr, yr, None, np.float32)
                spread = [float(abs(float(s[t]) / wsum - ref_l[t]) * wsum / max(sp[j], 1e-300))
                          for j, t in enumerate(out[:8])]
            print(json.dumps({"seed": seed, "rows": rows, "sticky": mode, "diff_over_spread": spread, "did_succeed_diff": int((ok != ref_ok).sum()),
                              "succeeding": int(m.sum()), "outside_1e-5": int(out.size),
                              "max_rel": float(np.max(rel[m])), "worst_trees": out[np.argsort(-rel[out])][:5].tolist(),
                              "worst_rel": sorted(rel[out].tolist(), reverse=True)[:5], "redone": int(redone)}),
                  flush=True)
        del ds
    os.environ.pop("SRHIP_JIT_STICKY_TREE", None)


def one_tree(ctx, o, tree, X, y, rows):
    sys.path.insert(0, str(ROOT / "tests"))
    from numerics import loss_spread

    print("tree:", srhip.node.string_tree(tree, o), flush=True)
    flat = srhip.flatten([tree], o, dtype=np.float32)
    os.environ["SRHIP_JIT"] = "1"  # tree code for a one-tree program (default: >= 256 trees)
    os.environ["SRHIP_JIT_FAST"] = "0"
    pprec = srhip.Program(ctx, flat, np.float32)
    os.environ["SRHIP_JIT_FAST"] = "1"
    prog = srhip.Program(ctx, flat, np.float32)
    ds = srhip.DeviceDataset(ctx, np.ascontiguousarray(X[:, :rows]), np.ascontiguousarray(y[:rows]))
    sp_, _, _ = pprec.eval_loss(ds, K.LOSS["L2"])
    print(json.dumps({"precise_tree_code_sum": float(sp_[0]), "tree_code": ctx.last_tree_code()}), flush=True)
    del ds

    def eng(Xs, ys):
        ds = srhip.DeviceDataset(ctx, np.ascontiguousarray(Xs), np.ascontiguousarray(ys))
        s, _, ok = prog.eval_loss(ds, K.LOSS["L2"])
        return float(s[0]), bool(ok[0]), ctx.last_jit_events()[1]

    def ref(Xs, ys):
        sm, _, ok = oracle.eval_loss_batch(flat, np.ascontiguousarray(Xs), np.ascontiguousarray(ys), None,
                                           K.LOSS["L2"], (0.0,), dtype=np.float32)
        return float(sm[0]), bool(ok[0])

    Xr, yr = X[:, :rows], y[:rows]
    s_all, ok_all, red = eng(Xr, yr)
    r_all, rok = ref(Xr, yr)
    sp = loss_spread([tree], o, np.ascontiguousarray(Xr), np.ascontiguousarray(yr), None, np.float32)
    print(json.dumps({"rows": rows, "engine_sum": s_all, "oracle_sum": r_all, "ok": [ok_all, rok], "redone": red,
                      "abs_diff": abs(s_all - r_all), "spread": float(sp[0])}), flush=True)
    diffs = []
    for t0 in range(0, rows, 256):
        se, _, rd = eng(Xr[:, t0:t0 + 256], yr[t0:t0 + 256])
        sr, _ = ref(Xr[:, t0:t0 + 256], yr[t0:t0 + 256])
        diffs.append((abs(se - sr), t0, se, sr, rd))
    diffs.sort(reverse=True)
    for d in diffs[:5]:
        print(json.dumps({"tile_row0": d[1], "abs_diff": d[0], "engine": d[2], "oracle": d[3], "redone": d[4]}),
              flush=True)
    t0 = diffs[0][1]
    fx, _ = oracle.eval_trees(flat, np.ascontiguousarray(Xr[:, t0:t0 + 256]).astype(np.float64), dtype=np.float64)
    rowd = []
    for r in range(t0, min(t0 + 256, rows)):
        se, _, _ = eng(Xr[:, r:r + 1], yr[r:r + 1])
        sr, _ = ref(Xr[:, r:r + 1], yr[r:r + 1])
        rowd.append((abs(se - sr), r, se, sr))
    rowd.sort(reverse=True)
    for d in rowd[:3]:
        print(json.dumps({"row": d[1], "abs_diff": d[0], "engine": d[2], "oracle": d[3], "x": Xr[:, d[1]].tolist(),
                          "y": float(yr[d[1]]), "f64": float(fx[0, d[1] - t0])}), flush=True)


if __name__ == "__main__":
    main()
