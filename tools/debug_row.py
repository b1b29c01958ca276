#!/usr/bin/env python3
"""Find where tree code goes wrong on one tree (GPU box): bisect the rows of a
disagreeing slice down to single rows, then evaluate every subtree of the
tree on those rows (tree code: loss against y = 0 gives value^2) next to the
oracle.

Usage: python tools/debug_row.py TREE ROW_BEGIN ROW_END
"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd"), str(ROOT / "oracle")]
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402

os.environ.setdefault("SRHIP_JIT", "1")


def subtrees(t):
    out = [t]
    if t.degree >= 1:
        out += subtrees(t.l)
    if t.degree == 2:
        out += subtrees(t.r)
    return out


def main():
    tid, a, b = (int(v) for v in sys.argv[1:4])
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(4096, o, 5, np.float32, seed=0)
    rng = np.random.default_rng(1)
    X = rng.standard_normal((5, 1_000_000)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    ctx = srhip.get_context(0)
    tree = trees[tid]
    prog = srhip.Program(ctx, srhip.flatten([tree] * 600, o, dtype=np.float32), np.float32)
    flat1 = srhip.flatten([tree], o, dtype=np.float32)

    def bad(lo, hi):
        ds = srhip.DeviceDataset(ctx, X, y, row_begin=lo, row_end=hi)
        s, w, ok = prog.eval_loss(ds, K.LOSS["L2"])
        _, l, okr = oracle.eval_loss_batch(flat1, X[:, lo:hi], y[lo:hi], dtype=np.float32)
        ref = float(l[0]) * (hi - lo)
        return bool(ok[0]) != bool(okr[0]) or (okr[0] and not abs(float(s[0]) - ref) <= 1e-5 * abs(ref) + 1e-30)

    rows = []
    stack = [(a, b)]
    while stack and len(rows) < 4:
        lo, hi = stack.pop()
        if not bad(lo, hi):
            continue
        if hi - lo == 1:
            rows.append(lo)
            continue
        m = (lo + hi) // 2
        stack += [(m, hi), (lo, m)]
    print(f"tree {tid}: {srhip.string_tree(tree, o)}\nrows where tree code disagrees: {rows}", flush=True)
    subs = subtrees(tree)
    sflat = srhip.flatten(subs * (600 // len(subs) + 1), o, dtype=np.float32)
    sprog = srhip.Program(ctx, sflat, np.float32)
    for r in rows:
        zero = np.zeros(1, np.float32)
        ds = srhip.DeviceDataset(ctx, X[:, r:r + 1].copy(), zero)
        s, w, ok = sprog.eval_loss(ds, K.LOSS["L2"])
        vals, okv = oracle.eval_trees(srhip.flatten(subs, o, dtype=np.float32), X[:, r:r + 1], dtype=np.float32)
        print(f"row {r}: x = {X[:, r].tolist()}")
        for k, st in enumerate(subs):
            got = np.sqrt(s[k]) if ok[k] else np.nan
            ref = abs(float(vals[k][0])) if okv[k] else np.nan
            flag = "" if (np.isnan(got) and np.isnan(ref)) or abs(got - ref) <= 1e-5 * abs(ref) + 1e-30 else "   <-- differs"
            print(f"   |{srhip.string_tree(st, o)[:90]}| = {got:.9g} (oracle {ref:.9g}, ok {bool(ok[k])}/{bool(okv[k])}){flag}")


if __name__ == "__main__":
    main()
