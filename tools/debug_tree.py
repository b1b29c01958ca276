#!/usr/bin/env python3
"""Debug one config #2 tree on the GPU box: its tree-code loss over row
slices under several knob settings against the oracle, and the oracle's
per-row values on the slices where they disagree.

Usage: python tools/debug_tree.py TREE [TREE ...]   (ids in config #2's batch, seed 0)
"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd"), str(ROOT / "oracle")]
import numpy as np  # noqa: E402

VARIANTS = ["", "SRHIP_JIT_DERIVE=0", "SRHIP_JIT_FAST=0", "SRHIP_JIT_MANUAL=0", "SRHIP_JIT=0"]
SLICES = 200


def child(tid):
    import srhip
    from srhip import constants as K

    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(4096, o, 5, np.float32, seed=0)
    rng = np.random.default_rng(1)
    X = rng.standard_normal((5, 1_000_000)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    # the tree among 600 others of the batch (tree code needs >= 512 trees unless SRHIP_JIT=1)
    batch = [trees[tid]] + trees[:599]
    ctx = srhip.get_context(0)
    prog = srhip.Program(ctx, srhip.flatten(batch, o, dtype=np.float32), np.float32)
    n = X.shape[1]
    out = []
    for k in range(SLICES):
        a, b = k * n // SLICES, (k + 1) * n // SLICES
        ds = srhip.DeviceDataset(ctx, X, y, row_begin=a, row_end=b)
        s, w, ok = prog.eval_loss(ds, K.LOSS["L2"])
        out.append([float(s[0]), int(ok[0])])
        del ds
    print(json.dumps(dict(slices=out, info=prog.jit_info())))


def main():
    if sys.argv[1] == "--child":
        return child(int(sys.argv[2]))
    import oracle
    import srhip

    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(4096, o, 5, np.float32, seed=0)
    rng = np.random.default_rng(1)
    X = rng.standard_normal((5, 1_000_000)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    n = X.shape[1]
    for tid in [int(v) for v in sys.argv[1:]]:
        print(f"== tree {tid}: {srhip.string_tree(trees[tid], o)}", flush=True)
        flat = srhip.flatten([trees[tid]], o, dtype=np.float32)
        ref = []
        for k in range(SLICES):
            a, b = k * n // SLICES, (k + 1) * n // SLICES
            _, l, okr = oracle.eval_loss_batch(flat, X[:, a:b], y[a:b], dtype=np.float32)
            ref.append((float(l[0]) * (b - a), bool(okr[0])))
        for var in VARIANTS:
            env = dict(os.environ)
            for kv in var.split():
                kk, vv = kv.split("=")
                env[kk] = vv
            r = subprocess.run([sys.executable, __file__, "--child", str(tid)], env=env, capture_output=True,
                               text=True, timeout=300)
            if r.returncode:
                print(f"  [{var}] FAILED {r.stderr[-1500:]}")
                continue
            d = json.loads(r.stdout.strip().splitlines()[-1])
            bad = []
            for k, ((s, ok), (rl, rok)) in enumerate(zip(d["slices"], ref)):
                if bool(ok) != rok or (rok and not (abs(s - rl) <= 1e-5 * abs(rl))):
                    bad.append((k, s, ok, rl, rok))
            print(f"  [{var or 'default'}] {len(bad)} slices differ; {bad[:4]}", flush=True)
            if bad and var == "":
                k = bad[0][0]
                a, b = k * n // SLICES, (k + 1) * n // SLICES
                v, okv = oracle.eval_trees(flat, X[:, a:b], dtype=np.float32)
                r_ = (v[0].astype(np.float64) - y[a:b])
                i = np.argsort(-np.abs(r_))[:5]
                print(f"    oracle largest residuals in slice {k}: rows {a + i} r={r_[i]} X={X[:, a + i].T.tolist()}")


if __name__ == "__main__":
    main()
