#!/usr/bin/env python3
"""Trees of tests/test_gpu_parity.py::test_random_trees_f32_losses (1000
trees, seed 7, 20000 rows) whose loss lies outside 4x the oracle's
perturbation spread: their expression and the loss under each tree-code
variant (GPU box). Usage: python tools/debug_outliers.py"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import numpy as np  # noqa: E402

VARIANTS = ["", "SRHIP_JIT_FAST=0", "SRHIP_JIT_MANUAL=0", "SRHIP_JIT_MANUAL_OFF=exp", "SRHIP_JIT_MANUAL_OFF=trig",
            "SRHIP_JIT_MANUAL_OFF=div", "SRHIP_JIT=0"]


def setup():
    import srhip

    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(1000, o, 5, np.float32, seed=7)
    X = np.random.default_rng(1).standard_normal((5, 20000)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    return srhip, o, trees, X, y


def child():
    srhip, o, trees, X, y = setup()
    ds = srhip.Dataset(X, y)
    losses, ok = srhip.eval_loss_batch_ok(trees, ds, o)
    print(json.dumps(dict(l=[float(v) for v in losses], ok=[int(v) for v in ok])))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        return child()
    import oracle
    from numerics import loss_spread

    srhip, o, trees, X, y = setup()
    _, ref, rok = oracle.eval_loss_batch(srhip.flatten(trees, o, dtype=np.float32), X, y, dtype=np.float32)
    res = {}
    for v in VARIANTS:
        env = dict(os.environ)
        for kv in v.split():
            k, val = kv.split("=")
            env[k] = val
        r = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True, timeout=300)
        res[v] = json.loads(r.stdout.strip().splitlines()[-1])
    d = res[""]
    l = np.array(d["l"])
    m = np.array(d["ok"], bool) & rok & np.isfinite(ref)
    rel = np.abs(l - ref) / np.abs(ref)
    cand = np.flatnonzero(m & ~(rel <= 1e-5))
    sp = loss_spread([trees[i] for i in cand], o, X, y, None, np.float32) / X.shape[1]
    for i, s in zip(cand, sp):
        e = abs(l[i] - ref[i]) / max(s, 1e-300)
        if e <= 4:
            continue
        print(f"tree {i}: err/spread {e:.1f}, oracle {ref[i]:.7g}: {srhip.string_tree(trees[i], o)}")
        for v in VARIANTS:
            print(f"   [{v or 'default'}] {res[v]['l'][i]:.7g} ok={res[v]['ok'][i]}")


if __name__ == "__main__":
    main()
