#!/usr/bin/env python3
"""Interleaved A/B of BUILD-time knobs of the loss tree code (GPU box).

Every variant's program is built in this one process with its environment
set (knobs the tree compiler reads per build: SRHIP_JIT_GCOLS,
SRHIP_JIT_GPREFETCH, ...), then the variants' eval_loss calls alternate
A B C A B C ... so that clock drift hits all of them alike. Prints, per
variant, the median kernel time of the call (HIP events of the context:
every launch of the call, the derive passes included) and checks that every
variant gives the first one's did_succeed exactly and its losses within
1e-5 (shared columns change FAST values into PRECISE ones).

Usage: python tools/ab_build.py [--ntrees 4096] [--steps 30] 'SRHIP_JIT_GCOLS=0' 'SRHIP_JIT_GCOLS=32' ...
"""
import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "symbolicregression.jl_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ntrees", type=int, default=4096)
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("variants", nargs="+")
    args = ap.parse_args()
    import numpy as np

    import srhip

    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(1)
    X = rng.standard_normal((5, args.rows)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    trees = srhip.random_population(4096, o, 5, np.float32, seed=1000)[: args.ntrees]
    ctx = srhip.get_context(0)
    ds = srhip.DeviceDataset(ctx, X, y)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    progs = []
    for v in args.variants:
        env = dict(kv.split("=", 1) for kv in v.split())
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            progs.append(srhip.Program(ctx, flat, np.float32))
        finally:
            for k, x in old.items():
                if x is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = x
    res = [p.eval_loss(ds, 0) for p in progs]
    for p in progs:  # warm-up
        for _ in range(3):
            p.eval_loss(ds, 0)
    times = [[] for _ in progs]
    for _ in range(args.steps):
        for k, p in enumerate(progs):
            p.eval_loss(ds, 0)
            times[k].append(ctx.last_kernel_time()[0])
    s0, w0, k0 = res[0]
    for v, (s, w, k), t in zip(args.variants, res, times):
        same_ok = bool(np.array_equal(k, k0))
        m = k & k0
        rel = float(np.max(np.abs(s[m] - s0[m]) / np.maximum(np.abs(s0[m]), 1e-30))) if m.any() else 0.0
        print(json.dumps({"variant": v, "median_ms": float(np.median(t)), "min_ms": float(np.min(t)),
                          "did_succeed_equal": same_ok, "max_rel_loss_diff": rel, "ntrees": args.ntrees}))
        sys.stdout.flush()


if __name__ == "__main__":
    main()
