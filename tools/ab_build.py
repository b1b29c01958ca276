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

--grad: config #5's gradient workload instead (tools/prof_grad.py: 16384
trees of 20 features over the 1.25M-row shard, eval_loss_grad), checking
did_succeed, losses and ∂L/∂c equal to the first variant's bit for bit.

Usage: python tools/ab_build.py [--grad] [--ntrees 4096] [--steps 30] 'SRHIP_JIT_GCOLS=0' 'SRHIP_JIT_GCOLS=32' ...
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
    ap.add_argument("--grad", action="store_true")
    ap.add_argument("variants", nargs="+")
    args = ap.parse_args()
    import numpy as np

    import srhip
    from srhip import constants as K

    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    if args.grad:
        rng = np.random.default_rng(5)
        X = rng.standard_normal((20, 1_250_000), dtype=np.float32)
        y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
        trees = srhip.random_population(16384, o, 20, np.float32, seed=5)[: args.ntrees]
    else:
        rng = np.random.default_rng(1)
        X = rng.standard_normal((5, args.rows)).astype(np.float32)
        y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
        trees = srhip.random_population(4096, o, 5, np.float32, seed=1000)[: args.ntrees]
    ctx = srhip.get_context(0)
    ds = srhip.DeviceDataset(ctx, X, y)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    progs = []
    for v in args.variants:
        env = dict(kv.split("=", 1) for kv in v.replace(",", " ").split())  # "A=1,B=0": two knobs
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            progs.append(srhip.Program(ctx, flat, np.float32))
            if args.grad:  # the gradient tree code is built at the first gradient call
                progs[-1].eval_loss_grad(ds, K.LOSS["L2"])
        finally:
            for k, x in old.items():
                if x is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = x
    call = (lambda p: p.eval_loss_grad(ds, K.LOSS["L2"])) if args.grad else (lambda p: p.eval_loss(ds, 0))
    res = [tuple(np.array(x, copy=True) if hasattr(x, "shape") else x for x in call(p)) for p in progs]
    for p in progs:  # warm-up
        for _ in range(3):
            call(p)
    times = [[] for _ in progs]
    for _ in range(args.steps):
        for k, p in enumerate(progs):
            call(p)
            times[k].append(ctx.last_kernel_time()[0])
    if args.grad:
        s0, g0, _, k0 = res[0]
        for v, (s, g, _, k), t, p in zip(args.variants, res, times, progs):
            okc = np.repeat(k & k0, np.diff(p.flat.const_off))
            print(json.dumps({"variant": v, "median_ms": float(np.median(t)), "min_ms": float(np.min(t)),
                              "did_succeed_equal": bool(np.array_equal(k, k0)),
                              "loss_equal": bool(np.array_equal(s[k & k0], s0[k & k0])),
                              "grad_equal": bool(np.array_equal(g[okc], g0[okc], equal_nan=True)),
                              # a variant that evaluates a derivative differently (SRHIP_GJIT_SINCOS):
                              # constants off the first variant's by > 1e-4 relative, and the largest
                              "grad_rel_gt_1e-4": int(np.sum(~(np.abs(g[okc] - g0[okc]) <= 1e-4 * np.abs(g0[okc])))),
                              "grad_max_rel": float(np.nanmax(np.abs(g[okc] - g0[okc]) / np.maximum(np.abs(g0[okc]), 1e-30))),
                              "grad_jit": p.grad_jit_info(),
                              "ntrees": len(trees)}))
            sys.stdout.flush()
        return
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
