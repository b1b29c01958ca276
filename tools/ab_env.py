#!/usr/bin/env python3
"""A/B of environment knobs on the loss tree code (experiments, GPU box).

Each variant runs in its own process (the knobs are read once per process):
config #2's batch (or a shard of it) x 1M rows, 5 warm-up calls, then K timed
calls; prints the mean kernel time (HIP events of the context) and the
per-call wall time, and checks that every variant returns the same losses
and did_succeed as the first one (bit for bit).

Usage: python tools/ab_env.py [--ntrees 4096,512] [--rows 30000,125000] [--rounds 2] [--steps 20] 'A=1 B=2' 'A=0' ...
(AB_CFG=5: config #5's 1.25M-row shard with 20 features, the first NTREES of its 16384 trees)
"""
import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def child(ntrees, steps, rows=1_000_000):
    sys.path.insert(0, str(ROOT / "symbolicregression.jl_amd"))
    import numpy as np

    import srhip
    from srhip import constants as K

    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    if os.environ.get("AB_CFG") == "5":  # config #5's shard: 20 features x 1.25M rows, 16384 trees
        rng = np.random.default_rng(5)
        X = rng.standard_normal((20, 1_250_000), dtype=np.float32)
        y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
        trees = srhip.random_population(16384, o, 20, np.float32, seed=5)[: ntrees]
    else:
        rng = np.random.default_rng(1)
        X = rng.standard_normal((5, 1_000_000)).astype(np.float32)
        y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
        trees = srhip.random_population(4096, o, 5, np.float32, seed=1000)
        trees = trees[::4096 // ntrees]
        X, y = np.ascontiguousarray(X[:, :rows]), np.ascontiguousarray(y[:rows])
    ctx = srhip.get_context(0)
    ds = srhip.DeviceDataset(ctx, X, y)
    prog = srhip.Program(ctx, srhip.flatten(trees, o, dtype=np.float32), np.float32)
    for _ in range(5):
        prog.eval_loss(ds, K.LOSS["L2"])
    ks = []
    t0 = time.perf_counter()
    for _ in range(steps):
        s, w, ok = prog.eval_loss(ds, K.LOSS["L2"])
        ks.append(ctx.last_kernel_time()[0])
    redone = ctx.last_jit_events()[1]
    wall = (time.perf_counter() - t0) / steps * 1e3
    print(json.dumps(dict(kernel_ms=float(np.mean(ks)), wall_ms=wall, redone=int(redone), sums=[float(v) for v in s],
                          ok=[int(v) for v in ok], info=prog.jit_info())))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ntrees", default="4096")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rows", default="1000000", help="config #2 only: the first ROWS rows (comma list)")
    ap.add_argument("--rounds", type=int, default=1, help="interleaved repeats of every variant")
    ap.add_argument("--child", type=int, default=0)
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    if a.child:
        return child(a.child, a.steps, int(a.rows))
    for nt, rows, rnd in [(int(n), int(r), k) for n in a.ntrees.split(",") for r in a.rows.split(",")
                          for k in range(a.rounds)]:
        ref = None
        for var in a.variants or [""]:
            env = dict(os.environ)
            for kv in var.split():
                k, v = kv.split("=", 1)
                env[k] = v
            r = subprocess.run([sys.executable, __file__, "--child", str(nt), "--steps", str(a.steps),
                                "--rows", str(rows)], env=env,
                               capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(f"{nt:5d} trees [{var}] FAILED rc={r.returncode}\n{r.stderr[-2000:]}", flush=True)
                return 1
            d = json.loads(r.stdout.strip().splitlines()[-1])
            same = ""
            if ref is None:
                ref = d
            else:
                import numpy as np
                s0, s1 = np.array(ref["sums"]), np.array(d["sums"])
                okeq = ref["ok"] == d["ok"]
                m = np.array(ref["ok"], bool)
                bit = np.array_equal(s0[m], s1[m])
                rel = float(np.nanmax(np.abs(s1[m] - s0[m]) / np.maximum(np.abs(s0[m]), 1e-300))) if m.any() else 0.0
                same = f" ok_equal={okeq} bit_equal={bit} max_rel={rel:.2e}"
            print(f"{nt:5d} trees x {rows} rows (round {rnd}) [{var or 'default'}] kernel {d['kernel_ms']:.3f} ms, call {d['wall_ms']:.3f} ms, "
                  f"tiles redone {d['redone']}"
                  f"{same}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
