#!/usr/bin/env python3
"""Config #3's per-row output call (eval_tree_array, 1024 Float64 trees x 100k
rows, 0.82 GB to a fresh host array) under host-copy thread counts
(SRHIP_COPY_THREADS), each in its own process: median call time of 5.
Usage: python tools/out_copy.py 8 16 32"""
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def child():
    sys.path.insert(0, str(ROOT / "symbolicregression.jl_amd"))
    import numpy as np

    import srhip

    o3 = srhip.Options(binary_operators=["+", "-", "*", "/", "^"], unary_operators=["safe_log", "safe_sqrt", "cos", "exp"])
    rng = np.random.default_rng(0)
    X3 = rng.uniform(-3, 3, (5, 100_000))
    y3 = np.cos(X3[3]) * 2 + X3[0] ** 2 - 2
    t3 = srhip.random_population(4096, o3, 5, np.float64, seed=3)[:1024]
    ctx = srhip.get_context(0)
    ds = srhip.DeviceDataset(ctx, X3, y3)
    if os.environ.get("AFTER_LOSS"):  # as tools/bench_configs.py: the 4096-tree eval_loss first
        from srhip import constants as K
        t4 = srhip.random_population(4096, o3, 5, np.float64, seed=3)
        p4 = srhip.Program(ctx, srhip.flatten(t4, o3, np.float64), np.float64)
        for _ in range(4):
            p4.eval_loss(ds, K.LOSS["L2"])
    p = srhip.Program(ctx, srhip.flatten(t3, o3, np.float64), np.float64)
    p.eval_tree_array(ds)
    ws = []
    for _ in range(5):
        t0 = time.perf_counter()
        v, ok = p.eval_tree_array(ds)[:2]
        ws.append(time.perf_counter() - t0)
        del v
    print(json.dumps(dict(call_ms=float(np.median(ws)) * 1e3, calls_ms=[round(w * 1e3, 1) for w in ws],
                          kernel_ms=ctx.last_kernel_time()[0])))


if __name__ == "__main__":
    if sys.argv[1:] == ["--child"]:
        child()
    else:
        for n in sys.argv[1:] or ["16"]:
            env = dict(os.environ, SRHIP_COPY_THREADS=n.split(":")[0])
            if n.endswith(":after"):
                env["AFTER_LOSS"] = "1"
            r = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True, timeout=300)
            print(f"SRHIP_COPY_THREADS={n}: {r.stdout.strip() or r.stderr[-800:]}", flush=True)
