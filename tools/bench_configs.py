"""Throughput of the BASELINE.json configurations other than the headline
(config #2 is bench.py), on one MI355X. One JSON line per measurement.

  #1  README quickstart shape: X 5x100 F32, ops [+,*,/,-]/[cos,exp]: call latency
  #3  NaN-heavy F64: [+,-,*,/,^]/[safe_log,safe_sqrt,cos,exp], X ~ U(-3,3),
      4096 trees x 100k rows: eval_loss, eval_loss_grad and eval_tree_array,
      did_succeed rate
  #5  20 features x 10M rows F32, 16k trees: eval_loss over all rows, over the
      1.25M-row shard one of 8 GPUs holds, and the fused constant gradients
      (eval_loss_grad) over the shard

Usage: python tools/bench_configs.py [--quick]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd")]
import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402


def timed(ctx, fn, reps=3):
    fn()
    ks, ws = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        ws.append(time.perf_counter() - t0)
        del r  # freeing a returned 0.8 GB array (munmap) is the caller's cost, not the call's
        ks.append(ctx.last_kernel_time()[0] * 1e-3)
    return float(np.median(ws)), float(np.median(ks))


def emit(**kw):
    print(json.dumps(kw), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="smaller #5 (for a smoke run)")
    ap.add_argument("--only", default="1,3,5", help="configs to run, e.g. 3")
    args = ap.parse_args()
    only = set(args.only.split(","))
    ctx = srhip.get_context(0)
    rng = np.random.default_rng(0)

    # ---- config #1 -------------------------------------------------------------
    if "1" in only:
        o1 = srhip.Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp"])
        rng = np.random.default_rng(0)
        X1 = rng.standard_normal((5, 100)).astype(np.float32)
        y1 = (2 * np.cos(X1[3]) + X1[0] ** 2 - 2).astype(np.float32)
        t1 = srhip.random_population(20, o1, 5, np.float32, seed=1)
        ds1 = srhip.DeviceDataset(ctx, X1, y1)
        p1 = srhip.Program(ctx, srhip.flatten(t1, o1, np.float32), np.float32)
        w, k = timed(ctx, lambda: p1.eval_loss(ds1, K.LOSS["L2"]), reps=20)
        emit(config="#1 README quickstart shape", what="eval_loss, 20 trees x 100 rows", call_ms=w * 1e3,
             kernel_ms=k * 1e3)

    # ---- config #3 -------------------------------------------------------------
    if "3" in only:
        o3 = srhip.Options(binary_operators=["+", "-", "*", "/", "^"],
                           unary_operators=["safe_log", "safe_sqrt", "cos", "exp"])
        n3 = 100_000
        X3 = rng.uniform(-3, 3, (5, n3))
        y3 = np.cos(X3[3]) * 2 + X3[0] ** 2 - 2
        t3 = srhip.random_population(4096, o3, 5, np.float64, seed=3)
        ds3 = srhip.DeviceDataset(ctx, X3, y3)
        p3 = srhip.Program(ctx, srhip.flatten(t3, o3, np.float64), np.float64)
        _, nodes3, _ = p3.info()
        w, k = timed(ctx, lambda: p3.eval_loss(ds3, K.LOSS["L2"]))
        ok = p3.eval_loss(ds3, K.LOSS["L2"])[2]
        emit(config="#3 NaN-heavy F64", what="eval_loss 4096 trees x 100k rows", dtype="f64",
             node_rows_per_s=nodes3 * n3 / k, call_node_rows_per_s=nodes3 * n3 / w, kernel_ms=k * 1e3,
             did_succeed_rate=float(np.mean(ok)), tree_code_trees=p3.jit_info()["ntrees"],
             ok_sum=int(np.sum(ok)))
        w, k = timed(ctx, lambda: p3.eval_loss_grad(ds3, K.LOSS["L2"]))
        emit(config="#3 NaN-heavy F64", what="eval_loss_grad (dL/dc of every constant) 4096 trees x 100k rows",
             dtype="f64", node_rows_per_s=nodes3 * n3 / k, kernel_ms=k * 1e3, call_ms=w * 1e3,
             grad_tree_code_trees=p3.grad_jit_info()["ntrees"], constants=int(p3.flat.const_off[-1]))
        p3o = srhip.Program(ctx, srhip.flatten(t3[:1024], o3, np.float64), np.float64)
        _, nodes3o, _ = p3o.info()
        w, k = timed(ctx, lambda: p3o.eval_tree_array(ds3))
        emit(config="#3 NaN-heavy F64", what="eval_tree_array 1024 trees x 100k rows (per-row outputs)",
             dtype="f64", node_rows_per_s=nodes3o * n3 / k, kernel_ms=k * 1e3,
             output_GB=1024 * n3 * 8 / 1e9, call_s=w)

    # ---- config #5 -------------------------------------------------------------
    if "5" in only:
        n5 = 1_000_000 if args.quick else 10_000_000
        nt5 = 2048 if args.quick else 16384
        o5 = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
        X5 = rng.standard_normal((20, n5), dtype=np.float32)
        y5 = (2 * np.cos(X5[3]) + X5[0] ** 2 - 2).astype(np.float32)
        t5 = srhip.random_population(nt5, o5, 20, np.float32, seed=5)
        p5 = srhip.Program(ctx, srhip.flatten(t5, o5, np.float32), np.float32)
        _, nodes5, _ = p5.info()
        ds5 = srhip.DeviceDataset(ctx, X5, y5)
        w, k = timed(ctx, lambda: p5.eval_loss(ds5, K.LOSS["L2"]))
        emit(config="#5 20 feat x 10M rows", what=f"eval_loss {nt5} trees x {n5} rows (one GPU, all rows)",
             dtype="f32", node_rows_per_s=nodes5 * n5 / k, kernel_ms=k * 1e3, X_GB=X5.nbytes / 1e9)
        del ds5
        shard = n5 // 8
        ds5s = srhip.DeviceDataset(ctx, X5, y5, row_begin=0, row_end=shard)
        w, k = timed(ctx, lambda: p5.eval_loss(ds5s, K.LOSS["L2"]))
        emit(config="#5 20 feat x 10M rows", what=f"eval_loss {nt5} trees x {shard}-row shard (1 of 8 GPUs)",
             dtype="f32", node_rows_per_s=nodes5 * shard / k, kernel_ms=k * 1e3)
        nconst = int(p5.flat.const_off[-1])
        w, k = timed(ctx, lambda: p5.eval_loss_grad(ds5s, K.LOSS["L2"]), reps=2)
        emit(config="#5 20 feat x 10M rows", what=f"eval_loss_grad (dL/dc of every constant) {nt5} trees x "
             f"{shard}-row shard", dtype="f32", node_rows_per_s=nodes5 * shard / k, kernel_ms=k * 1e3,
             constants=nconst)


if __name__ == "__main__":
    main()
