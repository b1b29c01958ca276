#!/usr/bin/env python3
"""Benchmark: batched eval_loss on the MI355X (BASELINE.json config #2).

One step = one srhip_eval_loss call over the whole batch: 4096 random trees
(maxsize 30, ops + - * / and cos exp) × 1M rows × 5 features, Float32, L2,
with the dataset and the compiled trees already resident in HBM; the step
returns the per-tree loss sums / did_succeed flags in host memory.

Metric: node·row evals/sec = Σ_trees count_nodes × rows ÷ wall time
(nominal count, no credit for early-failed trees).

Multi-GPU (torchrun, one rank per GPU): trees are independent, so each rank
evaluates its own 4096-tree batch (islands/trees sharded over GPUs) against
its own copy of the dataset, with no collective on the data path — weak
scaling. Timing: barrier + sync on both sides of the K timed steps, max over
ranks; value = all ranks' node·rows ÷ that time.

cpu_baseline: the oracle/ CPU restatement of the reference algorithm
(recursive per-node arrays with early exit, fused leaf patterns, separate
loss pass; the turbo=true-like vectorised build) on the host cores, threaded
over trees, on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "symbolicregression.jl_amd"))

# FP32 VALU peak in lane-ops/s: 256 CUs x 4 SIMD-32 x 32 lanes/clk x 2.4 GHz = 78.6e12
# (a wave64 v_fma_f32 issues in 2 cycles on a SIMD-32, MI355X_MICROARCH.md; x2 for
# FMA = the 157.3 TFLOPS spec). SURVEY.md §8d's 39.3e12 assumed SIMD-16; the
# microarchitecture guide's measured figure is used here.
PEAK_VALU_LANE_OPS = 256 * 4 * 32 * 2.4e9
METRIC = "node\u00b7row evals/sec (Float32, 4096 trees\u00d71M rows) at 1/2/4/8 GPUs; % VALU peak"
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--ntrees", type=int, default=4096)
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--nfeat", type=int, default=5)
    ap.add_argument("--maxsize", type=int, default=30)
    ap.add_argument("--dtype", default="f32", choices=["f32", "f64"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU baseline sample time")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: min(os.cpu_count(), 16)")
    ap.add_argument("--no-cpu", action="store_true")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist

        torch.cuda.set_device(local_rank)
        tdist.init_process_group("nccl")
        dist = (torch, tdist)

    import srhip
    from srhip import constants as K

    T = np.float32 if args.dtype == "f32" else np.float64
    options = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(1)
    X = rng.standard_normal((args.nfeat, args.rows)).astype(T)
    y = (T(2) * np.cos(X[3 % args.nfeat]) + X[0] * X[0] - T(2)).astype(T)
    t0 = time.time()
    trees = srhip.random_population(args.ntrees, options, args.nfeat, T, seed=1000 + rank, maxsize=args.maxsize)
    t_gen = time.time() - t0

    ctx = srhip.get_context(local_rank)
    ds = srhip.DeviceDataset(ctx, X, y)
    flat = srhip.flatten(trees, options, dtype=T)
    t0 = time.time()
    prog = srhip.Program(ctx, flat, T)
    t_compile = time.time() - t0
    _, total_nodes, _ = prog.info()
    node_rows = float(total_nodes) * args.rows

    def step():
        return prog.eval_loss(ds, K.LOSS["L2"])

    for _ in range(args.warmup):
        step()

    def barrier():
        ctx.sync()
        if dist:
            torch, tdist = dist
            torch.cuda.synchronize()
            tdist.barrier()

    barrier()
    kernel_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sums, wsum, ok = step()
        kernel_ms.append(ctx.last_kernel_time()[0])
    barrier()
    elapsed = time.perf_counter() - t0

    my_node_rows = node_rows * args.steps
    if dist:
        torch, tdist = dist
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
        nr = torch.tensor([my_node_rows], dtype=torch.float64, device="cuda")
        tdist.all_reduce(nr, op=tdist.ReduceOp.SUM)
        total_node_rows = float(nr.item())
    else:
        total_node_rows = my_node_rows

    value = total_node_rows / elapsed
    ms_per_step = elapsed * 1e3 / args.steps
    k_ms = float(np.mean(kernel_ms))
    kernel_rate = node_rows / (k_ms * 1e-3)  # this rank's kernel-only node·row/s

    if rank != 0:
        if dist:
            dist[1].destroy_process_group()
        return

    # ---- roofline of the dominant kernel (eval_kernel) --------------------------------
    roof = {
        "bound": "valu",
        "achieved": kernel_rate / 1e12,
        "peak": PEAK_VALU_LANE_OPS / 1e12,
        "unit": "T node·row/s vs T FP32 VALU lane-op/s (1 lane-op per node·row)",
        "frac": kernel_rate / PEAK_VALU_LANE_OPS,
        "traffic": None,
        "kernel_ms": k_ms,
    }
    esz = np.dtype(T).itemsize
    alg_bytes = args.rows * (args.nfeat + 1) * esz + prog.ntrees * 17
    roof["hbm_algorithmic_GBs"] = alg_bytes / (k_ms * 1e-3) / 1e9
    prof = ROOT / "profiles" / "current_pmc_summary.json"
    if prof.exists():
        try:
            pm = json.loads(prof.read_text())
            if pm.get("kernel") and pm.get("workload") == "config#2":
                roof["traffic"] = pm.get("hbm_bytes_per_launch")
                roof["valu_busy"] = pm.get("valu_busy")
                roof["pmc_source"] = "profiles/current_pmc_summary.json (rocprofv3 --pmc passes of this bench)"
        except Exception:
            pass

    # ---- CPU baseline (oracle, host cores) ----------------------------------------------
    cpu = None
    if not args.no_cpu:
        sys.path.insert(0, str(ROOT / "oracle"))
        import oracle

        threads = args.cpu_threads or min(os.cpu_count() or 1, 16)
        fl = srhip.flatten(trees, options, dtype=T)

        def run_cpu(nrows, variant="simd"):
            t_ = time.perf_counter()
            oracle.eval_loss_batch(fl, X[:, :nrows], y[:nrows], dtype=T, nthreads=threads, variant=variant)
            return time.perf_counter() - t_, float(fl.nodes.sum()) * nrows

        probe = min(args.rows, 10_000)
        dt, nr = run_cpu(probe)
        nrows = int(min(args.rows, max(probe, probe * args.cpu_seconds / max(dt, 1e-3))))
        dt, nr = run_cpu(nrows)
        cpu = {
            "value": nr / dt,
            "unit": "node·row/s",
            "cores": threads,
            "kind": "port",
            "sample": f"all {len(trees)} trees x first {nrows} rows; oracle simd build (turbo=true analogue), "
                      f"OpenMP over trees; {dt:.1f} s",
        }
        # turbo=false analogue (scalar build), a smaller sample
        ns = max(probe, nrows // 3)
        dts, nrs = run_cpu(ns, "scalar")
        cpu["turbo_false"] = {"value": nrs / dts, "sample": f"first {ns} rows; oracle scalar build; {dts:.1f} s"}

    out = {
        "metric": METRIC if T == np.float32 else "node·row evals/sec (Float64)",
        "value": value,
        "unit": "node·row/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (randn X, y = 2cos(x4) + x1^2 - 2; random trees per gen_random_tree_fixed_size)",
        "config": {
            "workload": f"config#2 batched eval_loss: {args.ntrees} trees (size U{{1..{args.maxsize}}}, "
                        f"+ - * / cos exp) x {args.nfeat} feat x {args.rows} rows, L2",
            "ntrees_per_gpu": args.ntrees,
            "rows": args.rows,
            "nfeat": args.nfeat,
            "total_nodes_per_gpu": int(total_nodes),
            "parallelism": f"trees sharded over {world} GPU(s), no data-path collective",
        },
        "roofline": roof,
        "cpu_baseline": cpu,
        "setup_s": {"tree_gen": round(t_gen, 2), "compile_upload": round(t_compile, 3)},
    }
    print(json.dumps(out))
    if dist:
        dist[1].destroy_process_group()


if __name__ == "__main__":
    main()
