#!/usr/bin/env python3
"""Benchmark: batched eval_loss on the MI355X (BASELINE.json config #2).

One step = one srhip_eval_loss call over the whole batch: 4096 random trees
(maxsize 30, ops + - * / and cos exp) × 1M rows × 5 features, Float32, L2,
with the dataset and the compiled trees already resident in HBM; the step
returns the per-tree loss sums / did_succeed flags in host memory. Large
Float32 batches run as tree code (csrc/jit.cpp): the program's creation
compiles every tree to machine code (reported under setup_s / tree_code).

Metric: node·row evals/sec = Σ_trees count_nodes × rows ÷ wall time
(nominal count, no credit for early-failed trees).

Multi-GPU (torchrun, one rank per GPU), strong scaling of the one batch:
  --shard rows (default) the 1M rows split over the N ranks, every rank
      evaluates all trees on its shard and the per-tree [Σw·ℓ, failed]
      partials + Σw are all-reduced on the device (RCCL, 64 KiB) each step;
  --shard trees  each rank evaluates its share of the 4096 trees against its
      own copy of the dataset, no collective on the data path; the share is
      cost-balanced (srhip.distributed.shard_trees_balanced: LPT on the
      estimated VALU cost; --partition strided: every N-th tree), plus a
      weak-scaling figure (4096 trees on every rank) as `weak`.
Rows by default since round 6: the whole batch's constant-free subtrees
shared by many trees are evaluated once per row (jit.h Columns), and a row
shard keeps every tree, so the sharing, while a 512-tree shard shares little
and derives its own columns over all 1M rows. Measured on one GPU at the
N = 8 sizes (profiles/r06_shard_probe.json): slowest row shard 0.52 ms
before its all-reduce, slowest balanced tree shard 0.65 ms, strided 0.63,
against 2.74 ms for the whole batch (projected 5.3x / 4.2x / 4.4x).
Timing: barrier + sync on both sides of the K timed steps, max over ranks;
value = the 4096 trees' node·rows ÷ that time.

cpu_baseline: the oracle/ CPU restatement of the reference algorithm
(recursive per-node arrays with early exit, fused leaf patterns, separate
loss pass) on the host cores this job may use, threaded over trees, both the
turbo=true-like vectorised build and the turbo=false-like scalar build on
the same bounded row sample of the same workload.
"""
from __future__ import annotations

import argparse
import hashlib
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
# SRHIP_BENCH_SHARED_GPU=1: every rank on GPU 0 over gloo (rehearsing the N > 1
# code paths on a one-GPU box; the numbers are not a measurement)
SHARED_GPU = os.environ.get("SRHIP_BENCH_SHARED_GPU") == "1"


def available_cpus() -> int:
    """CPUs this job may use: the cgroup CPU quota if one is set, else the
    affinity mask (a shared GPU box shows the whole machine in os.cpu_count())."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return max(n, 1)


def cpu_note() -> str:
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return f"affinity {aff}, os.cpu_count() {os.cpu_count()}, cgroup-limited {available_cpus()}"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--ntrees", type=int, default=4096)
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--nfeat", type=int, default=5)
    ap.add_argument("--maxsize", type=int, default=30)
    ap.add_argument("--dtype", default="f32", choices=["f32", "f64"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU baseline sample time")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every CPU this job may use")
    ap.add_argument("--partition", default="balanced", choices=["balanced", "strided"],
                    help="--shard trees: cost-balanced (LPT) or every N-th tree")
    ap.add_argument("--shard", default="rows", choices=["trees", "rows"],
                    help="N > 1: trees split over the ranks (no collective) or rows split over the ranks "
                         "(every rank all trees, partials all-reduced on the device per step)")
    ap.add_argument("--no-weak", action="store_true", help="skip the secondary weak-scaling measurement")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-row-shard", action="store_true",
                    help="skip the config #5 row-shard leg (rows over the GPUs, device-side all-reduce)")
    ap.add_argument("--rs-rows", type=int, default=10_000_000)
    ap.add_argument("--rs-trees", type=int, default=16384)
    ap.add_argument("--rs-nfeat", type=int, default=20)
    ap.add_argument("--rs-steps", type=int, default=5)
    ap.add_argument("--stub", action="store_true",
                    help="launcher test only (tests/test_bench_launcher.py): gloo, no GPU, no evaluation")
    return ap.parse_args()


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(nproc: int) -> int:
    """`python bench.py --gpus N` without a launcher around it: start N ranks
    through torch.distributed.run (one process per GPU, RCCL) and pass their
    output through. This parent never touches the GPU (no HIP call before the
    children start); rank 0 prints the JSON line."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(Path(__file__).resolve())] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}")
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist

        if args.stub:
            tdist.init_process_group("gloo")
        elif SHARED_GPU:
            # rehearsal of the N > 1 paths on a one-GPU box (tools/gpu_run.sh n2):
            # every rank on GPU 0, gloo, host-side reductions; not a measurement
            torch.cuda.set_device(0)
            tdist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local_rank)
            tdist.init_process_group("nccl")
        dist = (torch, tdist)
    if args.stub:
        return stub_main(args, world, rank, dist)

    import srhip
    from srhip import constants as K
    from srhip.distributed import DeviceRowShard, shard_range, shard_trees, shard_trees_balanced

    T = np.float32 if args.dtype == "f32" else np.float64
    options = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(1)
    X = rng.standard_normal((args.nfeat, args.rows)).astype(T)
    y = (T(2) * np.cos(X[3 % args.nfeat]) + X[0] * X[0] - T(2)).astype(T)
    t0 = time.time()
    # the same batch on every rank; rank r evaluates its share of the trees (strong scaling)
    all_trees = srhip.random_population(args.ntrees, options, args.nfeat, T, seed=1000, maxsize=args.maxsize)
    rows_mode = world > 1 and args.shard == "rows"
    if rows_mode:  # every tree on rows [rb, re)
        trees = all_trees
        rb, re = shard_range(args.rows, rank, world)
        X, y = np.ascontiguousarray(X[:, rb:re]), np.ascontiguousarray(y[rb:re])
    else:
        part = (shard_trees_balanced(all_trees, options, rank, world) if args.partition == "balanced"
                else shard_trees(len(all_trees), rank, world))
        trees = [all_trees[i] for i in part]
    t_gen = time.time() - t0

    ctx = srhip.get_context(0 if SHARED_GPU else local_rank)
    ds = srhip.DeviceDataset(ctx, X, y)
    flat = srhip.flatten(trees, options, dtype=T)
    t0 = time.time()
    prog = srhip.Program(ctx, flat, T)
    t_compile = time.time() - t0
    _, total_nodes, _ = prog.info()
    node_rows = float(total_nodes) * X.shape[1]
    rshard = DeviceRowShard(prog, ds, options.elementwise_loss) if rows_mode else None

    def barrier():
        ctx.sync()
        if dist:
            torch, tdist = dist
            torch.cuda.synchronize()
            tdist.barrier()

    step_ms = []  # per-step wall time of the headline loop (each call returns synchronised)

    def timed(p, steps, warmup, record=None):
        # one step: the loss of every tree on this rank's rows (rows mode: + the
        # all-reduce of the per-tree partials over the ranks)
        step = rshard.step if (rshard is not None and p is prog) else (lambda: p.eval_loss(ds, K.LOSS["L2"]))
        for _ in range(warmup):
            step()
        barrier()
        kms = []
        t_ = time.perf_counter()
        t_prev = t_
        for _ in range(steps):
            step()
            kms.append(ctx.last_kernel_time()[0])
            if record is not None:
                t_now = time.perf_counter()
                record.append((t_now - t_prev) * 1e3)
                t_prev = t_now
        barrier()
        return time.perf_counter() - t_, kms

    dev = "cpu" if SHARED_GPU else "cuda"

    def reduce_max_sum(elapsed_, node_rows_):
        if not dist:
            return elapsed_, node_rows_
        torch, tdist = dist
        t = torch.tensor([elapsed_], dtype=torch.float64, device=dev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        nr = torch.tensor([node_rows_], dtype=torch.float64, device=dev)
        tdist.all_reduce(nr, op=tdist.ReduceOp.SUM)
        return float(t.item()), float(nr.item())

    elapsed, kernel_ms = timed(prog, args.steps, args.warmup, step_ms)
    elapsed, total_node_rows = reduce_max_sum(elapsed, node_rows * args.steps)
    tree_code = prog.jit_info()

    # secondary: weak scaling (the whole batch on every rank)
    weak = None
    if world > 1 and not args.no_weak and not rows_mode:
        wprog = srhip.Program(ctx, srhip.flatten(all_trees, options, dtype=T), T)
        _, wnodes, _ = wprog.info()
        w_el, _ = timed(wprog, max(args.steps // 2, 3), 1)
        w_el, w_nr = reduce_max_sum(w_el, float(wnodes) * args.rows * max(args.steps // 2, 3))
        weak = {"value": w_nr / w_el, "unit": "node·row/s", "ntrees_per_gpu": len(all_trees),
                "ms_per_step": w_el * 1e3 / max(args.steps // 2, 3)}
        del wprog

    row_shard = None if args.no_row_shard else row_shard_leg(args, world, rank, ctx, dist, barrier)

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
    alg_bytes = X.shape[1] * (args.nfeat + 1) * esz + prog.ntrees * 17
    roof["hbm_algorithmic_GBs"] = alg_bytes / (k_ms * 1e-3) / 1e9
    # counter fields from the rocprofv3 --pmc passes of this bench command
    # (tools/gpu_run.sh profile → profiles/current_pmc_summary.json), attached
    # only when that summary measured the kernel this run launched, from the
    # same libsrhip.so (kernel symbol + sha256 of the library)
    ran = ctx.last_kernel_name()
    lib_sha = hashlib.sha256(srhip._lib.LIB_PATH.read_bytes()).hexdigest()
    roof["kernel"] = ran
    prof = ROOT / "profiles" / "current_pmc_summary.json"
    if prof.exists():
        try:
            pm = json.loads(prof.read_text())
            same = pm.get("kernel") == ran and pm.get("lib_sha256") == lib_sha and pm.get("workload") == "config#2"
            if same and args.rows == 1_000_000 and args.ntrees == 4096 and world == 1:
                roof["traffic"] = pm.get("hbm_bytes_per_launch")
                roof["valu_busy"] = pm.get("valu_busy")
                roof["pmc_source"] = "profiles/current_pmc_summary.json (rocprofv3 --pmc passes of this bench)"
            else:
                roof["pmc_source"] = (f"none: profiles/current_pmc_summary.json measured {pm.get('kernel')} "
                                      f"from lib {str(pm.get('lib_sha256'))[:12]}, this run {ran} from {lib_sha[:12]}")
        except Exception:
            pass

    # ---- CPU baseline (oracle, host cores) ----------------------------------------------
    cpu = None
    if not args.no_cpu and world == 1:  # rank 0 at N = 1 only
        sys.path.insert(0, str(ROOT / "oracle"))
        import oracle

        threads = args.cpu_threads or available_cpus()
        fl = srhip.flatten(trees, options, dtype=T)

        def run_cpu(nrows, variant="simd", reps=1):
            t_ = time.perf_counter()
            for _ in range(reps):
                oracle.eval_loss_batch(fl, X[:, :nrows], y[:nrows], dtype=T, nthreads=threads, variant=variant)
            return time.perf_counter() - t_, float(fl.nodes.sum()) * nrows * reps

        probe = min(args.rows, 10_000)
        dt, nr = run_cpu(probe)
        nrows = int(min(args.rows, max(probe, probe * args.cpu_seconds / max(dt, 1e-3))))
        # the whole workload in less than the target time: repeated, so the
        # sample is about --cpu-seconds of CPU work
        reps = max(1, int(round(args.cpu_seconds / max(dt * nrows / probe, 1e-3)))) if nrows == args.rows else 1
        dt, nr = run_cpu(nrows, reps=reps)
        cpu = {
            "value": nr / dt,
            "unit": "node·row/s",
            "cores": threads,
            "kind": "port",
            "sample": f"all {len(trees)} trees x first {nrows} rows" + (f", {reps} passes" if reps > 1 else "") +
                      "; oracle simd build (turbo=true analogue), "
                      f"OpenMP over trees on {threads} threads (the CPUs this job may use: {cpu_note()}); "
                      f"{dt:.1f} s",
        }
        # turbo=false analogue (scalar build) on the same rows
        dts, nrs = run_cpu(nrows, "scalar", reps=reps)
        cpu["turbo_false"] = {"value": nrs / dts, "sample": f"same {nrows} rows x {reps}; oracle scalar build; {dts:.1f} s"}

    out = {
        "metric": METRIC if T == np.float32 else "node·row evals/sec (Float64)",
        "value": value,
        "unit": "node·row/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (randn X, y = 2cos(x4) + x1^2 - 2; random trees per gen_random_tree_fixed_size)",
        "config": {
            "workload": f"config#2 batched eval_loss: {args.ntrees} trees (size U{{1..{args.maxsize}}}, "
                        f"+ - * / cos exp) x {args.nfeat} feat x {args.rows} rows, L2",
            "ntrees": args.ntrees,
            "ntrees_per_gpu": len(trees),
            "rows": args.rows,
            "nfeat": args.nfeat,
            "total_nodes_per_gpu": int(total_nodes),
            "parallelism": (f"the {args.rows} rows sharded over {world} GPU(s) (strong scaling): every tree on "
                            "each shard, [Σw·ℓ, failed] per tree + Σw all-reduced on the device (RCCL) each step"
                            if rows_mode else
                            f"the {args.ntrees} trees sharded over {world} GPU(s) ({args.partition}, strong "
                            "scaling), no data-path collective"),
        },
        "weak": weak,
        "row_shard": row_shard,
        "tree_code": tree_code,
        "roofline": roof,
        "cpu_baseline": cpu,
        "setup_s": {"tree_gen": round(t_gen, 2), "compile_upload": round(t_compile, 3)},
        "steps_detail": step_stats(step_ms, kernel_ms),
    }
    print(json.dumps(out))
    if dist:
        dist[1].destroy_process_group()


def step_stats(wall_ms, kern_ms):
    """Rank 0's per-step wall time (host clock between the returns of
    consecutive synchronous calls) and kernel time (HIP events on the
    context's stream): min / median / max and the first three steps, so a
    single stall and a uniform per-call cost can be told apart."""
    def s(v):
        a = np.asarray(v, dtype=np.float64)
        if a.size == 0:
            return None
        return {"min": round(float(a.min()), 4), "median": round(float(np.median(a)), 4),
                "max": round(float(a.max()), 4), "first3": [round(float(x), 4) for x in a[:3]]}
    gap = [w - k for w, k in zip(wall_ms, kern_ms)]
    return {"wall_ms": s(wall_ms), "kernel_ms": s(kern_ms), "non_kernel_ms": s(gap)}


def row_shard_leg(args, world, rank, ctx, dist, barrier):
    """Config #5: 16384 trees x 20 features x 10M rows, the
    rows split over the N ranks (contiguous shards, shard_range), every rank
    evaluating every tree on its shard; per step: srhip_eval_loss_packed into
    a device buffer, then one all_reduce(SUM) of [Σw·ℓ, failed] per tree + Σw
    over RCCL (srhip.distributed.DeviceRowShard). The dataset is generated in
    fixed blocks of rows (seeded per block), so every N sees the same 10M
    rows. Reports the step time (max over ranks), the evaluation and the
    all-reduce time separately, and node·row/s of the whole job."""
    import srhip
    from srhip import constants as K
    from srhip.distributed import DeviceRowShard, shard_range

    n, F = args.rs_rows, args.rs_nfeat
    rb, re = shard_range(n, rank, world)
    blk = max(1, n // 8)
    Xs = np.empty((F, re - rb), dtype=np.float32)
    for b in range(rb // blk, (re - 1) // blk + 1):
        b0, b1 = b * blk, min(n, (b + 1) * blk)
        lo, hi = max(b0, rb), min(b1, re)
        if lo >= hi:
            continue
        Xb = np.random.default_rng(900 + b).standard_normal((F, b1 - b0), dtype=np.float32)
        Xs[:, lo - rb:hi - rb] = Xb[:, lo - b0:hi - b0]
    ys = (np.float32(2) * np.cos(Xs[3 % F]) + Xs[0] * Xs[0] - np.float32(2)).astype(np.float32)
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(args.rs_trees, o, F, np.float32, seed=52)
    ds = srhip.DeviceDataset(ctx, Xs, ys)
    prog = srhip.Program(ctx, srhip.flatten(trees, o, dtype=np.float32), np.float32)
    _, nodes, _ = prog.info()
    rs = DeviceRowShard(prog, ds, o.elementwise_loss)
    rs.step()  # warm-up (code load, buffers, the first collective)
    barrier()
    ev, red = [], []
    t0 = time.perf_counter()
    for _ in range(args.rs_steps):
        rs.step()
        ev.append(rs.eval_ms)
        red.append(rs.reduce_ms)
    barrier()
    el = time.perf_counter() - t0
    vals = [el, float(np.mean(ev)), float(np.mean(red))]
    if dist:
        torch, tdist = dist
        t = torch.tensor(vals, dtype=torch.float64, device="cpu" if SHARED_GPU else "cuda")
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        vals = t.tolist()
    el, ev_ms, red_ms = vals
    _, ok = rs.result()
    return {
        "workload": f"config#5 row-sharded eval_loss: {args.rs_trees} trees (+ - * / cos exp) x {F} feat x {n} rows, "
                    f"L2, rows split over {world} GPU(s)",
        "metric": "node·row evals/sec (Float32), whole job",
        "value": float(nodes) * n * args.rs_steps / el,
        "unit": "node·row/s",
        "scaling": "strong",
        "steps": args.rs_steps,
        "ms_per_step": el * 1e3 / args.rs_steps,
        "eval_ms": ev_ms,
        "allreduce_ms": red_ms,
        "allreduce_bytes": 8 * (2 * args.rs_trees + 1),
        "rows_per_gpu": re - rb,
        "did_succeed": int(ok.sum()),
        "note": "eval_ms / allreduce_ms: mean over the timed steps, max over ranks (host clock around a "
                "synchronised stream / collective); all-reduce on the device buffer (RCCL, no host copy)",
    }


def stub_main(args, world, rank, dist):
    """Launcher test (no GPU): every rank reports its world and rank through
    the same barrier / max-over-ranks path; no evaluation, no metric."""
    import torch

    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    if dist:
        dist[1].barrier()
        dist[1].all_reduce(t, op=dist[1].ReduceOp.SUM)
    if rank == 0:
        print(json.dumps({"stub": True, "n_gpus": world, "rank_sum": float(t.item()), "steps": args.steps,
                          "warmup": args.warmup}))
    if dist:
        dist[1].destroy_process_group()


if __name__ == "__main__":
    main()
