"""Loss-parity guard thresholds over several config #2-shaped batches (4096
trees of random_population seed S, maxsize 30 like bench.py, 1M rows): for
each setting of SRHIP_JIT_CAN_LOG2 / SRHIP_JIT_EXP_GUARD_LOG2 /
SRHIP_JIT_TRIG_GUARD_LOG2 (read once per process: compiled into the tree
code), trees outside 1e-5 of the oracle, the worst relative loss error,
did_succeed mismatches, tiles redone and the kernel time (median of 8
calls). Usage: KC=.. TE=.. TT=.. guard_seeds.py SEED[,SEED...] LABEL
(tools/guard_seeds.sh runs one process per setting). The oracle's losses are
cached per seed under gpurun_out/. One JSON line per seed."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd"), str(ROOT / "oracle")]
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402


def main():
    seeds = [int(s) for s in sys.argv[1].split(",")]
    label = sys.argv[2]
    kc, te, tt = (int(os.environ[k]) for k in ("KC", "TE", "TT"))
    os.environ.update({"SRHIP_JIT_CAN_LOG2": str(kc), "SRHIP_JIT_EXP_GUARD_LOG2": str(te),
                       "SRHIP_JIT_TRIG_GUARD_LOG2": str(tt), "SRHIP_JIT": "1"})
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(1)
    X = rng.standard_normal((5, 1_000_000)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    n = X.shape[1]
    ctx = srhip.get_context(0)
    ds = srhip.DeviceDataset(ctx, X, y)
    for seed in seeds:
        trees = srhip.random_population(4096, o, 5, np.float32, seed=seed, maxsize=30)
        flat = srhip.flatten(trees, o, dtype=np.float32)
        cache = ROOT / "gpurun_out" / f"guard_oracle_{seed}.npz"
        if cache.exists():
            z = np.load(cache)
            ref_l, ref_ok = z["l"], z["ok"]
        else:
            _, ref_l, ref_ok = oracle.eval_loss_batch(flat, X, y, dtype=np.float32, nthreads=16)
            cache.parent.mkdir(exist_ok=True)
            np.savez(cache, l=ref_l, ok=ref_ok)
        prog = srhip.Program(ctx, flat, np.float32)
        s, _, ok = prog.eval_loss(ds, K.LOSS["L2"])
        s, ok = s.copy(), ok.copy()
        redone = int(ctx.last_jit_events()[1])
        kms = []
        for _ in range(8):
            prog.eval_loss(ds, K.LOSS["L2"])
            kms.append(ctx.last_kernel_time()[0])
        losses = s / n
        m = ok & ref_ok & np.isfinite(ref_l)
        with np.errstate(invalid="ignore", divide="ignore"):
            rel = np.abs(losses - ref_l.astype(np.float64)) / np.abs(ref_l.astype(np.float64))
        relm = np.where(m, rel, 0.0)
        print(json.dumps(dict(seed=seed, label=label, kc=kc, te=te, tt=tt,
                              did_succeed_mismatch=int((ok != ref_ok).sum()), succeeding=int(m.sum()),
                              outside_1e5=int((m & ~(rel <= 1e-5)).sum()), max_rel=float(np.nanmax(relm)),
                              redone_tiles=redone, kernel_ms=float(np.median(kms)))), flush=True)


if __name__ == "__main__":
    main()
