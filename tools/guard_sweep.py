"""Round-4 loss-parity guards: one setting (thresholds from the environment:
SRHIP_JIT_CAN_LOG2, SRHIP_JIT_EXP_GUARD_LOG2, SRHIP_JIT_TRIG_GUARD_LOG2,
SRHIP_JIT_STICKY) measured on config #2's parity batch (tools/fast_parity.py:
4096 trees, seed 0, 1M rows): trees outside 1e-5 of the oracle, the worst
relative loss error, did_succeed mismatches, PRECISE-redone tiles and the
kernel time (median of 10 calls). The oracle's losses are cached in
gpurun_out/ so a sweep runs it once. Prints one JSON line."""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd"), str(ROOT / "oracle"), str(ROOT / "tools")]
import numpy as np  # noqa: E402

import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402
from fast_parity import workload  # noqa: E402


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else "default"
    o, trees, X, y = workload("cfg2")
    n = X.shape[1]
    flat = srhip.flatten(trees, o, dtype=np.float32)
    cache = ROOT / "gpurun_out" / "guard_sweep_oracle.npz"
    if cache.exists():
        z = np.load(cache)
        ref_l, ref_ok = z["l"], z["ok"]
    else:
        import oracle

        _, ref_l, ref_ok = oracle.eval_loss_batch(flat, X, y, dtype=np.float32, nthreads=16)
        cache.parent.mkdir(exist_ok=True)
        np.savez(cache, l=ref_l, ok=ref_ok)
    ctx = srhip.get_context(0)
    ds = srhip.DeviceDataset(ctx, X, y)
    os.environ["SRHIP_JIT"] = "1"
    prog = srhip.Program(ctx, flat, np.float32)
    s, w, ok = prog.eval_loss(ds, K.LOSS["L2"])
    redone = int(ctx.last_jit_events()[1])
    kms = []
    for _ in range(10):
        prog.eval_loss(ds, K.LOSS["L2"])
        kms.append(ctx.last_kernel_time()[0])
    losses = s / n
    m = ok & ref_ok & np.isfinite(ref_l)
    with np.errstate(invalid="ignore", divide="ignore"):
        rel = np.abs(losses - ref_l.astype(np.float64)) / np.abs(ref_l.astype(np.float64))
    bad = np.flatnonzero(m & ~(rel <= 1e-5))
    out = dict(label=label, env={k: v for k, v in os.environ.items() if k.startswith("SRHIP_JIT_")},
               did_succeed_mismatch=int((ok != ref_ok).sum()), succeeding=int(m.sum()), outside_1e5=int(bad.size),
               max_rel=float(np.nanmax(np.where(m, rel, 0))), worst=[int(t) for t in np.argsort(-np.where(m, rel, 0))[:5]],
               redone_tiles=redone, kernel_ms=float(np.median(kms)))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
