"""A/B of per-tree losses between library builds (SRHIP_LIB) on config #2
(4096 trees x 1M rows, FAST path): each build runs in its own process and
writes gpurun_out/ab_<tag>.npz; `compare` prints the trees that differ.
Usage: python tools/ab_losses.py run <tag> | compare <tagA> <tagB>"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd")]
import numpy as np  # noqa: E402

CFG = dict(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])


def run(tag):
    import srhip
    from srhip import constants as K
    o = srhip.Options(**CFG)
    trees = srhip.random_population(4096, o, 5, np.float32, seed=0)
    X = np.random.default_rng(1).standard_normal((5, 1_000_000)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    ctx = srhip.get_context(0)
    ds = srhip.DeviceDataset(ctx, X, y)
    prog = srhip.Program(ctx, srhip.flatten(trees, o, dtype=np.float32), np.float32)
    s, w, ok = prog.eval_loss(ds, K.LOSS["L2"])
    np.savez(ROOT / "gpurun_out" / f"ab_{tag}.npz", s=s, ok=ok, redo=np.array(ctx.last_jit_events()))
    print(tag, "ok", int(ok.sum()), "inf", int(np.isinf(s[ok]).sum()), "events", ctx.last_jit_events())


def compare(a, b):
    import srhip
    o = srhip.Options(**CFG)
    trees = srhip.random_population(4096, o, 5, np.float32, seed=0)
    A = np.load(ROOT / "gpurun_out" / f"ab_{a}.npz")
    B = np.load(ROOT / "gpurun_out" / f"ab_{b}.npz")
    d = np.flatnonzero((A["ok"] != B["ok"]) | ((A["s"] != B["s"]) & A["ok"]))
    print(f"{a} vs {b}: {d.size} trees differ")
    for t in d[:15]:
        print(t, A["ok"][t], B["ok"][t], A["s"][t], B["s"][t], srhip.string_tree(trees[t], o))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        compare(sys.argv[2], sys.argv[3])
