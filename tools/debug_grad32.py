"""Which constants of tests/test_jit_grad_gpu.py's batches leave the tight
bound against the oracle's Float32 gradients (1e-5·Σ|terms| + a 4-ulp move of
ŷ), for the tree code with the FAST forward, the tree code with the PRECISE
forward (SRHIP_GJIT_FAST=0, own process) and the interpreter. Prints one
JSON line per mode with the worst trees."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import numpy as np  # noqa: E402

import srhip  # noqa: E402
from test_jit_grad_gpu import OPSETS, run, scales32  # noqa: E402


def main():
    opset = sys.argv[1] if len(sys.argv) > 1 else "cfg5"
    weighted = len(sys.argv) > 2 and sys.argv[2] == "w"
    b_ops, u_ops = OPSETS[opset]
    o = srhip.Options(binary_operators=b_ops, unary_operators=u_ops)
    rng = np.random.default_rng(5 + weighted)
    n = 3001
    X = rng.standard_normal((5, n)).astype(np.float32)
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
    w = np.abs(rng.standard_normal(n)).astype(np.float32) if weighted else None
    trees = srhip.random_population(600, o, 5, np.float32, seed=91 + weighted)
    S32, G32, DV = scales32(trees, o, X, y, w)
    for label, gjit in (("tree_code", True), ("interpreter", False)):
        s, g, _, ok, info, prog = run(trees, o, X, y, w, gjit)
        co = prog.flat.const_off
        ok_c = np.repeat(ok, np.diff(co))
        tree_of = np.repeat(np.arange(len(trees)), np.diff(co))
        sel = ok_c & np.isfinite(S32) & np.isfinite(G32) & (S32 < 1e20)
        with np.errstate(invalid="ignore"):
            ratio = np.abs(g - G32) / (1e-5 * S32 + DV + 1e-30)
        bad = np.flatnonzero(sel & ~(ratio <= 1))
        worst = sorted(bad, key=lambda j: -ratio[j])[:8]
        print(json.dumps(dict(mode=label, fast=os.environ.get("SRHIP_GJIT_FAST", "1"), nbad=int(bad.size),
                              nsel=int(sel.sum()), worst=[dict(const=int(j), ratio=float(ratio[j]),
                                                               rel=float(abs(g[j] - G32[j]) / S32[j]),
                                                               tree=srhip.string_tree(trees[tree_of[j]], o))
                                                          for j in worst])), flush=True)


if __name__ == "__main__":
    main()
