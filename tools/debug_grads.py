#!/usr/bin/env python3
"""The gradient comparisons of tests/test_jit_grad_gpu.py::
test_grad_tree_code_matches_interpreter_and_oracle for every parametrisation
(GPU box): the fraction of constants beyond the bound in each comparison and
the worst constants, with their tree, both GPU values, the Float64 value, S
and N; the tight comparisons against the oracle's Float32 gradients too.
Usage: python tools/debug_grads.py [OPSET ...]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import numpy as np  # noqa: E402

import srhip  # noqa: E402
from test_jit_grad_gpu import OPSETS, S_MAX, run, scales, scales32  # noqa: E402


def report(g, ref, S, N, ok_c, rtol, owner, trees, o, msg, cond=None, N64=None):
    sel = ok_c & np.isfinite(S) & np.isfinite(ref) & (S < S_MAX) & np.isfinite(N)
    if cond is not None:
        sel &= cond
    with np.errstate(invalid="ignore", divide="ignore"):
        err = np.abs(g - ref)
        bound = rtol * S + 1e-30 + 4 * N
        r = err / bound
    same = (g == ref) | (np.isnan(g) & np.isnan(ref))
    bad = sel & ~same & ~(err <= bound)
    print(f"  {msg}: {int(bad.sum())} of {int(sel.sum())} beyond ({bad.sum() / max(sel.sum(), 1):.4f})", flush=True)
    for j in np.flatnonzero(bad)[np.argsort(-r[bad])][:4]:
        t = owner[j]
        print(f"    const {j} (tree {t}): got {g[j]:.6g} ref {ref[j]:.6g} S {S[j]:.3g} N {N[j]:.3g} err/bound {r[j]:.1f}"
              + (f" N64/S {N64[j] / S[j]:.2g}" if N64 is not None else "")
              + f"\n      {srhip.string_tree(trees[t], o)[:160]}", flush=True)


def main():
    for opset in sys.argv[1:] or OPSETS:
        for weighted in (False, True):
            b_ops, u_ops = OPSETS[opset]
            o = srhip.Options(binary_operators=b_ops, unary_operators=u_ops)
            rng = np.random.default_rng(5 + weighted)
            n = 3001
            X = rng.standard_normal((5, n)).astype(np.float32)
            if opset == "cfg3":
                X = (np.abs(X) + np.float32(0.1)).astype(np.float32)
            y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
            w = np.abs(rng.standard_normal(n)).astype(np.float32) if weighted else None
            trees = srhip.random_population(600 if opset != "cfg3" else 1500, o, 5, np.float32, seed=91 + weighted)
            s1, g1, w1, ok1, info, prog = run(trees, o, X, y, w, True)
            s0, g0, w0, ok0, info0, _ = run(trees, o, X, y, w, False)
            co = prog.flat.const_off
            owner = np.repeat(np.arange(len(trees)), np.diff(co))
            ok_c = np.repeat(ok1, np.diff(co))
            S, ref, N = scales(trees, o, X, y, w, with_noise=True)
            print(f"== {opset} weighted={weighted}", flush=True)
            report(g1, g0, S, N, ok_c, 1e-4, owner, trees, o, "tree code vs interpreter")
            report(g1, ref, S, N, ok_c, 1e-4, owner, trees, o, "tree code vs Float64 oracle")
            report(g0, ref, S, N, ok_c, 1e-4, owner, trees, o, "interpreter vs Float64 oracle")
            S32, G32, DV = scales32(trees, o, X, y, w)
            report(g1, G32, S32, DV / 4, ok_c, 1e-5, owner, trees, o, "tree code vs Float32 oracle", None, N)
            report(g0, G32, S32, DV / 4, ok_c, 1e-5, owner, trees, o, "interpreter vs Float32 oracle", None, N)


if __name__ == "__main__":
    main()
