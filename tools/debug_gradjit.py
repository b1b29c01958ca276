#!/usr/bin/env python3
"""Debug helper: the constants where the gradient tree code and the
forward-mode interpreter disagree (tests/test_jit_grad_gpu.py's case)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "symbolicregression.jl_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))
import srhip  # noqa: E402
from test_jit_grad_gpu import OPSETS, run, scales  # noqa: E402

opset, weighted = sys.argv[1], sys.argv[2] == "1"
b_ops, u_ops = OPSETS[opset]
o = srhip.Options(binary_operators=b_ops, unary_operators=u_ops)
rng = np.random.default_rng(5 + weighted)
n = 3001
X = rng.standard_normal((5, n)).astype(np.float32)
y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
w = np.abs(rng.standard_normal(n)).astype(np.float32) if weighted else None
trees = srhip.random_population(600, o, 5, np.float32, seed=91 + weighted)
s1, g1, _, ok1, info, prog = run(trees, o, X, y, w, True)
s0, g0, _, ok0, _, _ = run(trees, o, X, y, w, False)
print(info)
co = prog.flat.const_off
S, ref = scales(trees, o, X, y, w)
ok_c = np.repeat(ok1, np.diff(co))
owner = np.repeat(np.arange(len(trees)), np.diff(co))
for k in np.flatnonzero(ok_c):
    err = abs(g1[k] - g0[k])
    if not (err <= 1e-4 * S[k]):
        t = owner[k]
        print(f"tree {t} const {k - co[t]}: jit {g1[k]!r} interp {g0[k]!r} f64 {ref[k]!r} S {S[k]!r}\n   {trees[t]}")
