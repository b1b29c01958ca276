#!/usr/bin/env python3
"""Tree-code driver check: one config #2 batch through tree code and the
interpreter; did_succeed combinations and loss agreement (debugging aid)."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "symbolicregression.jl_amd"))
import srhip  # noqa: E402
from srhip import constants as K  # noqa: E402

nt = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
n = int(sys.argv[2]) if len(sys.argv) > 2 else 50_000
o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
rng = np.random.default_rng(1)
X = rng.standard_normal((5, n)).astype(np.float32)
y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
trees = srhip.random_population(nt, o, 5, np.float32, seed=0)
ctx = srhip.get_context(0)
ds = srhip.DeviceDataset(ctx, X, y)
flat = srhip.flatten(trees, o, dtype=np.float32)
res = {}
for mode in ("0", "1"):
    os.environ["SRHIP_JIT"] = mode
    os.environ["SRHIP_JIT_FAST"] = "0"
    prog = srhip.Program(ctx, flat, np.float32)
    res[mode] = prog.eval_loss(ds, K.LOSS["L2"])
    if mode == "1":
        print("jit_info", prog.jit_info(), "ran", ctx.last_tree_code())
(si, wi, oki), (sj, wj, okj) = res["0"], res["1"]
print("combos ok_i/ok_j:", {(a, b): int(((oki == a) & (okj == b)).sum()) for a in (0, 1) for b in (0, 1)})
m = oki & okj
rel = np.abs(sj[m] - si[m]) / np.abs(si[m])
print("both ok:", int(m.sum()), "rel>1e-5:", int((rel > 1e-5).sum()), "max rel", float(rel.max()) if rel.size else 0)
bad = np.flatnonzero(oki != okj)
print("first differing trees:", bad[:20].tolist())
for t in bad[:8]:
    print(t, "interp", oki[t], si[t], "jit", okj[t], sj[t], "nodes", int(flat.node_off[t + 1] - flat.node_off[t]))
