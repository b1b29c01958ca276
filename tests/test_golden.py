"""Golden vectors (tests/golden/golden.npz, made by tests/golden/make_golden.py).

CPU: the oracle reproduces every fixture bit for bit (guards the restatement
that the reference's known-answer tests pin). GPU: the engine, called through
the C ABI (srhip_program_create / srhip_eval_tree_array / srhip_eval_loss),
matches the fixtures — did_succeed exactly; per-row outputs bit-exact for
trees made only of + - * /, within the per-operator bound (≤ 4 ulp,
propagated through the tree by the oracle's ulp-perturbation spread)
otherwise; losses within 1e-5 relative (f32) / 1e-10 (f64).
"""
from pathlib import Path

import numpy as np
import pytest

import oracle
import srhip
from numerics import assert_close_conditioned, loss_spread_flat, output_spread_flat
from srhip import constants as K

G = np.load(Path(__file__).parent / "golden" / "golden.npz", allow_pickle=False)
CASES = sorted({k.split("/")[0] for k in G.files})
EXACT_BOPS = {K.BOP[n] for n in ("ADD", "SUB", "MUL", "DIV")}


def case(name):
    g = {k.split("/", 1)[1]: G[k] for k in G.files if k.startswith(name + "/")}
    nodes = np.diff(g["node_off"]).astype(np.int64)
    flat = srhip.node.FlatTrees(g["node_off"], g["kind"], g["arg"], g["const_off"], g["consts"], nodes)
    return g, flat


def test_cases_present():
    assert {"cfg1_f32", "cfg2_f32", "cfg3_f64", "grid_f32", "grid_f64"} <= set(CASES)


@pytest.mark.parametrize("name", CASES)
def test_oracle_reproduces_golden(name):
    g, flat = case(name)
    T = g["X"].dtype
    out, ok = oracle.eval_trees(flat, g["X"], dtype=T)
    assert np.array_equal(ok, g["ok"])
    assert np.array_equal(out[ok], g["out"][ok], equal_nan=True)
    sums, losses, lok = oracle.eval_loss_batch(flat, g["X"], g["y"], dtype=T)
    assert np.array_equal(lok, g["loss_ok"])
    assert np.array_equal(sums, g["loss_sum"], equal_nan=True)


def _exact_tree(g, t):
    b, e = g["node_off"][t], g["node_off"][t + 1]
    kind, arg = g["kind"][b:e], g["arg"][b:e]
    if np.any(kind == K.NODE_UNARY):
        return False
    return all(int(a) in EXACT_BOPS for a in arg[kind == K.NODE_BINARY])


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_engine_matches_golden(gpu_ctx, name):
    g, flat = case(name)
    T = g["X"].dtype
    prog = srhip.Program(gpu_ctx, flat, T)
    ds = srhip.DeviceDataset(gpu_ctx, np.ascontiguousarray(g["X"]), g["y"])
    out, ok = prog.eval_tree_array(ds)
    assert np.array_equal(ok, g["ok"]), f"did_succeed differs on trees {np.flatnonzero(ok != g['ok'])}"
    spread = output_spread_flat(flat, g["X"], T)
    rtol = 1e-5 if T == np.float32 else 1e-12
    nexact = 0
    for t in np.flatnonzero(ok):
        if _exact_tree(g, t):
            assert np.array_equal(out[t], g["out"][t]), f"{name} tree {t}: + - * / tree not bit-exact"
            nexact += 1
        else:
            assert_close_conditioned(out[t], g["out"][t], spread[t], rtol=rtol, atol=rtol,
                                     msg=f"{name} tree {t}")
    if name.startswith("cfg"):
        assert nexact > 0
    sums, _, lok = prog.eval_loss(ds, K.LOSS["L2"])
    assert np.array_equal(lok, g["loss_ok"])
    m = lok & np.isfinite(g["loss_sum"])
    lsp = loss_spread_flat(flat, g["X"], g["y"], None, T, srhip.options.L2DistLoss())
    assert_close_conditioned(sums[m], g["loss_sum"][m], lsp[m], rtol=1e-5 if T == np.float32 else 1e-10,
                             msg=f"{name} loss sums")
