"""Per-row output tree code (srhip_eval_tree_array through jit::Options::out;
VERDICT r03 missing 2): the tree code of a Float32 program stores each tile's
root values to the tree's output rows (one global_store_dwordx4 per wave and
tile) with the PRECISE routines only, every tile of every tree, as the
interpreter's MODE_OUT does. So its outputs are the interpreter's bit for bit
— failing trees' rows included — and did_succeed is the same; both are also
checked against the oracle's Float32 evaluation (eval_tree_array of
InterfaceDynamicExpressions.jl:50-52)."""
import os

import numpy as np
import pytest

import oracle
import srhip
from numerics import assert_close_conditioned, output_spread_flat
from srhip import constants as K

pytestmark = pytest.mark.gpu

OPSETS = {
    "cfg2": (["+", "-", "*", "/"], ["cos", "exp"]),
    "wide": (["+", "-", "*", "/", "^", "max", "min"], ["sin", "cos", "exp", "neg", "square", "cube", "abs",
                                                      "safe_log", "safe_sqrt", "tanh"]),
}


def _programs(ctx, flat, varying=False):
    progs = {}
    for mode in ("1", "0"):
        os.environ["SRHIP_JIT"] = mode
        try:
            progs[mode] = srhip.Program(ctx, flat, np.float32, varying_constants=varying)
        finally:
            del os.environ["SRHIP_JIT"]
    return progs


@pytest.mark.parametrize("opset", list(OPSETS))
def test_output_tree_code_equals_interpreter(gpu_ctx, opset):
    b_ops, u_ops = OPSETS[opset]
    o = srhip.Options(binary_operators=b_ops, unary_operators=u_ops)
    rng = np.random.default_rng(17)
    n = 30_001  # a partial last tile
    X = rng.standard_normal((5, n)).astype(np.float32)
    y = np.zeros(n, np.float32)
    trees = srhip.random_population(700, o, 5, np.float32, seed=18)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    ctx = gpu_ctx
    ds = srhip.DeviceDataset(ctx, X, y)
    progs = _programs(ctx, flat)
    out1, ok1 = progs["1"].eval_tree_array(ds)
    ran = ctx.last_tree_code()
    out0, ok0 = progs["0"].eval_tree_array(ds)
    assert ctx.last_tree_code() == 0
    assert ran >= 0.7 * len(trees), ran
    assert np.array_equal(ok1, ok0)
    np.testing.assert_array_equal(out1, out0)  # every tree, failing ones included (NaN where NaN)
    # against the oracle's Float32 evaluation on the succeeding trees
    ref, rok = oracle.eval_trees(flat, X, np.float32)
    assert np.array_equal(ok1, rok.astype(bool))
    # condition-aware (numerics.py): per row, cancellations amplify the
    # per-operator rounding differences (tanh, ^, safe_log in f32) far past 1e-5
    m = np.flatnonzero(ok1)
    spread = output_spread_flat(flat, X, np.float32)
    assert_close_conditioned(out1[m], ref[m], spread[m], rtol=1e-5, atol=1e-6, msg=f"{opset} outputs")


def test_output_tree_code_after_new_constants(gpu_ctx):
    """Memory-constant programs (set_constants without new code): the output
    code reads the new constants too."""
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(19)
    n = 5000
    X = rng.standard_normal((4, n)).astype(np.float32)
    trees = srhip.random_population(600, o, 4, np.float32, seed=20)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    ctx = gpu_ctx
    ds = srhip.DeviceDataset(ctx, X, np.zeros(n, np.float32))
    progs = _programs(ctx, flat, varying=True)
    newc = (flat.consts * np.float32(1.25) + np.float32(0.5)).astype(np.float32)
    for p in progs.values():
        p.set_constants(newc)
    out1, ok1 = progs["1"].eval_tree_array(ds)
    assert ctx.last_tree_code() > 300
    out0, ok0 = progs["0"].eval_tree_array(ds)
    assert np.array_equal(ok1, ok0)
    np.testing.assert_array_equal(out1, out0)


@pytest.mark.parametrize("varying", [False, True])
def test_output_tree_code_dynamic_deal_equals_static(gpu_ctx, varying):
    """sr_jit_out_d / sr_jit_out_md (jit_template.hip jit_eval_body DYN: the
    waves take their trees from an LDS counter, as the loss loops do) against
    the static deal (SRHIP_JIT_DYNLOOP=0, read per launch): the same per-row
    outputs bit for bit, every tree (VERDICT r05 missing 4)."""
    if os.environ.get("SRHIP_JIT_DYNLOOP") == "0":
        pytest.skip("the static tree loops are forced for the whole run (tools/gpu_run.sh variants)")
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(23)
    n = 20_001
    X = rng.standard_normal((5, n)).astype(np.float32)
    trees = srhip.random_population(1500, o, 5, np.float32, seed=24)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    ctx = gpu_ctx
    ds = srhip.DeviceDataset(ctx, X, np.zeros(n, np.float32))
    prog = _programs(ctx, flat, varying=varying)["1"]
    if varying:
        prog.set_constants((flat.consts * np.float32(0.75)).astype(np.float32))
    out_d, ok_d = (np.array(v, copy=True) for v in prog.eval_tree_array(ds))
    assert ctx.last_tree_code() > 1000
    assert ctx.last_kernel_name() == ("sr_jit_out_md" if varying else "sr_jit_out_d")
    os.environ["SRHIP_JIT_DYNLOOP"] = "0"
    try:
        out_s, ok_s = prog.eval_tree_array(ds)
        assert ctx.last_kernel_name() == ("sr_jit_out_m" if varying else "sr_jit_out")
    finally:
        del os.environ["SRHIP_JIT_DYNLOOP"]
    assert np.array_equal(ok_d, ok_s)
    np.testing.assert_array_equal(out_d, out_s)
