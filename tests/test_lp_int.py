"""LPDistLoss{n} with an INTEGER n (SRHIP_LOSS_LPINT): Julia
evaluates abs(r)^P with P an Int by its T^Integer methods (Base math.jl,
Julia 1.9+), not by the Float64 pow of LPDistLoss(3.0):

- Float32: x*x*x for n = 3 and (1/x)^2 for n = -2 in Float32 (literal_pow's
  rounding), otherwise Base.power_by_squaring in Float64 rounded once;
- Float64: pow_body's compensated power by squaring.

LossFunctions' deriv is P * abs(r)^(P-1) * sign(r) in T. Julia's Base is not in
/root/reference and Julia is absent, so the rules are restated from its
published source: parity unpinned beyond that restatement. The CPU tests pin
the oracle against an independent Python restatement (and the Float64 values
within an ulp of the exact rational power); the GPU tests check the
element values of the tree code's integer-n loss routine (gen_jit.py /
gen_jit64.py l_lpint, d_lpint: the interpreter's device_ops.h code) bit for
bit against the oracle through one-row datasets (ŷ = x1·c = c, y = 0), their
gradients, and the sums at size against the interpreter and the oracle.
"""
import os
from fractions import Fraction

import numpy as np
import pytest

import oracle
import srhip
from srhip import constants as K
from numerics import assert_loss_tail

F32 = np.float32


def _pbs(x: float, p: int) -> float:
    """Base.power_by_squaring (intfuncs.jl) in Python floats (Float64)."""
    if p == 0:
        return 1.0
    if p == 1:
        return x
    if p == 2:
        return x * x
    t = ((p & -p).bit_length() - 1) + 1
    p >>= t
    t -= 1
    while t > 0:
        x = x * x
        t -= 1
    y = x
    while p > 0:
        t = ((p & -p).bit_length() - 1) + 1
        p >>= t
        t -= 1
        while t >= 0:
            x = x * x
            t -= 1
        y = y * x
    return y


def _ipow_f32(x, n: int):
    x = F32(x)
    with np.errstate(all="ignore"):
        if n == -2:
            i = F32(1) / x
            return i * i
        if n == 3:
            return x * x * x
        if n < 0:
            return F32(_pbs(1.0 / float(x), -n)) if x != 0 else F32(np.inf)
        return F32(_pbs(float(x), n))


def test_python_constructor_picks_the_integer_kind():
    assert srhip.LPDistLoss(3).kind == K.LOSS["LPINT"] and srhip.LPDistLoss(3).params == [3.0]
    assert srhip.LPDistLoss(np.int64(4)).kind == K.LOSS["LPINT"]
    assert srhip.LPDistLoss(3.0).kind == K.LOSS["LP"]
    assert K.LOSS["LPINT"] == 10


@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 5, 7, 10, 13, -1, -2, -3, -5])
def test_oracle_float32_integer_power(n):
    rng = np.random.default_rng(100 + n)
    xs = np.concatenate([rng.standard_normal(400) * 3, rng.uniform(0.9, 1.1, 200), [0.0, 1.0, -1.0, 2.0, 0.5]])
    for x in xs.astype(F32):
        got = F32(oracle.elem_loss(K.LOSS["LPINT"], [float(n)], x, F32(0), dtype=F32))
        want = _ipow_f32(abs(x), n)
        assert (got == want) or (np.isnan(got) and np.isnan(want)), (n, float(x), float(got), float(want))


def test_float32_cube_is_literal_pow_not_rounded_once():
    """n = 3 keeps Float32 x*x*x: some |r| where that differs from the Float64
    cube rounded once (what LPDistLoss(3.0) gives)."""
    rng = np.random.default_rng(5)
    xs = np.abs(rng.standard_normal(20000)).astype(F32)
    diff = 0
    for x in xs[:2000]:
        a = F32(oracle.elem_loss(K.LOSS["LPINT"], [3.0], x, F32(0), dtype=F32))
        b = F32(oracle.elem_loss(K.LOSS["LP"], [3.0], x, F32(0), dtype=F32))
        assert a == x * x * x
        diff += a != b
    assert diff > 0


@pytest.mark.parametrize("n", [2, 3, 4, 5, 7, 11, 25, -1, -2, -3, -6])
def test_oracle_float64_integer_power_within_an_ulp(n):
    rng = np.random.default_rng(200 + n)
    xs = np.abs(np.concatenate([rng.standard_normal(300) * 2, rng.uniform(0.95, 1.05, 100)]))
    exact_hits = 0
    for x in xs:
        got = oracle.elem_loss(K.LOSS["LPINT"], [float(n)], float(x), 0.0, dtype=np.float64)
        ex = Fraction(float(x)) ** n
        want = float(ex)  # correctly rounded
        if n == 3:  # x*x*x (literal_pow): two roundings
            assert got == (x * x) * x
            continue
        if n == -2:
            assert got == (1.0 / x) * (1.0 / x)
            continue
        assert abs(Fraction(got) - ex) <= Fraction(np.spacing(want)), (n, x, got, want)
        exact_hits += got == want
    if n not in (3, -2):
        assert exact_hits >= 0.95 * len(xs)


# ---- GPU: the interpreter -------------------------------------------------------

def _const_trees(cs, dtype):
    """x1 * c per constant: with x1 = 1 the prediction is c exactly."""
    o = srhip.Options(binary_operators=["+", "*"], unary_operators=[])
    trees = [o.make_binary("*", srhip.Node("x1"), srhip.Node(val=dtype(c))) for c in cs]
    return o, srhip.flatten(trees, o, dtype=dtype)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("n", [2, 3, 4, 5, -2, -3])
def test_gpu_integer_lp_values_bit_exact(gpu_ctx, dtype, n):
    rng = np.random.default_rng(300 + n)
    cs = np.concatenate([rng.standard_normal(700) * 2, rng.uniform(0.9, 1.1, 300)]).astype(dtype)
    o, flat = _const_trees(cs, dtype)
    X = np.ones((1, 1), dtype=dtype)
    y = np.zeros(1, dtype=dtype)
    ds = srhip.DeviceDataset(gpu_ctx, X, y)
    prog = srhip.Program(gpu_ctx, flat, dtype)
    loss = srhip.LPDistLoss(n)
    s, wsum, ok = prog.eval_loss(ds, loss.kind, loss.params)
    assert wsum == 1.0 and ok.all()
    want = np.array([oracle.elem_loss(loss.kind, loss.params, dtype(c), dtype(0), dtype=dtype) for c in cs])
    np.testing.assert_array_equal(s.astype(dtype), want.astype(dtype))
    assert gpu_ctx.last_tree_code() > 900  # constant trees: tree code with the integer-n loss routine
    # gradient: dℓ/dc = n |c|^(n-1) sign(c) in T (gradient tree code seeded by the dℓ/dr routine)
    s2, g, w2, ok2 = prog.eval_loss_grad(ds, loss.kind, loss.params)
    assert ok2.all()
    with np.errstate(all="ignore"):
        if dtype == np.float32:
            want_g = np.array([F32(n) * _ipow_f32(abs(c), n - 1) * np.sign(c) for c in cs], dtype=F32)
        else:
            want_g = np.array([n * oracle.elem_loss(loss.kind, [float(n - 1)], abs(float(c)), 0.0, dtype=np.float64)
                               * np.sign(c) for c in cs])
    np.testing.assert_array_equal(np.asarray(g).astype(dtype), want_g.astype(dtype))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_gpu_integer_lp_sums_match_oracle(gpu_ctx, dtype):
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(77)
    n = 20_001
    X = rng.standard_normal((5, n)).astype(dtype)
    y = (2 * np.cos(X[3]) + X[0] * X[0] - 2).astype(dtype)
    w = np.abs(rng.standard_normal(n)).astype(dtype)
    trees = srhip.random_population(512, o, 5, dtype, seed=78)
    flat = srhip.flatten(trees, o, dtype=dtype)
    progs = {}
    for mode in ("1", "0"):
        os.environ["SRHIP_JIT"] = mode
        try:
            progs[mode] = srhip.Program(gpu_ctx, flat, dtype)
        finally:
            del os.environ["SRHIP_JIT"]
    prog = progs["1"]
    for p in (3, 4):
        loss = srhip.LPDistLoss(p)
        for weights in (None, w):
            ds = srhip.DeviceDataset(gpu_ctx, X, y, weights)
            s, wsum, ok = prog.eval_loss(ds, loss.kind, loss.params)
            assert gpu_ctx.last_tree_code() > 300  # the integer-n loss routine in the tile tail
            si, wi, oki = progs["0"].eval_loss(ds, loss.kind, loss.params)
            assert gpu_ctx.last_tree_code() == 0 and wi == wsum and np.array_equal(ok, oki)
            mi = ok & np.isfinite(si) & (si != 0)
            with np.errstate(invalid="ignore", divide="ignore"):
                reli = np.abs(s - si) / np.abs(si)
            assert np.all(reli[mi] <= (1e-5 if dtype == np.float32 else 1e-11)), float(np.nanmax(reli[mi]))
            _, rl, rok = oracle.eval_loss_batch(flat, X, y, weights, loss.kind, loss.params, dtype=dtype, nthreads=16)
            assert np.array_equal(ok, rok)
            m = ok & np.isfinite(rl) & (rl != 0)
            with np.errstate(invalid="ignore", divide="ignore"):
                rel = np.abs(s / wsum - rl) / np.abs(rl)
            assert m.sum() > 100
            if dtype == np.float32:
                assert np.all(rel[m] <= 1e-5), float(np.nanmax(rel[m]))
            else:
                # a few trees of this population take cos / exp of huge or cancelling
                # arguments, where 1-ulp device / host differences move the value
                # anywhere (as in test_jit64_gpu's losses): 95 % within 1e-9 of the
                # oracle, and every tree's integer-n sum within 1e-12 of the same
                # engine's LPDistLoss(float(n)) sum, whose element values differ by
                # the few ulp of x*x*x / pow_body vs pow (the conditioning of the
                # tree is then the same on both sides)
                # every tree within 1e-9, or within 4x the oracle's perturbation spread
                assert_loss_tail(f"lp_int_f64_p{p}_{'w' if weights is not None else 'u'}", s / wsum, rl, m, flat,
                                 X, y, weights, dtype, loss.kind, loss.params, rtol=1e-9)
                assert np.median(rel[m]) <= 1e-13, np.sort(rel[m])[-5:]
                sf, wf, okf = prog.eval_loss(ds, K.LOSS["LP"], [float(p)])
                assert np.array_equal(ok, okf) and wf == wsum
                mf = ok & np.isfinite(sf) & (sf != 0)
                with np.errstate(invalid="ignore", divide="ignore"):
                    relf = np.abs(s - sf) / np.abs(sf)
                assert np.all(relf[mf] <= 1e-12), float(np.nanmax(relf[mf]))
    with pytest.raises(Exception, match="integer n"):  # srhip.h: INVALID for a non-integral n
        prog.eval_loss(ds, K.LOSS["LPINT"], [2.5])


@pytest.mark.gpu
@pytest.mark.parametrize("p", [2.5, 0.5, 1.7])
def test_gpu_fractional_lp_values_within_an_ulp_of_pow(gpu_ctx, p):
    """LPDistLoss(p) with a non-integer p on Float32 data: Julia promotes the
    residual to Float64 and takes pow; the engine takes exp(p·ln|r|) in
    Float64 (device_ops.h lp_pow, relative error ~2^-44), rounded to Float32
    once. Bound: every element value and dℓ/dc within 1 ulp (Float32) of the
    Float64 pow rounded once, and at most 2 of 1000 values not bit-equal (a
    rounding boundary within 2^-44 relative is that rare)."""
    rng = np.random.default_rng(int(p * 10))
    cs = np.concatenate([rng.standard_normal(700) * 3, rng.uniform(0.9, 1.1, 300)]).astype(F32)
    o, flat = _const_trees(cs, F32)
    X = np.ones((1, 1), dtype=F32)
    y = np.zeros(1, dtype=F32)
    ds = srhip.DeviceDataset(gpu_ctx, X, y)
    prog = srhip.Program(gpu_ctx, flat, F32)
    s, wsum, ok = prog.eval_loss(ds, K.LOSS["LP"], [p])
    assert ok.all()
    want = np.array([F32(abs(float(c)) ** p) for c in cs], dtype=F32)
    got = s.astype(F32)
    ulp = np.abs(got.view(np.int32).astype(np.int64) - want.view(np.int32).astype(np.int64))
    assert ulp.max() <= 1 and (ulp > 0).sum() <= 2, (int(ulp.max()), int((ulp > 0).sum()))
    _, g, _, ok2 = prog.eval_loss_grad(ds, K.LOSS["LP"], [p])
    assert ok2.all()
    want_g = np.array([F32(p * abs(float(c)) ** (p - 1) * np.sign(float(c))) for c in cs], dtype=F32)
    got_g = np.asarray(g).astype(F32)
    ulp_g = np.abs(got_g.view(np.int32).astype(np.int64) - want_g.view(np.int32).astype(np.int64))
    assert ulp_g.max() <= 1 and (ulp_g > 0).sum() <= 2, (int(ulp_g.max()), int((ulp_g > 0).sum()))
