"""Batched constant optimisation (srhip.optimize_constants_batch), the
batched form of optimize_constants (src/ConstantOptimization.jl:22-65).

CPU tests drive the same optimiser over the oracle (forward-mode gradients of
the C restatement, L2 loss in fp64): known-answer recoveries in the spirit of
test/test_optimizer_mutation.jl / test_derivatives.jl. GPU tests run it on the
engine and compare with the oracle-driven run."""
import numpy as np
import pytest

import oracle
import srhip
from srhip import Node


class OracleEvaluator:
    """Test-only evaluator: loss and ∂L/∂c of every candidate on the CPU oracle."""

    def __init__(self, cands, options, X, y):
        self.flat = srhip.flatten(cands, options, dtype=np.float64)
        self.X, self.y = X.astype(np.float64), y.astype(np.float64)

    def _one(self, t, c):
        k, a, _ = self.flat.tree(t)
        out, g, ok = oracle.eval_grad_consts(k, a, c, self.X, len(c))
        if not ok:
            return np.inf, np.full(len(c), np.nan)
        r = out - self.y
        return float(np.mean(r * r)), 2.0 * (g @ r) / len(r)

    def loss_grad(self, consts):
        co = self.flat.const_off
        fs, gs = [], []
        for t in range(self.flat.ntrees):
            f, g = self._one(t, np.asarray(consts[co[t]:co[t + 1]], dtype=np.float64))
            fs.append(f)
            gs.append(g)
        return np.asarray(fs), (np.concatenate(gs) if gs else np.zeros(0))

    def loss_only(self, consts):
        return self.loss_grad(consts)[0]


def problem(T=np.float64, n=200, seed=1):
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((5, n)).astype(T)
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(T)
    B, U = o.make_binary, o.make_unary
    x1, x4 = Node("x1"), Node("x4")
    three = B("+", B("+", B("*", Node(val=1.0), U("cos", x4)), B("*", Node(val=0.5), B("*", x1, x1))),
              Node(val=0.0))
    one = B("+", B("*", Node(val=0.7), U("cos", Node("x4"))), B("-", B("*", Node("x1"), Node("x1")),
                                                                  Node(val=2.0)))
    none = B("*", Node("x1"), Node("x1"))
    return o, X, y, [three, one, none]


def oracle_factory(o, X, y):
    return lambda cands: OracleEvaluator(cands, o, X, y)


def test_recovers_constants_on_oracle():
    o, X, y, trees = problem()
    ds = srhip.Dataset(X, y)
    res = srhip.optimize_constants_batch(ds, trees, o, rng=np.random.default_rng(0),
                                         evaluator_factory=oracle_factory(o, X, y))
    assert res.converged[0] and res.converged[1]
    assert np.allclose(srhip.get_constants(trees[0]), [2.0, 1.0, -2.0], atol=1e-6)
    assert np.allclose(srhip.get_constants(trees[1]), [2.0, 2.0], atol=1e-6)  # BFGS, 2 constants
    assert res.losses[0] < 1e-10 and res.losses[1] < 1e-10
    assert not res.converged[2] and res.num_evals[2] == 0  # no constants: untouched (:27-29)
    assert res.num_evals[0] > 3 and res.num_evals[1] > 3


def test_not_converged_keeps_x0():
    """With one iteration nothing converges: constants go back to x0 (:61-63)."""
    o, X, y, trees = problem()
    o.optimizer_iterations = 1
    x0 = [srhip.get_constants(t) for t in trees]
    ds = srhip.Dataset(X, y)
    res = srhip.optimize_constants_batch(ds, trees, o, rng=np.random.default_rng(0),
                                         evaluator_factory=oracle_factory(o, X, y))
    assert not res.converged[0]
    assert srhip.get_constants(trees[0]) == x0[0]


def test_failing_tree_stays_failed():
    o, X, y, _ = problem()
    # exp(exp(c * x1)) overflows on every start → loss Inf, never converges
    t = o.make_unary("exp", o.make_unary("exp", o.make_binary("*", Node(val=40.0), Node("x1"))))
    ds = srhip.Dataset(X, y)
    res = srhip.optimize_constants_batch(ds, [t], o, rng=np.random.default_rng(0),
                                         evaluator_factory=oracle_factory(o, X, y))
    assert not res.converged[0] and np.isinf(res.losses[0])
    assert srhip.get_constants(t) == [40.0]


def test_nelder_mead_recovers_constants_on_oracle():
    """optimizer_algorithm = "NelderMead" (ConstantOptimization.jl:35-36): the
    3- and 2-constant trees go through the batched Nelder-Mead, a 1-constant
    tree still through Newton (:32-33)."""
    o, X, y, trees = problem()
    B, U = o.make_binary, o.make_unary
    x1, x4 = Node("x1"), Node("x4")
    single = B("-", B("+", B("+", U("cos", x4), U("cos", x4)), B("*", x1, x1)), Node(val=1.5))
    trees.append(single)
    o.optimizer_algorithm = "NelderMead"
    o.optimizer_iterations = 600
    ds = srhip.Dataset(X, y)
    res = srhip.optimize_constants_batch(ds, trees, o, rng=np.random.default_rng(0),
                                         evaluator_factory=oracle_factory(o, X, y))
    assert res.converged[0] and res.converged[1] and res.converged[3]
    assert np.allclose(srhip.get_constants(trees[0]), [2.0, 1.0, -2.0], atol=1e-3)
    assert np.allclose(srhip.get_constants(trees[1]), [2.0, 2.0], atol=1e-3)
    assert np.allclose(srhip.get_constants(trees[3]), [2.0], atol=1e-9)  # Newton: exact
    assert res.losses[0] < 1e-6 and res.losses[3] < 1e-12
    assert res.num_evals[0] > 3 * 8  # 3 starts, each at least its simplex and a few iterations


def test_nelder_mead_default_iterations_never_worse():
    """8 iterations (Options.jl optimizer_iterations): a converged start only
    replaces x0 when its loss is the minimum; else x0 stays (:56-63)."""
    o, X, y, _ = problem()
    o.optimizer_algorithm = "NelderMead"
    pop = srhip.random_population(40, o, 5, np.float64, seed=11, maxsize=15)
    pop = [t for t in pop if len(srhip.get_constants(t)) >= 2]
    assert len(pop) >= 5
    x0 = [list(srhip.get_constants(t)) for t in pop]
    ev = OracleEvaluator([t.copy() for t in pop], o, X, y)
    f0 = ev.loss_only(np.concatenate([np.asarray(c, dtype=np.float64) for c in x0]))
    ds = srhip.Dataset(X, y)
    res = srhip.optimize_constants_batch(ds, pop, o, rng=np.random.default_rng(3),
                                         evaluator_factory=oracle_factory(o, X, y))
    for i, t in enumerate(pop):
        if res.converged[i]:  # the simplex minimum never exceeds its x0 vertex
            assert res.losses[i] <= f0[i] * (1 + 1e-12) or not np.isfinite(f0[i])
        else:
            assert srhip.get_constants(t) == x0[i]
            assert res.losses[i] == f0[i] or not np.isfinite(f0[i])
        assert res.num_evals[i] >= 3 * (len(x0[i]) + 1)


def test_unknown_algorithm_raises():
    o, X, y, trees = problem()
    o.optimizer_algorithm = "LBFGS"
    with pytest.raises(ValueError):
        srhip.optimize_constants_batch(srhip.Dataset(X, y), trees, o,
                                       evaluator_factory=oracle_factory(o, X, y))


@pytest.mark.gpu
@pytest.mark.parametrize("T", [np.float64, np.float32])
def test_engine_nelder_mead(gpu_ctx, T):
    """The batched Nelder-Mead on the engine (loss-only launches: points and
    whole simplices) recovers the known constants like the oracle-driven run."""
    o, X, y, trees = problem(T)
    _, _, _, trees_ref = problem(T)
    for oo in (o,):
        oo.optimizer_algorithm = "NelderMead"
        oo.optimizer_iterations = 600
    ds = srhip.Dataset(X, y)
    res = srhip.optimize_constants_batch(ds, trees, o, rng=np.random.default_rng(0))
    ref = srhip.optimize_constants_batch(ds, trees_ref, o, rng=np.random.default_rng(0),
                                         evaluator_factory=oracle_factory(o, X, y))
    atol = 1e-3 if T == np.float64 else 5e-3
    assert res.converged[0] and ref.converged[0]
    assert np.allclose(srhip.get_constants(trees[0]), [2.0, 1.0, -2.0], atol=atol)
    assert np.allclose(srhip.get_constants(trees[0]), srhip.get_constants(trees_ref[0]), atol=2 * atol)
    assert res.losses[0] < (1e-6 if T == np.float64 else 1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("T", [np.float64, np.float32])
def test_engine_optimizer_matches_oracle_driver(gpu_ctx, T):
    o, X, y, trees = problem(T)
    _, _, _, trees_ref = problem(T)
    ds = srhip.Dataset(X, y)
    res = srhip.optimize_constants_batch(ds, trees, o, rng=np.random.default_rng(0))
    ref = srhip.optimize_constants_batch(ds, trees_ref, o, rng=np.random.default_rng(0),
                                         evaluator_factory=oracle_factory(o, X, y))
    atol = 1e-6 if T == np.float64 else 2e-3
    assert res.converged[1] and ref.converged[1]
    for t, r in zip(trees, trees_ref):
        assert np.allclose(srhip.get_constants(t), srhip.get_constants(r), atol=atol)
    assert np.allclose(srhip.get_constants(trees[0]), [2.0, 1.0, -2.0], atol=atol)
    assert res.losses[0] < (1e-10 if T == np.float64 else 1e-5)


@pytest.mark.gpu
def test_engine_optimizer_random_population(gpu_ctx):
    """Random config-#2-style population: the optimiser never makes a loss
    worse, and converged trees' losses are the engine's own eval_loss."""
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(256, o, 5, np.float32, seed=3)
    rng = np.random.default_rng(2)
    X = rng.standard_normal((5, 4000)).astype(np.float32)
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
    ds = srhip.Dataset(X, y)
    before = srhip.eval_loss_batch(trees, ds, o)
    res = srhip.optimize_constants_batch(ds, trees, o, rng=np.random.default_rng(0))
    after = srhip.eval_loss_batch(trees, ds, o)
    assert np.array_equal(np.isfinite(after), np.isfinite(res.losses))
    m = np.isfinite(before)
    assert np.all(after[m] <= before[m] * (1 + 1e-4) + 1e-9)
    assert res.converged.any()



class _env:
    """Environment variables set for a block (knobs read when a program is built)."""

    def __init__(self, **kw):
        self.kw, self.old = kw, {}

    def __enter__(self):
        import os
        for k, v in self.kw.items():
            self.old[k] = os.environ.get(k)
            os.environ[k] = v

    def __exit__(self, *a):
        import os
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.gpu
def test_set_constants_static_failure_in_place(gpu_ctx):
    """A constant set that makes some trees fail statically (a non-finite
    constant) keeps the program layout: the update is in place (no rebuild of
    the tree code), those trees fail, every other tree equals a fresh
    program's result; restoring finite constants is in place too."""
    from srhip import constants as K

    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(700, o, 5, np.float32, seed=13)
    rng = np.random.default_rng(14)
    X = rng.standard_normal((5, 5001)).astype(np.float32)
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
    ds = srhip.DeviceDataset(gpu_ctx, X, y)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    c0 = np.asarray(flat.consts, dtype=np.float32)
    with _env(SRHIP_JIT="1", SRHIP_JIT_MEMC="1"):
        prog = srhip.Program(gpu_ctx, flat, np.float32)
    assert prog.jit_info()["ntrees"] > 500
    # one constant of every 7th tree with constants becomes Inf
    c1 = c0 * np.float32(1.01)
    hit = [t for t in range(len(trees)) if flat.const_off[t + 1] > flat.const_off[t]][::7]
    for t in hit:
        c1[flat.const_off[t]] = np.inf
    for k, c in enumerate((c1, c0 * np.float32(0.99))):
        prog.set_constants(c)
        with _env(SRHIP_JIT_GCOLS="0"):  # memory-constant code has no shared-subtree columns
            fresh = srhip.Program(gpu_ctx, srhip.FlatTrees(flat.node_off, flat.kind, flat.arg, flat.const_off, c,
                                                           flat.nodes), np.float32)
        s1, _, ok1 = prog.eval_loss(ds, K.LOSS["L2"])
        s2, _, ok2 = fresh.eval_loss(ds, K.LOSS["L2"])
        assert np.array_equal(ok1, ok2)
        np.testing.assert_array_equal(s1[ok1], s2[ok2])
        if k == 0:
            assert not ok1[hit].any()  # an Inf constant fails its tree
    st = prog.update_stats()
    assert st["rebuilt"] == 0 and st["inplace"] == 2, st


@pytest.mark.gpu
@pytest.mark.parametrize("T,n", [(np.float32, 600), (np.float64, 200)])
def test_set_constants_in_place(gpu_ctx, T, n):
    """srhip_program_set_constants overwrites the device programs' immediates
    in place (same folding / static verdicts) and the losses, gradients and
    did_succeed equal those of a program built from the new constants. A
    tree-code program (600 Float32 trees, SRHIP_JIT=1) is rebuilt once, as
    memory-constant tree code that reads its constants from the updated
    programs (bit for bit the literal tree code of a fresh program); a
    program built that way from the start (SRHIP_JIT_MEMC=1) is never
    rebuilt."""
    import os
    from srhip import constants as K

    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(n, o, 5, T, seed=11)
    rng = np.random.default_rng(12)
    X = rng.standard_normal((5, 3001)).astype(T)
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(T)
    ctx = gpu_ctx
    ds = srhip.DeviceDataset(ctx, X, y)
    flat = srhip.flatten(trees, o, dtype=T)
    old = os.environ.get("SRHIP_JIT")
    os.environ["SRHIP_JIT"] = "1"
    try:
        for memc_env in ("0", "1"):
            if memc_env == "1" and T != np.float32:
                continue
            with _env(SRHIP_JIT_MEMC=memc_env):
                prog = srhip.Program(ctx, flat, T)
            jit0 = prog.jit_info()["ntrees"]
            prog.eval_loss_grad(ds, K.LOSS["L2"])  # gradient programs built
            c0 = np.asarray(flat.consts, dtype=T)
            for k in range(3):
                c = (c0 * T(1 + 0.01 * (k + 1)) + T(0.001 * k)).astype(T)
                prog.set_constants(c)
                fresh_flat = srhip.FlatTrees(flat.node_off, flat.kind, flat.arg, flat.const_off, c, flat.nodes)
                # tree code with the constants compiled in (Float64: a program
                # with new constants runs interpreted, jit64.cpp literals, so the
                # fresh one is interpreted too: the same summation order)
                # (no shared-subtree columns: memory-constant code has none, and
                # their PRECISE values differ from FAST tree code in the last bits)
                with _env(SRHIP_JIT="1" if T == np.float32 else "0", SRHIP_JIT_GCOLS="0"):
                    fresh = srhip.Program(ctx, fresh_flat, T)
                s1, w1, ok1 = prog.eval_loss(ds, K.LOSS["L2"])
                s2, w2, ok2 = fresh.eval_loss(ds, K.LOSS["L2"])
                assert np.array_equal(ok1, ok2)
                np.testing.assert_array_equal(s1[ok1], s2[ok2])
                g1 = prog.eval_loss_grad(ds, K.LOSS["L2"])
                g2 = fresh.eval_loss_grad(ds, K.LOSS["L2"])
                for a, b in zip(g1, g2):
                    np.testing.assert_array_equal(np.asarray(a), np.asarray(b))
            st = prog.update_stats()
            if T == np.float64:  # Float64 tree code: rebuilt once, interpreted from then on
                assert prog.jit_info()["ntrees"] == 0
                assert st["rebuilt"] == (1 if jit0 else 0) and st["inplace"] == (2 if jit0 else 3)
                continue
            assert prog.jit_info()["ntrees"] == jit0  # still tree code
            if jit0 and memc_env == "0":
                assert st["rebuilt"] == 1 and st["inplace"] == 2
            else:
                assert st["rebuilt"] == 0 and st["inplace"] == 3
    finally:
        if old is None:
            os.environ.pop("SRHIP_JIT", None)
        else:
            os.environ["SRHIP_JIT"] = old


def test_vectorised_backtrack_step_matches_scalar():
    """_backtrack_steps (all candidates at once) equals _backtrack_step (the
    LineSearches BackTracking order-3 interpolation) element by element."""
    from constopt_reference import _backtrack_step, _backtrack_steps

    rng = np.random.default_rng(4)
    n = 2000
    a1 = rng.uniform(0.01, 1, n)
    a2 = a1 * rng.uniform(0.1, 0.9, n)
    phi0 = rng.standard_normal(n)
    dphi0 = -np.abs(rng.standard_normal(n))
    phix0 = phi0 + np.abs(rng.standard_normal(n))
    phix1 = phi0 + rng.standard_normal(n)
    phix1[::17] = np.inf
    phix1[::29] = phi0[::29] + dphi0[::29] * a2[::29]  # den == 0 on the first shrink
    first = rng.random(n) < 0.5
    vec = _backtrack_steps(a1, a2, phi0, dphi0, phix0, phix1, first)
    with np.errstate(all="ignore"):
        ref = np.array([_backtrack_step(a1[k], a2[k], phi0[k], dphi0[k], phix0[k], phix1[k], first[k])
                        for k in range(n)])
    np.testing.assert_allclose(vec, ref, rtol=1e-14)  # a1**3 on arrays may round differently by an ulp


def test_flat_take_matches_flatten():
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(60, o, 4, np.float32, seed=2)
    flat = srhip.flatten(trees, o, dtype=np.float32)
    idx = [5, 5, 0, 59, 17, 5]
    got = flat.take(idx)
    ref = srhip.flatten([trees[i] for i in idx], o, dtype=np.float32)
    for k in ("node_off", "kind", "arg", "const_off", "consts", "nodes"):
        np.testing.assert_array_equal(getattr(got, k), getattr(ref, k))
    c = np.arange(ref.const_off[-1], dtype=np.float32)
    np.testing.assert_array_equal(flat.take(idx, c).consts, c)


def test_nelder_mead_minimiser_follows_julia_findmin():
    """Optim's after_while! takes findmin of the simplex losses: a NaN vertex is
    the minimum (findmin propagates NaN), and `f_centroid < NaN` is false, so
    that vertex is the result."""
    from constopt_reference import julia_findmin
    assert julia_findmin([3.0, 1.0, 2.0]) == 1
    assert julia_findmin([3.0, np.nan, 1.0, np.nan]) == 1
    assert julia_findmin([1.0, 1.0]) == 0
    assert not (0.5 < np.nan)  # the centroid never replaces a NaN minimum
