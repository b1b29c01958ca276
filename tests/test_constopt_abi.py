"""The C++ lockstep constant optimiser (csrc/constopt.cpp behind
srhip_optimize_constants_cb) against its checker, tests/constopt_reference.py
(the Python restatement): same oracle evaluator, same start noise, identical
trajectories — constants, losses, convergence flags and evaluation counts bit
for bit — for BFGS / Newton and Nelder-Mead, Float32 and Float64 trees.
CPU only: the callback entry uses no device.

Reference: optimize_constants, src/ConstantOptimization.jl:22-65."""
import numpy as np
import pytest

import constopt_reference as ref
import srhip
from srhip.constant_optimization import start_noise
from test_constant_optimization import oracle_factory, problem


def _population(T, n_trees=24, seed=3):
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((5, 150)).astype(T)
    y = (T(2) * np.cos(X[3]) + X[0] * X[0] - T(2)).astype(T)
    trees = srhip.random_population(n_trees, o, 5, T, seed=seed + 1, maxsize=16)
    return o, X, y, trees


def _run_both(o, X, y, trees, T, seed):
    ds = srhip.Dataset(X, y)
    fac = oracle_factory(o, X, y)
    t_cpp = [t.copy() for t in trees]
    t_ref = [t.copy() for t in trees]
    r_cpp = srhip.optimize_constants_batch(ds, t_cpp, o, rng=np.random.default_rng(seed), evaluator_factory=fac)
    flat = srhip.flatten(trees, o, dtype=T)
    noise = start_noise(flat, int(o.optimizer_nrestarts), np.random.default_rng(seed))
    r_ref = ref.optimize_constants_batch(ds, t_ref, o, noise, fac)
    return r_cpp, r_ref, t_cpp, t_ref


def _assert_identical(r_cpp, r_ref, t_cpp, t_ref):
    np.testing.assert_array_equal(r_cpp.converged, r_ref.converged)
    np.testing.assert_array_equal(r_cpp.num_evals, r_ref.num_evals)
    np.testing.assert_array_equal(r_cpp.losses, r_ref.losses)
    for a, b in zip(t_cpp, t_ref):
        ca, cb = srhip.get_constants(a), srhip.get_constants(b)
        assert [float(v) for v in ca] == [float(v) for v in cb]


@pytest.mark.parametrize("T", [np.float64, np.float32])
@pytest.mark.parametrize("algorithm", ["BFGS", "NelderMead"])
def test_cpp_driver_matches_reference_on_random_population(T, algorithm):
    o, X, y, trees = _population(T)
    o.optimizer_algorithm = algorithm
    r_cpp, r_ref, t_cpp, t_ref = _run_both(o, X, y, trees, T, seed=11)
    _assert_identical(r_cpp, r_ref, t_cpp, t_ref)
    assert r_cpp.converged.any() and r_cpp.num_evals.max() > 10


@pytest.mark.parametrize("algorithm", ["BFGS", "NelderMead"])
def test_cpp_driver_matches_reference_on_known_answer_problem(algorithm):
    o, X, y, trees = problem()
    o.optimizer_algorithm = algorithm
    r_cpp, r_ref, t_cpp, t_ref = _run_both(o, X, y, trees, np.float64, seed=0)
    _assert_identical(r_cpp, r_ref, t_cpp, t_ref)


def test_more_iterations_and_restarts():
    o, X, y, trees = _population(np.float64, n_trees=12, seed=8)
    o.optimizer_iterations = 20
    o.optimizer_nrestarts = 4
    r_cpp, r_ref, t_cpp, t_ref = _run_both(o, X, y, trees, np.float64, seed=2)
    _assert_identical(r_cpp, r_ref, t_cpp, t_ref)


def test_evaluator_errors_propagate():
    o, X, y, trees = problem()

    class Boom:
        def __init__(self, cands):
            pass

        def loss_grad(self, consts):
            raise RuntimeError("boom")

        def loss_only(self, consts):
            raise RuntimeError("boom")

    with pytest.raises(RuntimeError, match="boom"):
        srhip.optimize_constants_batch(srhip.Dataset(X, y), trees, o, rng=np.random.default_rng(0),
                                       evaluator_factory=Boom)


def test_unknown_algorithm_is_rejected():
    o, X, y, trees = problem()
    o.optimizer_algorithm = "Foo"
    with pytest.raises(ValueError):
        srhip.optimize_constants_batch(srhip.Dataset(X, y), trees, o, rng=np.random.default_rng(0),
                                       evaluator_factory=oracle_factory(o, X, y))
