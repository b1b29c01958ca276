"""Lockstep search driver, `fast_cycle=true` variant (srhip.search): the
callers of the hot path batched across islands (SURVEY.md §8(f) rank 1;
RegularizedEvolution.jl fast_cycle, SingleIteration.jl, SymbolicRegression.jl
migration). The default path (fast_cycle=false) is tests/test_evolution.py.

CPU tests run the driver over the oracle (scorer / evaluator_factory
injection); the GPU test runs it on the engine with the README quickstart
(config #1) and checks the hall of fame against the engine's own eval_loss."""
import numpy as np
import pytest

import oracle
import srhip
from srhip.search import mutate
from test_constant_optimization import OracleEvaluator


def quickstart(n=100, T=np.float32, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((5, n)).astype(T)
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(T)
    o = srhip.Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp"], npopulations=4,
                      ncycles_per_iteration=40, fast_cycle=True, crossover_probability=0.0,
                      tournament_selection_p=1.0)
    return X, y, o


def oracle_scorer(o, X, y):
    def score(trees):
        flat = srhip.flatten(trees, o, dtype=X.dtype)
        _, losses, ok = oracle.eval_loss_batch(flat, X, y, dtype=X.dtype)
        return np.where(ok, losses.astype(np.float64), np.inf)
    return score


def test_mutations_keep_trees_valid():
    X, y, o = quickstart()
    rng = np.random.default_rng(3)
    trees = srhip.random_population(50, o, 5, np.float32, seed=4)
    for name in ("mutate_constant", "mutate_operator", "add_node", "insert_node", "delete_node", "randomize",
                 "do_nothing"):
        for t in trees:
            before = srhip.string_tree(t, o)
            m = mutate(t, name, o, 5, np.float32, 1.0, 20, rng)
            assert srhip.string_tree(t, o) == before  # the parent is never modified
            srhip.flatten([m], o)  # structurally valid
            if name == "add_node":
                assert srhip.count_nodes(m) > srhip.count_nodes(t)
            if name == "mutate_operator":
                assert srhip.count_nodes(m) == srhip.count_nodes(t)


def test_search_on_oracle_improves_and_hof_is_consistent():
    X, y, o = quickstart()
    score = oracle_scorer(o, X, y)
    hof, stats = srhip.equation_search(X, y, o, niterations=3, seed=1, scorer=score,
                                       evaluator_factory=lambda c: OracleEvaluator(c, o, X, y))
    front = hof.dominating()
    assert front and stats["launches"] >= 3 * 40
    baseline = score([srhip.Node(val=float(np.mean(y)))])[0]
    assert min(m.loss for m in front) < 0.75 * baseline
    # stored losses are the evaluator's losses of the stored trees
    losses = score([m.tree for m in front])
    np.testing.assert_allclose(losses, [m.loss for m in front], rtol=1e-5)
    assert all(srhip.compute_complexity(m.tree, o) <= o.maxsize for m in front)
    assert srhip.print_hall_of_fame(hof, o)


def test_options_search_parameters_and_unknown_keywords():
    o = srhip.Options(npop=100, ncycles_per_iteration=100, annealing=True, alpha=0.5, tournament_selection_n=7)
    assert (o.npop, o.ncycles_per_iteration, o.annealing, o.alpha, o.tournament_selection_n) == (100, 100, True,
                                                                                                 0.5, 7)
    d = srhip.Options()  # the reference defaults (src/Options.jl:315-370)
    assert (d.npop, d.ncycles_per_iteration, d.topn, d.fraction_replaced_hof) == (33, 550, 12, 0.035)
    with pytest.raises(TypeError):
        srhip.Options(not_an_option=1)  # Options.jl:389: error("Unknown keyword argument")
    with pytest.warns(UserWarning):
        w = srhip.Options(output_file="hof.csv")  # control-plane keyword: kept, ignored
    assert w.ignored == {"output_file": "hof.csv"}
    assert srhip.Options(crossover_probability=0.1).crossover_probability == 0.1  # a search option now


def test_annealing_acceptance_uses_ieee_semantics():
    from srhip.search import _acceptance
    o = srhip.Options(annealing=True, alpha=0.1)
    assert _acceptance(1.0, 2.0, 0.0, o) == np.inf      # improvement at T = 0: exp(+Inf)
    assert _acceptance(2.0, 1.0, 0.0, o) == 0.0         # worse at T = 0: exp(-Inf)
    assert _acceptance(-100.0, 0.0, 1.0, o) == np.inf   # exponent 1000 overflows to Inf, no exception
    nan = _acceptance(np.inf, np.inf, 1.0, o)
    assert np.isnan(nan) and not (nan < 0.5)  # `NaN < rand()` is false in Julia: the baby is KEPT (Mutate.jl:247)
    assert _acceptance(1.0, 2.0, 1.0, srhip.Options()) == 1.0


def test_search_with_annealing_and_batching_on_oracle():
    X, y, o = quickstart()
    o.annealing = True
    o.batching, o.batch_size = True, 30
    score = oracle_scorer(o, X, y)

    sizes = []

    def batch_score(trees, idx):
        sizes.append(len(idx))
        return oracle_scorer(o, X[:, idx], y[idx])(trees)

    hof, stats = srhip.equation_search(X, y, o, niterations=2, seed=2, scorer=score, batch_scorer=batch_score,
                                       evaluator_factory=lambda c: OracleEvaluator(c, o, X, y))
    front = hof.dominating()
    assert front
    # every cycle: one minibatch launch re-scoring the parents (Mutate.jl:41-47)
    # and one for the babies, each with batch_size rows
    assert len(sizes) >= 2 * (2 * 40 - 2) and set(sizes) == {30}
    # num_evals counts both minibatch evaluations per next_generation (Mutate.jl:44,200)
    assert stats["evals"] > 0


@pytest.mark.gpu
def test_search_on_engine(gpu_ctx):
    X, y, o = quickstart()
    hof, stats = srhip.equation_search(X, y, o, niterations=3, seed=1)
    front = hof.dominating()
    ds = srhip.Dataset(X, y)
    got = srhip.eval_loss_batch([m.tree for m in front], ds, o)
    np.testing.assert_allclose(got, [m.loss for m in front], rtol=1e-6)
    ref = oracle_scorer(o, X, y)([m.tree for m in front])
    np.testing.assert_allclose(got, ref, rtol=1e-5)
    assert min(m.loss for m in front) < 0.75 * float(np.var(y))  # Inf-loss babies are accepted (Mutate.jl:207)


def _island_worker(rank, world, port, q):
    import os
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root / "symbolicregression.jl_amd"), str(root / "oracle"), str(root / "tests")]
    import torch.distributed as dist

    import srhip as S
    from test_constant_optimization import OracleEvaluator as OE
    from test_search import oracle_scorer as osc, quickstart as qs

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X, y, o = qs()
    o.ncycles_per_iteration = 10
    hof, stats = S.equation_search(X, y, o, niterations=2, seed=5, rank=rank, world=world,
                                   scorer=osc(o, X, y), evaluator_factory=lambda c: OE(c, o, X, y))
    front = hof.dominating()
    q.put((rank, min(m.loss for m in front), stats["evals"]))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_islands_sharded_gloo_world2():
    """npopulations islands split over 2 ranks (no data-path collective); the
    hall of fame is merged on the host every iteration, so both ranks end
    with the same best loss."""
    import torch.multiprocessing as mp
    from test_distributed import free_port

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_island_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert res[0][1] == res[1][1]
    assert res[0][2] > 0 and res[1][2] > 0


def test_options_deprecated_aliases_and_optimizer_options():
    """Deprecated keyword aliases (src/Options.jl:122-143) apply under their new
    names with a DeprecationWarning; optimizer_options' `iterations` overrides
    optimizer_iterations (:606-621); other Optim.Options fields are refused,
    not dropped."""
    import warnings
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        o = srhip.Options(batchSize=77, ncyclesperiteration=9, ns=5, hofMigration=False,
                          optimizer_options={"iterations": 3})
    assert (o.batch_size, o.ncycles_per_iteration, o.tournament_selection_n, o.optimizer_iterations) == (77, 9, 5, 3)
    assert o.ignored == {} and o.hof_migration is False
    assert sum(issubclass(x.category, DeprecationWarning) for x in w) == 4
    with pytest.raises(srhip.Unsupported):
        srhip.Options(optimizer_options={"g_abstol": 1e-3})
    with pytest.raises(TypeError):
        srhip.Options(notAnOption=1)
