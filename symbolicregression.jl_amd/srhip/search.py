"""Lockstep search driver: the hot path's callers batched.

`equation_search` dispatches: default Options (`fast_cycle=false`) run the
reference's regularized evolution in srhip.evolution; this module keeps the
`fast_cycle=true` variant described below.

The reference scores one candidate at a time: `next_generation`
(src/Mutate.jl:41-205) calls `score_func` per mutated tree, inside
`reg_evol_cycle` (src/RegularizedEvolution.jl:13-155), inside `s_r_cycle`
(src/SingleIteration.jl:16-58), per island. This module keeps that algorithm
and moves the batch point up: in every cycle the babies of ALL islands (the
`fast_cycle` variant, RegularizedEvolution.jl:33-79: one baby per
`tournament_selection_n`-member subsample) are scored by one engine launch,
as are population initialisation (Population.jl:31-46), `finalize_scores`
(:134-148) and constant optimisation (`optimize_constants_batch`).

Kept from the reference: MutationWeights defaults (OptionsStruct.jl:41-49),
mutate_constant / mutate_operator / append / prepend / insert / delete /
randomize / do_nothing (MutationFunctions.jl), `check_constraints` on size,
the annealing acceptance rule (Mutate.jl:229-254), replace-oldest, the hall of
fame per complexity, migration from the other islands' best and from the hall
of fame (SymbolicRegression.jl:717-778). Left out (host bookkeeping that does
not change what the engine evaluates): simplify/combine_operators (treated as
do_nothing), crossover (fast_cycle forbids it, :41), `use_frequency`
adaptive parsimony, the recorder, progress output, early stopping. One
deviation: with `batching=true` the babies of one launch share one minibatch
row sample, and the parents' re-scores (Mutate.jl:41-47) another (the
reference draws one per `score_func_batch` call).

Islands are independent between migrations, so with `world > 1` each rank
runs its own islands (no data-path collective) and the best members are
exchanged on the host with `all_gather_object` once per iteration.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence

import numpy as np

from .constant_optimization import optimize_constants_batch
from .dataset import Dataset
from .interface import compute_complexity, eval_loss_batch, loss_to_score, update_baseline_loss_
from .node import Node, _postorder, string_tree
from .options import Options
from .trees import gen_random_tree

MUTATION_WEIGHTS = dict(mutate_constant=0.048, mutate_operator=0.47, add_node=0.79, insert_node=5.1,
                        delete_node=1.7, simplify=0.0020, randomize=0.00023, do_nothing=0.21, optimize=0.0)
SEARCH_DEFAULTS = dict(npop=33, ncycles_per_iteration=550, tournament_selection_n=12, topn=12, alpha=0.1,
                       perturbation_factor=0.076, annealing=False, probability_negate_constant=0.01,
                       fraction_replaced=0.00036, fraction_replaced_hof=0.035, maxdepth=None)


@dataclass
class PopMember:
    tree: Node
    score: float
    loss: float
    birth: int


@dataclass
class HallOfFame:
    """Best member per complexity 1..maxsize (HallOfFame.jl)."""
    members: dict = field(default_factory=dict)

    def update(self, m: PopMember, options: Options) -> None:
        c = compute_complexity(m.tree, options)
        if 0 < c <= options.maxsize and np.isfinite(m.loss):
            cur = self.members.get(c)
            if cur is None or m.loss < cur.loss:
                self.members[c] = PopMember(m.tree.copy(), m.score, m.loss, m.birth)

    def dominating(self) -> List[PopMember]:
        """Pareto front: members better than every simpler one."""
        out, best = [], math.inf
        for c in sorted(self.members):
            m = self.members[c]
            if m.loss < best:
                out.append(m)
                best = m.loss
        return out


def _opt(options: Options, name: str):
    return getattr(options, name, SEARCH_DEFAULTS[name])


def _acceptance(after: float, before: float, temperature: float, options: Options) -> float:
    """probChange of next_generation (src/Mutate.jl:229-233) with Julia's IEEE
    semantics: exp(-delta / (T * alpha)) where T = 0 on the last annealing cycle
    gives exp(±Inf) (0 or Inf) and an overflowing exponent gives Inf, not an
    exception. A NaN (Inf - Inf, or 0/0 at T = 0) makes `probChange < rand()`
    false, so the reference keeps such a baby; the caller compares the same way."""
    if not _opt(options, "annealing"):
        return 1.0
    with np.errstate(all="ignore"):
        delta = np.float64(after) - np.float64(before)
        return float(np.exp(-delta / (np.float64(temperature) * np.float64(_opt(options, "alpha")))))


def _depth(t: Node) -> int:
    if t.degree == 0:
        return 1
    return 1 + max(_depth(t.l), _depth(t.r) if t.degree == 2 else 0)


def mutate(tree: Node, choice: str, options: Options, nfeat: int, T, temperature: float, curmaxsize: int,
           rng: np.random.Generator) -> Node:
    """One mutation of a copy of `tree` (MutationFunctions.jl), by the same
    functions as the default path (srhip.evolution; one implementation of the
    mutation rules for both search variants)."""
    from . import evolution as E

    t = E.copy_node(tree)
    if choice == "mutate_constant":
        return E.mutate_constant(t, temperature, options, T, rng)
    if choice == "mutate_operator":
        return E.mutate_operator(t, options, rng)
    if choice == "add_node":  # Mutate.jl: append or prepend with equal probability
        if rng.random() < 0.5:
            return E.append_random_op(t, options, nfeat, T, rng)
        return E.prepend_random_op(t, options, nfeat, T, rng)
    if choice == "insert_node":
        return E.insert_random_op(t, options, nfeat, T, rng)
    if choice == "delete_node":
        return E.delete_random_op(t, options, nfeat, T, rng)
    if choice == "randomize":
        return E.gen_random_tree_fixed_size(int(rng.integers(1, curmaxsize + 1)), options, nfeat, T, rng)
    return t  # do_nothing / simplify


class _CallbackEvaluator:
    """srhip.evolution's evaluator over the test hooks of equation_search."""

    def __init__(self, dataset, options, scorer, batch_scorer, evaluator_factory):
        self.dataset, self.options = dataset, options
        self.scorer, self.batch_scorer, self.factory = scorer, batch_scorer, evaluator_factory

    def losses(self, trees):
        return np.asarray(self.scorer(trees), dtype=np.float64)

    def losses_rows(self, trees, rows):
        # a NaN loss is a failed evaluation (score 0, loss Inf: batch_score_of);
        # a completed Inf loss keeps its Inf score, as score_func_batch's
        out = np.asarray([self.batch_scorer([t], r)[0] for t, r in zip(trees, rows)], dtype=np.float64)
        return out, ~np.isnan(out)

    def optimize(self, trees, noise):
        return optimize_constants_batch(self.dataset, trees, self.options, noise=noise,
                                        evaluator_factory=self.factory)


def equation_search(X: np.ndarray, y: np.ndarray, options: Options, niterations: int = 10,
                    weights: Optional[np.ndarray] = None, seed: int = 0, rank: int = 0, world: int = 1,
                    group=None, scorer: Optional[Callable[[Sequence[Node]], np.ndarray]] = None,
                    evaluator_factory: Optional[Callable] = None, verbose: bool = False,
                    batch_scorer: Optional[Callable[[Sequence[Node], np.ndarray], np.ndarray]] = None,
                    evaluator=None, lockstep: bool = True):
    """EquationSearch(X, y; niterations, options). Returns (hall_of_fame, stats).

    Default Options run the reference's regularized evolution
    (`fast_cycle=false`: srhip.evolution, every island's candidates scored in
    one launch); `options.fast_cycle=True` runs the fast_cycle variant below.
    `evaluator` (losses / losses_rows / optimize), or the older hooks
    `scorer(trees) -> losses`, `batch_scorer(trees, row_idx) -> losses` and
    `evaluator_factory`, replace the engine (tests run the search over the CPU
    oracle). `lockstep=False` answers every request alone, island after
    island (the reference's one-tree-per-call schedule)."""
    if not getattr(options, "fast_cycle", False):
        from .evolution import EngineEvaluator, equation_search_default

        dataset = Dataset(np.asarray(X), np.asarray(y), weights)
        if evaluator is None and scorer is None:
            evaluator = EngineEvaluator(dataset, options)
        elif evaluator is None:
            evaluator = _CallbackEvaluator(dataset, options, scorer, batch_scorer, evaluator_factory)
        base = Node(val=dataset.avg_y)
        dataset.baseline_loss = dataset.T(np.asarray(evaluator.losses([base]), dtype=np.float64)[0])
        res = equation_search_default(dataset, options, niterations, evaluator, seed=seed, lockstep=lockstep,
                                      rank=rank, world=world, group=group, verbose=verbose)
        res.stats["result"] = res
        return res.hall_of_fame, res.stats
    return _equation_search_fast_cycle(X, y, options, niterations, weights, seed, rank, world, group, scorer,
                                       evaluator_factory, verbose, batch_scorer)


def _equation_search_fast_cycle(X, y, options, niterations, weights, seed, rank, world, group, scorer,
                                evaluator_factory, verbose, batch_scorer):
    """EquationSearch with `fast_cycle=true` (RegularizedEvolution.jl:32-79):
    one baby per `tournament_selection_n`-member subsample, all islands in
    lockstep."""
    # RegularizedEvolution.jl:38-39
    if options.tournament_selection_p != 1.0 or options.crossover_probability != 0.0:
        raise AssertionError("fast_cycle needs tournament_selection_p == 1 and crossover_probability == 0")
    rng = np.random.default_rng(seed + 1000 * rank)
    dataset = Dataset(np.asarray(X), np.asarray(y), weights)
    T = np.dtype(dataset.T).type
    nfeat = dataset.nfeatures
    score_losses = scorer or (lambda trees: eval_loss_batch(trees, dataset, options))
    if scorer is None:
        update_baseline_loss_(dataset, options)
    else:
        dataset.baseline_loss = float(scorer([Node(val=dataset.avg_y)])[0])
    nisl_total = options.npopulations
    islands_here = [i for i in range(nisl_total) if i % world == rank]
    npop = _opt(options, "npop")
    ns = _opt(options, "tournament_selection_n")
    maxsize = options.maxsize
    birth = [0]
    stats = dict(evals=0.0, launches=0, seconds=0.0, iterations=0)

    def born():
        birth[0] += 1
        return birth[0]

    def score(trees: List[Node]):
        stats["launches"] += 1
        stats["evals"] += len(trees)
        losses = np.asarray(score_losses(trees), dtype=np.float64) if trees else np.zeros(0)
        scores = [float(loss_to_score(T(l), dataset.baseline_loss, t, options)) if np.isfinite(l) else math.inf
                  for l, t in zip(losses, trees)]
        return scores, losses

    def score_babies(trees: List[Node]):
        """next_generation's scoring (Mutate.jl:199-205): score_func, or with
        options.batching score_func_batch on batch_size rows sampled with
        replacement (one sample per launch, shared by the launch's babies)."""
        if not options.batching or not trees:
            return score(trees)
        stats["launches"] += 1
        stats["evals"] += len(trees) * options.batch_size / dataset.n
        idx = rng.integers(0, dataset.n, size=options.batch_size)
        if batch_scorer is not None:
            losses = np.asarray(batch_scorer(trees, idx), dtype=np.float64)
        else:
            losses = np.asarray(eval_loss_batch(trees, dataset, options, row_idx=idx), dtype=np.float64)
        # a failed minibatch evaluation scores (0, Inf) (LossFunctions.jl:102-104)
        scores = [float(loss_to_score(T(l), dataset.baseline_loss, t, options)) if np.isfinite(l) else 0.0
                  for l, t in zip(losses, trees)]
        return scores, losses

    t0 = time.perf_counter()
    # Population(dataset; npop): gen_random_tree(3, ...) per member, all islands in one launch
    trees = [gen_random_tree(3, options, nfeat, T, rng) for _ in islands_here for _ in range(npop)]
    sc, lo = score(trees)
    pops = [[PopMember(trees[k * npop + j], sc[k * npop + j], lo[k * npop + j], born()) for j in range(npop)]
            for k in range(len(islands_here))]
    hof = HallOfFame()
    weights_base = dict(MUTATION_WEIGHTS)
    ncycles = _opt(options, "ncycles_per_iteration")
    for it in range(niterations):
        for cyc in range(ncycles):
            temperature = 1.0 - cyc / max(ncycles - 1, 1) if _opt(options, "annealing") else 1.0
            curmaxsize = maxsize
            babies, parents = [], []
            for k, pop in enumerate(pops):
                order = rng.permutation(len(pop))  # shuffle!(pop.members)
                pops[k] = pop = [pop[i] for i in order]
                for i in range(round(len(pop) / ns)):
                    allstar = min(pop[i * ns:(i + 1) * ns], key=lambda m: m.score)
                    w = dict(weights_base)
                    nconst = sum(1 for n in _postorder(allstar.tree) if n.degree == 0 and n.constant)
                    w["mutate_constant"] *= min(8, nconst) / 8.0
                    depth_limit = _opt(options, "maxdepth") or maxsize
                    if compute_complexity(allstar.tree, options) >= curmaxsize or _depth(allstar.tree) >= depth_limit:
                        w["add_node"] = w["insert_node"] = 0.0
                    names = list(w)
                    p = np.asarray([w[n] for n in names])
                    choice = names[rng.choice(len(names), p=p / p.sum())]
                    baby = None
                    for _ in range(10):  # max_attempts (Mutate.jl:87-88)
                        cand = mutate(allstar.tree, choice, options, nfeat, T, temperature, curmaxsize, rng)
                        if compute_complexity(cand, options) <= curmaxsize:
                            baby = cand
                            break
                    parents.append((k, allstar, choice, baby))
                    if baby is not None and choice not in ("do_nothing", "simplify", "optimize"):
                        babies.append(baby)
            # with options.batching every next_generation first re-scores its
            # parent on a fresh minibatch (Mutate.jl:41-47): one launch for all
            # parents of the cycle, on a row sample of its own
            if options.batching and parents:
                psc, plo = score_babies([allstar.tree for _, allstar, _, _ in parents])
            else:
                psc = [allstar.score for _, allstar, _, _ in parents]
                plo = [allstar.loss for _, allstar, _, _ in parents]
            sc, lo = score_babies(babies)  # ONE launch for every island's babies
            b = 0
            for q, (k, allstar, choice, baby) in enumerate(parents):
                before_score, before_loss = psc[q], plo[q]
                if baby is None:
                    continue  # failed mutation: skip_mutation_failures (default true)
                if choice in ("do_nothing", "simplify", "optimize"):
                    new = PopMember(baby, before_score, before_loss, born())
                else:
                    s, l = sc[b], lo[b]
                    b += 1
                    if np.isnan(s):  # Mutate.jl:207: only a NaN score is rejected outright
                        continue
                    prob = _acceptance(s, before_score, temperature, options)
                    if prob < rng.random():  # Mutate.jl:247 `probChange < rand()`: a NaN prob is kept
                        continue
                    new = PopMember(baby, s, l, born())
                pop = pops[k]
                oldest = min(range(len(pop)), key=lambda j: pop[j].birth)
                pop[oldest] = new
        # optimize_and_simplify_population: constants of a random subset, batched
        if getattr(options, "should_optimize_constants", True) and options.optimizer_probability > 0:
            sel = [(k, j) for k, pop in enumerate(pops) for j in range(len(pop))
                   if rng.random() < options.optimizer_probability]
            if sel:
                trees = [pops[k][j].tree for k, j in sel]
                res = optimize_constants_batch(dataset, trees, options, rng=rng,
                                               evaluator_factory=evaluator_factory)
                stats["evals"] += float(res.num_evals.sum())
                for (k, j), l, ok in zip(sel, res.losses, res.converged):
                    if ok:
                        m = pops[k][j]
                        m.loss = float(l)
                        m.score = float(loss_to_score(T(l), dataset.baseline_loss, m.tree, options))
                        m.birth = born()
        for pop in pops:
            for m in pop:
                hof.update(m, options)
        # migration (SymbolicRegression.jl:717-778): other islands' best and the hall of fame
        topn = _opt(options, "topn")
        best = [m for pop in pops for m in sorted(pop, key=lambda m: m.score)[:topn]]
        if world > 1:
            import torch.distributed as dist

            gathered = [None] * world
            dist.all_gather_object(gathered, [(m.tree, m.score, m.loss) for m in best], group=group)
            best = [PopMember(t, s, l, 0) for part in gathered for (t, s, l) in part]
            hofs = [None] * world
            dist.all_gather_object(hofs, [(m.tree, m.score, m.loss) for m in hof.members.values()], group=group)
            for part in hofs:
                for (t, s, l) in part:
                    hof.update(PopMember(t, s, l, 0), options)
        front = hof.dominating()
        for pop in pops:
            for frac, source in ((_opt(options, "fraction_replaced"), best),
                                 (_opt(options, "fraction_replaced_hof"), front)):
                if not source:
                    continue
                for j in range(len(pop)):
                    if rng.random() < frac:
                        m = source[rng.integers(len(source))]
                        pop[j] = PopMember(m.tree.copy(), m.score, m.loss, born())
        stats["iterations"] += 1
        if verbose and rank == 0:
            print(f"iteration {it + 1}: best loss {min(m.loss for m in front) if front else math.inf:.4g}")
    stats["seconds"] = time.perf_counter() - t0
    stats["evals_per_s"] = stats["evals"] / max(stats["seconds"], 1e-12)
    stats["seconds_per_iteration"] = stats["seconds"] / max(niterations, 1)
    return hof, stats


def print_hall_of_fame(hof: HallOfFame, options: Options) -> List[str]:
    return [f"{compute_complexity(m.tree, options)}\t{m.loss:.6g}\t{string_tree(m.tree, options)}"
            for m in hof.dominating()]
