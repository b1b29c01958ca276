"""Regularized evolution with the reference's DEFAULT Options, every island's
candidates scored in one engine launch.

The reference's default search (`fast_cycle=false`, src/Options.jl:331;
`crossover_probability=0.066`, :343; `tournament_selection_p=0.86`, :322;
`use_frequency` / `use_frequency_in_tournament`, :345-346) runs, per island
and per cycle, `round(npop / tournament_selection_n)` sequential steps
(src/RegularizedEvolution.jl:81-155): `best_of_sample` (Population.jl:79-119),
then `next_generation` (Mutate.jl:25-282) or, with probability 0.066,
`crossover_generation` (Mutate.jl:285-341), each scoring ONE tree per
`score_func` call, and replace-oldest. Step i+1 sees step i's replacement, so
an island cannot be batched with itself; islands are independent between
two visits of the head node (SymbolicRegression.jl:670-866), so the batch
point is ACROSS islands.

Structure (no change to what any island computes):

* every piece of an island's work — `Population` init (Population.jl:31-46),
  `s_r_cycle` (SingleIteration.jl:17-61) with `reg_evol_cycle`,
  `optimize_and_simplify_population` (SingleIteration.jl:63-127), the
  batching re-score of the island's best-seen members
  (SymbolicRegression.jl:616-625, 817-829) — is a Python generator that
  YIELDS a request (`Score`: full-data losses of some trees; `ScoreRows`:
  minibatch losses, one row sample per tree as `score_func_batch` draws
  it, LossFunctions.jl:95-115; `Optimize`: `optimize_constants` of some
  trees with the start noise the island drew, ConstantOptimization.jl:22-65)
  and receives the answer;
* each island owns its random stream (a numpy Generator per island id) and
  its birth counter, so its trajectory depends on nothing but its own draws
  and the answers;
* `run_lockstep` advances every island to its next request, answers ALL
  pending requests with one evaluator call per kind (one engine launch for
  the scores of every island), and resumes them; `run_serial` runs the
  islands one after the other and answers each request alone, one tree per
  call, as the reference does. Both give the same result bit for bit
  (tests/test_evolution.py, over the oracle);
* the head node (hall of fame, adaptive-parsimony frequencies, migration,
  `warmup_maxsize_by`) is the reference's, with the semantics of its
  multiprocessing mode: an island's cycle runs on a snapshot of the
  frequencies normalised when it is spawned, and the head takes the islands
  in the fixed shuffled order `all_idx` (SymbolicRegression.jl:661-676). A
  round spawns and completes every island once; `niterations` rounds
  complete `npopulations × niterations` island cycles, the reference's
  `total_cycles` (:634). The reference's last round spawns cycles whose
  results it never reads; they are not run here.

Host routines restated for it: the MutationFunctions.jl mutations, crossover
and random trees; CheckConstraints.jl (including its `0 > size > maxsize`
size test, which is always false, so size is not enforced: SURVEY.md a10);
AdaptiveParsimony.jl; HallOfFame.jl; Migration.jl; and DynamicExpressions
0.4.x `simplify_tree` / `combine_operators` (not vendored in the reference:
restated from the published package, parity unpinned), whose operator
arithmetic is the engine's own host folding (`srhip_op_eval`). Julia's RNG
streams cannot be reproduced; the distributions are the reference's.

With `world > 1` (torch.distributed) each rank runs the islands
`i % world == rank` and, once per round, every rank receives every island's
result (`all_gather_object`) and runs the same head-node code with the same
head stream, so a sharded search gives exactly the single-process result.
"""
from __future__ import annotations

import bisect
import ctypes as C
import itertools
import math
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, Iterator, List, Optional, Sequence

import numpy as np

from . import constants as K
from .node import Node

MAX_DEGREE = 2  # src/ProgramConstants.jl:3
MUTATIONS = ("mutate_constant", "mutate_operator", "add_node", "insert_node", "delete_node", "simplify",
             "randomize", "do_nothing", "optimize")  # OptionsStruct.jl:8-18 field order
DEFAULT_MUTATION_WEIGHTS = (0.048, 0.47, 0.79, 5.1, 1.7, 0.0020, 0.00023, 0.21, 0.0)  # OptionsStruct.jl:38-48

_new_node = Node.__new__


# ---------------------------------------------------------------- trees (host)
def copy_node(t: Node) -> Node:
    """DynamicExpressions.copy_node (deep copy)."""
    n = _new_node(Node)
    d = t.degree
    n.degree = d
    n.constant = t.constant
    n.val = t.val
    n.feature = t.feature
    n.op = t.op
    if d == 0:
        n.l = None
        n.r = None
    elif d == 1:
        n.l = copy_node(t.l)
        n.r = None
    else:
        n.l = copy_node(t.l)
        n.r = copy_node(t.r)
    return n


def _leaf_const(val) -> Node:
    n = _new_node(Node)
    n.degree, n.constant, n.val, n.feature, n.op, n.l, n.r = 0, True, val, 0, 0, None, None
    return n


def _leaf_feature(f: int) -> Node:
    n = _new_node(Node)
    n.degree, n.constant, n.val, n.feature, n.op, n.l, n.r = 0, False, 0.0, f, 0, None, None
    return n


def _op_node(op: int, l: Node, r: Optional[Node] = None) -> Node:
    n = _new_node(Node)
    n.degree, n.constant, n.val, n.feature, n.op, n.l, n.r = (1 if r is None else 2), False, 0.0, 0, op, l, r
    return n


def set_node(dst: Node, src: Node) -> None:
    """DynamicExpressions.set_node!"""
    dst.degree, dst.constant, dst.val, dst.feature, dst.op, dst.l, dst.r = (
        src.degree, src.constant, src.val, src.feature, src.op, src.l, src.r)


def nodes_preorder(t: Node) -> List[Node]:
    out, stack = [], [t]
    while stack:
        n = stack.pop()
        out.append(n)
        if n.degree == 2:
            stack.append(n.r)
        if n.degree >= 1:
            stack.append(n.l)
    return out


def count_depth(t: Node) -> int:
    if t.degree == 0:
        return 1
    if t.degree == 1:
        return 1 + count_depth(t.l)
    return 1 + max(count_depth(t.l), count_depth(t.r))


def count_constants(t: Node) -> int:
    return sum(1 for n in nodes_preorder(t) if n.degree == 0 and n.constant)


def _info(t: Node):
    """(node count, depth, constant count) of t."""
    d = t.degree
    if d == 0:
        return 1, 1, 1 if t.constant else 0
    n, h, k = _info(t.l)
    if d == 1:
        return n + 1, h + 1, k
    n2, h2, k2 = _info(t.r)
    return n + n2 + 1, (h if h > h2 else h2) + 1, k + k2


def tree_info(t: Node, options):
    """(compute_complexity, count_depth, count_constants) in one traversal."""
    if options.complexity_use:
        return compute_complexity(t, options), count_depth(t), count_constants(t)
    return _info(t)


def compute_complexity(t: Node, options) -> int:
    """src/Complexity.jl:13-40."""
    if not options.complexity_use:
        return len(nodes_preorder(t))

    def rec(n: Node) -> float:
        if n.degree == 0:
            return options.constant_complexity if n.constant else options.variable_complexity
        if n.degree == 1:
            return options.unaop_complexities[n.op - 1] + rec(n.l)
        return options.binop_complexities[n.op - 1] + rec(n.l) + rec(n.r)

    return int(round(rec(t)))


# ------------------------------------------------------- MutationFunctions.jl
def _rand_int(rng, lo: int, hi: int) -> int:
    """rand(lo:hi): floor(U·n) (one uniform draw, 4x cheaper than Generator.integers)"""
    return lo + int(rng.random() * (hi - lo + 1))


def _rand_index(rng, n: int) -> int:
    return int(rng.random() * n)


def make_random_leaf(nfeatures: int, T, rng) -> Node:
    """:151-157"""
    if rng.random() > 0.5:
        return _leaf_const(T(rng.standard_normal()))
    return _leaf_feature(_rand_int(rng, 1, nfeatures))


def random_node(tree: Node, rng) -> Node:
    """:8-29 (uniform over the nodes)"""
    nodes = nodes_preorder(tree)
    return nodes[_rand_index(rng, len(nodes))]


def mutate_operator(tree: Node, options, rng) -> Node:
    """:33-47"""
    ops = [n for n in nodes_preorder(tree) if n.degree > 0]
    if not ops:
        return tree
    node = ops[_rand_index(rng, len(ops))]
    node.op = _rand_int(rng, 1, options.nuna if node.degree == 1 else options.nbin)
    return tree


def mutate_constant(tree: Node, temperature, options, T, rng) -> Node:
    """:50-79 — including `rand() > probability_negate_constant` negating the
    constant, as the reference is written."""
    consts = [n for n in nodes_preorder(tree) if n.degree == 0 and n.constant]
    if not consts:
        return tree
    node = consts[_rand_index(rng, len(consts))]
    max_change = T(options.perturbation_factor) * T(temperature) + T(1.1)  # T(1 + 1//10)
    u = rng.random(dtype=np.float32) if T == np.float32 else rng.random()
    factor = T(float(max_change) ** float(u))  # T ^ T: the power in Float64, rounded once
    if rng.random() > 0.5:
        node.val = T(T(node.val) * factor)
    else:
        node.val = T(T(node.val) / factor)
    if rng.random() > options.probability_negate_constant:
        node.val = T(-node.val)
    return tree


def _new_op_choice(options, rng) -> bool:
    return rng.random() < options.nbin / (options.nuna + options.nbin)


def append_random_op(tree: Node, options, nfeatures: int, T, rng, make_new_bin_op: Optional[bool] = None) -> Node:
    """:82-111"""
    leaves = [n for n in nodes_preorder(tree) if n.degree == 0]
    node = leaves[_rand_index(rng, len(leaves))]
    if make_new_bin_op is None:
        make_new_bin_op = _new_op_choice(options, rng)
    if make_new_bin_op:
        l = make_random_leaf(nfeatures, T, rng)
        r = make_random_leaf(nfeatures, T, rng)
        new = _op_node(_rand_int(rng, 1, options.nbin), l, r)
    else:
        new = _op_node(_rand_int(rng, 1, options.nuna), make_random_leaf(nfeatures, T, rng))
    set_node(node, new)
    return tree


def insert_random_op(tree: Node, options, nfeatures: int, T, rng) -> Node:
    """:114-130"""
    node = random_node(tree, rng)
    make_bin = _new_op_choice(options, rng)
    left = copy_node(node)
    if make_bin:
        right = make_random_leaf(nfeatures, T, rng)
        new = _op_node(_rand_int(rng, 1, options.nbin), left, right)
    else:
        new = _op_node(_rand_int(rng, 1, options.nuna), left)
    set_node(node, new)
    return tree


def prepend_random_op(tree: Node, options, nfeatures: int, T, rng) -> Node:
    """:133-149"""
    make_bin = _new_op_choice(options, rng)
    left = copy_node(tree)
    if make_bin:
        right = make_random_leaf(nfeatures, T, rng)
        new = _op_node(_rand_int(rng, 1, options.nbin), left, right)
    else:
        new = _op_node(_rand_int(rng, 1, options.nuna), left)
    set_node(tree, new)
    return tree


def random_node_and_parent(tree: Node, rng):
    """:160-189: (node, parent or None, side 'l' / 'r' / 'n'), uniform over nodes."""
    out, stack = [], [(tree, None, "n")]
    while stack:
        n, p, s = stack.pop()
        out.append((n, p, s))
        if n.degree == 2:
            stack.append((n.r, n, "r"))
        if n.degree >= 1:
            stack.append((n.l, n, "l"))
    return out[_rand_index(rng, len(out))]


def delete_random_op(tree: Node, options, nfeatures: int, T, rng) -> Node:
    """:193-233"""
    node, parent, side = random_node_and_parent(tree, rng)
    if node.degree == 0:
        set_node(node, make_random_leaf(nfeatures, T, rng))
        return tree
    keep = node.l if (node.degree == 1 or rng.random() < 0.5) else node.r
    if parent is None:
        return keep
    if side == "l":
        parent.l = keep
    else:
        parent.r = keep
    return tree


def gen_random_tree(length: int, options, nfeatures: int, T, rng) -> Node:
    """:236-246"""
    tree = _leaf_const(T(1))
    for _ in range(length):
        tree = append_random_op(tree, options, nfeatures, T, rng)
    return tree


def gen_random_tree_fixed_size(node_count: int, options, nfeatures: int, T, rng) -> Node:
    """:248-263"""
    tree = make_random_leaf(nfeatures, T, rng)
    cur = 1
    while cur < node_count:
        if cur == node_count - 1:
            if options.nuna == 0:
                break
            tree = append_random_op(tree, options, nfeatures, T, rng, make_new_bin_op=False)
        else:
            tree = append_random_op(tree, options, nfeatures, T, rng)
        cur = len(nodes_preorder(tree))
    return tree


def crossover_trees(tree1: Node, tree2: Node, rng):
    """:266-294"""
    tree1, tree2 = copy_node(tree1), copy_node(tree2)
    node1, parent1, side1 = random_node_and_parent(tree1, rng)
    node2, parent2, side2 = random_node_and_parent(tree2, rng)
    node1 = copy_node(node1)
    if side1 == "l":
        parent1.l = copy_node(node2)
    elif side1 == "r":
        parent1.r = copy_node(node2)
    else:
        tree1 = copy_node(node2)
    if side2 == "l":
        parent2.l = node1
    elif side2 == "r":
        parent2.r = node1
    else:
        tree2 = node1
    return tree1, tree2


# ------------------------------------------------------- CheckConstraints.jl
def _flag_bin(tree: Node, op: int, cons, options) -> bool:
    if tree.degree == 0:
        return False
    if tree.degree == 1:
        return _flag_bin(tree.l, op, cons, options)
    if tree.op == op:
        if (cons[0] > -1 and compute_complexity(tree.l, options) > cons[0]) or (
                cons[1] > -1 and compute_complexity(tree.r, options) > cons[1]):
            return True
    return _flag_bin(tree.l, op, cons, options) or _flag_bin(tree.r, op, cons, options)


def _flag_una(tree: Node, op: int, cons: int, options) -> bool:
    if tree.degree == 0:
        return False
    if tree.degree == 1:
        if tree.op == op and cons > -1 and compute_complexity(tree.l, options) > cons:
            return True
        return _flag_una(tree.l, op, cons, options)
    return _flag_una(tree.l, op, cons, options) or _flag_una(tree.r, op, cons, options)


def _count_max_nestedness(tree: Node, degree: int, op: int) -> int:
    if tree.degree == 0:
        return 0
    if tree.degree == 1:
        return (1 if degree == 1 and tree.op == op else 0) + _count_max_nestedness(tree.l, degree, op)
    return (1 if degree == 2 and tree.op == op else 0) + max(_count_max_nestedness(tree.l, degree, op),
                                                             _count_max_nestedness(tree.r, degree, op))


def _fast_max_nestedness(tree: Node, degree: int, op: int, nd: int, nop: int) -> int:
    if tree.degree == 0:
        return 0
    if tree.degree == 1:
        if degree != 1 or tree.op != op:
            return _fast_max_nestedness(tree.l, degree, op, nd, nop)
        return _count_max_nestedness(tree.l, nd, nop)
    if degree != 2 or tree.op != op:
        return max(_fast_max_nestedness(tree.l, degree, op, nd, nop),
                   _fast_max_nestedness(tree.r, degree, op, nd, nop))
    return max(_count_max_nestedness(tree.l, nd, nop), _count_max_nestedness(tree.r, nd, nop))


def check_constraints(tree: Node, options, maxsize: int) -> bool:
    """src/CheckConstraints.jl:142-166. The size test is `0 > size > maxsize`
    (:144), which Julia reads as `0 > size && size > maxsize` — never true —
    so, exactly as in the reference, size is not enforced here."""
    if not options.has_constraints:
        return True  # the size test below is never true
    size = compute_complexity(tree, options)
    if 0 > size > maxsize:  # the reference's expression, kept as written
        return False
    for i, cons in enumerate(options.bin_constraints, start=1):
        if tuple(cons) != (-1, -1) and _flag_bin(tree, i, cons, options):
            return False
    for i, cons in enumerate(options.una_constraints, start=1):
        if cons != -1 and _flag_una(tree, i, cons, options):
            return False
    for degree, op, nested in options.nested_constraints or ():
        for nd, nop, max_nest in nested:
            if _fast_max_nestedness(tree, degree, op, nd, nop) > max_nest:
                return False
    return True


# --------------------------------------- DynamicExpressions 0.4 simplification
_op_out = C.c_double()


def _op_eval(T, arity: int, engine_id: int, a, b=0.0):
    from ._lib import check, lib

    check(lib().srhip_op_eval(0 if T == np.float32 else 1, arity, engine_id, float(a), float(b),
                              C.byref(_op_out)))
    return T(_op_out.value)


def _finite(x) -> bool:
    return bool(np.isfinite(x))


def simplify_tree(tree: Node, options, T) -> Node:
    """DynamicExpressions 0.4.x `simplify_tree` (SimplifyEquation.jl; not
    vendored, restated — parity unpinned): an operator whose children are all
    finite constants becomes the (finite) constant it evaluates to."""
    bin_ids, una_ids = options.engine_operator_ids()
    if tree.degree == 1:
        tree.l = simplify_tree(tree.l, options, T)
        if tree.l.degree == 0 and tree.l.constant:
            lv = T(tree.l.val)
            if _finite(lv):
                out = _op_eval(T, 1, una_ids[tree.op - 1], lv)
                if _finite(out):
                    return _leaf_const(out)
    elif tree.degree == 2:
        tree.l = simplify_tree(tree.l, options, T)
        tree.r = simplify_tree(tree.r, options, T)
        if tree.l.degree == 0 and tree.l.constant and tree.r.degree == 0 and tree.r.constant:
            lv, rv = T(tree.l.val), T(tree.r.val)
            if not (_finite(lv) and _finite(rv)):
                return tree
            out = _op_eval(T, 2, bin_ids[tree.op - 1], lv, rv)
            if not _finite(out):
                return tree
            return _leaf_const(out)
    return tree


def _is_const(n: Node) -> bool:
    return n.degree == 0 and n.constant


def combine_operators(tree: Node, options, T) -> Node:
    """DynamicExpressions 0.4.x `combine_operators` (restated, parity
    unpinned): ((c + x) + c') → (x + c+c'), likewise for *, with the constant
    moved to the right; the four (c − x) / (x − c) nestings under −."""
    if tree.degree == 0:
        return tree
    tree.l = combine_operators(tree.l, options, T)
    if tree.degree == 2:
        tree.r = combine_operators(tree.r, options, T)
    if tree.degree != 2:
        return tree
    name = options.binary_operators[tree.op - 1]
    top_level_constant = _is_const(tree.l) or _is_const(tree.r)
    if name in ("*", "+") and top_level_constant:
        op = tree.op
        if _is_const(tree.l):
            tree.l, tree.r = tree.r, tree.l
        top = T(tree.r.val)
        below = tree.l
        if below.degree == 2 and below.op == op:
            f = (lambda a, b: T(a * b)) if name == "*" else (lambda a, b: T(a + b))
            if _is_const(below.l):
                tree = below
                tree.l.val = f(T(tree.l.val), top)
            elif _is_const(below.r):
                tree = below
                tree.r.val = f(T(tree.r.val), top)
    if tree.degree == 2 and options.binary_operators[tree.op - 1] == "-" and (
            _is_const(tree.l) or _is_const(tree.r)):
        l, r = tree.l, tree.r
        if _is_const(l):
            if r.degree == 2 and options.binary_operators[r.op - 1] == "-":
                if _is_const(r.l):
                    # (c − (c' − x)) → (x − (c' − c))... as written: (x − (−(c − c')))
                    simplified = T(-T(T(l.val) - T(r.l.val)))
                    tree.l = r.r
                    tree.r = l
                    tree.r.val = simplified
                elif _is_const(r.r):
                    # (c − (x − c')) → ((c + c') − x)
                    simplified = T(T(l.val) + T(r.r.val))
                    tree.r = r.l
                    tree.l.val = simplified
        else:
            if l.degree == 2 and options.binary_operators[l.op - 1] == "-":
                if _is_const(l.l):
                    # ((c − x) − c') → ((c − c') − x)
                    simplified = T(T(l.l.val) - T(r.val))
                    tree.r = l.r
                    tree.l = r
                    tree.l.val = simplified
                elif _is_const(l.r):
                    # ((x − c) − c') → (x − (c' + c))
                    simplified = T(T(r.val) + T(l.r.val))
                    tree.l = l.l
                    tree.r.val = simplified
    return tree


# ---------------------------------------------------------- AdaptiveParsimony.jl
class RunningSearchStatistics:
    """src/AdaptiveParsimony.jl:20-95."""

    def __init__(self, options, window_size: int = 100000):
        n = options.maxsize + MAX_DEGREE
        self.window_size = window_size
        self.frequencies = np.ones(n, dtype=np.float64)
        self.normalized_frequencies = self.frequencies / self.frequencies.sum()

    def update_frequencies(self, size: int) -> None:
        if 0 < size <= len(self.frequencies):
            self.frequencies[size - 1] += 1

    def move_window(self) -> None:
        f = self.frequencies
        smallest = 1
        cur = f.sum()
        if cur > self.window_size:
            diff = cur - self.window_size
            loops = 0
            while diff > 0:
                idx = np.flatnonzero(f > smallest)
                nrem = idx.size
                amount = min(diff / nrem, f[idx].min() - smallest)
                f[idx] -= amount
                total = amount * nrem
                diff -= total
                loops += 1
                if loops > 1000 or total < 1e-6:
                    break

    def normalize(self) -> None:
        self.normalized_frequencies = self.frequencies / self.frequencies.sum()

    def snapshot(self) -> np.ndarray:
        """normalize_frequencies! on the copy a spawned island works with."""
        return self.frequencies / self.frequencies.sum()


# ------------------------------------------------------------- members / HoF
@dataclass
class PopMember:
    """src/PopMember.jl:9-16. Scores and losses are held as Python floats
    whose values are exactly the reference's T values."""
    tree: Node
    score: float
    loss: float
    birth: int
    ref: int = 0
    parent: int = -1
    info: Optional[tuple] = None  # tree_info of `tree` (None: not computed / tree changed)


def copy_member(m: PopMember) -> PopMember:
    return PopMember(copy_node(m.tree), m.score, m.loss, m.birth, m.ref, m.parent, m.info)


def minfo(m: PopMember, options) -> tuple:
    if m.info is None:
        m.info = tree_info(m.tree, options)
    return m.info


class HallOfFame:
    """src/HallOfFame.jl:10-86: best member per complexity 1..maxsize+2."""

    def __init__(self, options, T):
        n = options.maxsize + MAX_DEGREE
        self.options = options
        self.members = [PopMember(_leaf_const(T(1)), 0.0, math.inf, 0) for _ in range(n)]
        self.exists = [False] * n

    def pareto(self) -> List[PopMember]:
        """calculate_pareto_frontier (:76-110)."""
        out = []
        for size in range(len(self.members)):
            if not self.exists[size]:
                continue
            m = self.members[size]
            if all(not self.exists[i] or not (m.loss >= self.members[i].loss) for i in range(size)):
                out.append(copy_member(m))
        return out

    def dominating(self) -> List[PopMember]:
        return self.pareto()


# ------------------------------------------------------------- requests
@dataclass
class Score:
    """score_func on the whole dataset for each tree (LossFunctions.jl:86-92)."""
    trees: List[Node]


@dataclass
class ScoreRows:
    """score_func_batch: each tree with the row sample its call drew (:95-115)."""
    trees: List[Node]
    rows: List[np.ndarray]


@dataclass
class Optimize:
    """optimize_constants of each tree (in place) with this start noise."""
    trees: List[Node]
    noise: np.ndarray


@dataclass
class OptimizeAnswer:
    losses: np.ndarray
    converged: np.ndarray
    num_evals: np.ndarray


# ------------------------------------------------------------- the island
class Island:
    """The worker side of one population: its stream, birth counter and state."""

    def __init__(self, idx: int, seed: int):
        self.idx = idx
        self.rng = np.random.default_rng(np.random.SeedSequence([seed, 1, idx]))
        self.clock = 0
        self.pop: List[PopMember] = []
        self.best_seen: Optional[HallOfFame] = None
        self.num_evals = 0.0

    def born(self) -> int:
        self.clock += 1
        return self.clock


class Search:
    """State shared by the islands of one search: dataset facts, options, T."""

    def __init__(self, options, nfeatures: int, n_rows: int, T, baseline: float):
        self.options = options
        self.nfeatures = nfeatures
        self.n = n_rows
        self.T = T
        self.baseline = baseline
        self._pars = {}
        self.weights = list(_mutation_weights(options))
        p, n = options.tournament_selection_p, options.tournament_selection_n
        self.tournament_weights = [p * (1 - p) ** k for k in range(n)]  # sample_tournament (:122-132)
        # the same draw as _sample_weighted(tournament_weights): u < c over the running sums
        self.tournament_wsum = sum(self.tournament_weights)
        self.tournament_cum = list(itertools.accumulate(self.tournament_weights))
        self.tournament_last = max(i for i, w in enumerate(self.tournament_weights) if w > 0) if n else 0
        self.freq_scale = float(T(options.adaptive_parsimony_scaling))

    def batch_score_of(self, loss_ok, size: int):
        """score_func_batch's (score, loss): (0, Inf) when the evaluation
        failed (LossFunctions.jl:102-104)."""
        loss, ok = float(loss_ok[0]), bool(loss_ok[1])
        if not ok:
            return 0.0, math.inf
        return self.score_of(loss, size), loss

    def score_of(self, loss: float, size: int) -> float:
        """loss_to_score (LossFunctions.jl:73-82) in T; size = compute_complexity."""
        T = self.T
        pt = self._pars.get(size)
        if pt is None:
            pt = self._pars[size] = T(np.float32(size) * np.float32(self.options.parsimony))
        b = T(self.baseline)
        norm = T(0.01) if b < T(0.01) else b
        return float(T(T(T(loss) / norm) + pt))  # (numpy warnings are off for the whole search)


def _mutation_weights(options):
    w = getattr(options, "mutation_weights", None)
    if w is None:
        return DEFAULT_MUTATION_WEIGHTS
    if isinstance(w, dict):
        d = dict(zip(MUTATIONS, DEFAULT_MUTATION_WEIGHTS))
        d.update(w)
        return tuple(float(d[k]) for k in MUTATIONS)
    w = [float(v) for v in w]
    return tuple(w + [0.0] * (len(MUTATIONS) - len(w)))  # Options.jl:409-417


def _sample_weighted(p, rng) -> int:
    """StatsBase.sample(items, Weights(w)): index by the cumulative weights."""
    u = rng.random() * sum(p)
    c = 0.0
    for i, w in enumerate(p):
        c += w
        if u < c:
            return i
    return max(i for i, w in enumerate(p) if w > 0)


def best_of_sample(isl: Island, S: Search, freqs: np.ndarray) -> PopMember:
    """Population.jl:79-119."""
    o, rng = S.options, isl.rng
    n_t = o.tournament_selection_n
    pop = isl.pop
    sample = [pop[i] for i in rng.permutation(len(pop))[:n_t].tolist()]  # sample_pop, replace=false
    if o.use_frequency_in_tournament:
        scale = S.freq_scale
        maxsize = o.maxsize
        fr = freqs.tolist()
        exp = math.exp
        f32 = S.T is np.float32
        scores = []
        for m in sample:
            size = (m.info or minfo(m, o))[0]
            scores.append(m.score * exp(scale * (fr[size - 1] if 0 < size <= maxsize else 0.0)))
        if f32:  # T(...), all at once (Float64 values are already T)
            scores = np.array(scores).astype(np.float32).tolist()
    else:
        scores = [m.score for m in sample]
    if o.tournament_selection_p == 1.0:  # argmin(scores) (Population.jl:109-110): the first NaN, else the first minimum
        best, bv = 0, math.inf
        for i, v in enumerate(scores):
            if v != v:
                return sample[i]
            if v < bv:
                best, bv = i, v
        return sample[best]
    else:  # StatsBase.sample(1:n, Weights(w)) by the cumulative weights (_sample_weighted)
        k = bisect.bisect_right(S.tournament_cum, rng.random() * S.tournament_wsum)
        if k >= n_t:
            k = S.tournament_last
    if k == 0:  # partialsortperm(scores, 1): the first smallest, NaN last (isless)
        best, bv = 0, math.nan
        for i, v in enumerate(scores):
            if v < bv or (bv != bv and v == v):
                best, bv = i, v
        return sample[best]
    # partialsortperm(scores, k+1): NaN sorts last (isless)
    order = sorted(range(n_t), key=lambda i: (math.isnan(scores[i]), scores[i]))
    return sample[order[k]]


def next_generation(isl: Island, S: Search, member: PopMember, temperature, curmaxsize: int,
                    freqs: np.ndarray):
    """Mutate.jl:25-282. Returns (baby, accepted, num_evals)."""
    o, rng, T = S.options, isl.rng, S.T
    prev = member.tree
    num_evals = 0.0
    if o.batching:
        rows = rng.integers(0, S.n, size=o.batch_size)
        ans = yield ScoreRows([prev], [rows])
        before_score, before_loss = S.batch_score_of(ans[0], minfo(member, o)[0])
        num_evals += o.batch_size / S.n
    else:
        before_score, before_loss = member.score, member.loss
    w = list(S.weights)
    n, depth, nconst = minfo(member, o)
    w[0] *= min(8, nconst) / 8.0
    maxdepth = o.maxdepth if o.maxdepth is not None else o.maxsize
    if n >= curmaxsize or depth >= maxdepth:
        w[2] = 0.0
        w[3] = 0.0
    choice = MUTATIONS[_sample_weighted(w, rng)]
    successful = False
    attempts = 0
    tree = prev
    while not successful and attempts < 10:
        tree = copy_node(prev)
        successful = True
        if choice == "mutate_constant":
            tree = mutate_constant(tree, temperature, o, T, rng)
        elif choice == "mutate_operator":
            tree = mutate_operator(tree, o, rng)
        elif choice == "add_node":
            if rng.random() < 0.5:
                tree = append_random_op(tree, o, S.nfeatures, T, rng)
            else:
                tree = prepend_random_op(tree, o, S.nfeatures, T, rng)
        elif choice == "insert_node":
            tree = insert_random_op(tree, o, S.nfeatures, T, rng)
        elif choice == "delete_node":
            tree = delete_random_op(tree, o, S.nfeatures, T, rng)
        elif choice == "simplify":
            tree = simplify_tree(tree, o, T)
            tree = combine_operators(tree, o, T)
            return PopMember(tree, before_score, before_loss, isl.born(), parent=member.ref), True, num_evals
        elif choice == "randomize":
            tree = gen_random_tree_fixed_size(_rand_int(rng, 1, curmaxsize), o, S.nfeatures, T, rng)
        elif choice == "optimize":
            cur = PopMember(tree, before_score, before_loss, isl.born(), parent=member.ref)
            ev = yield from optimize_members(isl, S, [cur])
            return cur, True, num_evals + ev
        else:  # do_nothing
            return PopMember(tree, before_score, before_loss, isl.born(), parent=member.ref), True, num_evals
        successful = successful and check_constraints(tree, o, curmaxsize)
        attempts += 1
    if not successful:
        return _rejected(isl, S, prev, before_score, before_loss, member), False, num_evals
    info = tree_info(tree, o)
    if o.batching:
        rows = rng.integers(0, S.n, size=o.batch_size)
        ans = yield ScoreRows([tree], [rows])
        after_score, after_loss = S.batch_score_of(ans[0], info[0])
        num_evals += o.batch_size / S.n
    else:
        ans = yield Score([tree])
        after_loss = float(ans[0])
        after_score = S.score_of(after_loss, info[0])
        num_evals += 1
    if math.isnan(after_score):
        return _rejected(isl, S, prev, before_score, before_loss, member), False, num_evals
    prob = 1.0
    if o.annealing:
        with np.errstate(all="ignore"):
            delta = T(T(after_score) - T(before_score))
            prob *= float(np.exp(T(-delta / T(T(temperature) * T(o.alpha)))))
    if o.use_frequency:
        old_size = n
        new_size = info[0]
        old_f = freqs[old_size - 1] if 0 < old_size <= o.maxsize else 1e-6
        new_f = freqs[new_size - 1] if 0 < new_size <= o.maxsize else 1e-6
        prob *= old_f / new_f
    if prob < rng.random():  # Mutate.jl:247 (a NaN probChange keeps the baby)
        return _rejected(isl, S, prev, before_score, before_loss, member), False, num_evals
    return PopMember(tree, after_score, after_loss, isl.born(), parent=member.ref, info=info), True, num_evals


def _rejected(isl: Island, S: Search, prev: Node, score: float, loss: float, member: PopMember) -> PopMember:
    """The PopMember(copy_node(prev), ...) a rejected mutation returns. With
    skip_mutation_failures (default) the caller drops it unread, so the tree
    copy is skipped; the birth order is still consumed."""
    tree = prev if S.options.skip_mutation_failures else copy_node(prev)
    return PopMember(tree, score, loss, isl.born(), parent=member.ref, info=member.info)


def crossover_generation(isl: Island, S: Search, m1: PopMember, m2: PopMember, curmaxsize: int):
    """Mutate.jl:285-341. Returns (baby1, baby2, accepted, num_evals)."""
    o, rng = S.options, isl.rng
    c1, c2 = crossover_trees(m1.tree, m2.tree, rng)
    tries = 1
    while True:
        if check_constraints(c1, o, curmaxsize) and check_constraints(c2, o, curmaxsize):
            break
        if tries > 10:
            return m1, m2, False, 0.0
        c1, c2 = crossover_trees(m1.tree, m2.tree, rng)
        tries += 1
    if o.batching:
        r1 = rng.integers(0, S.n, size=o.batch_size)
        r2 = rng.integers(0, S.n, size=o.batch_size)
        a1, a2 = yield ScoreRows([c1, c2], [r1, r2])
        s1, l1 = S.batch_score_of(a1, compute_complexity(c1, o))
        s2, l2 = S.batch_score_of(a2, compute_complexity(c2, o))
        ev = 2 * (o.batch_size / S.n)
    else:
        l1, l2 = yield Score([c1, c2])
        s1, s2 = S.score_of(l1, compute_complexity(c1, o)), S.score_of(l2, compute_complexity(c2, o))
        ev = o.batch_size / S.n  # as written (:321)
    b1 = PopMember(c1, s1, float(l1), isl.born(), parent=m1.ref)
    b2 = PopMember(c2, s2, float(l2), isl.born(), parent=m2.ref)
    return b1, b2, True, ev


def _oldest(pop: List[PopMember]) -> int:
    best, bi = None, 0
    for i, m in enumerate(pop):
        if best is None or m.birth < best:
            best, bi = m.birth, i
    return bi


def reg_evol_cycle(isl: Island, S: Search, temperature, curmaxsize: int, freqs: np.ndarray):
    """RegularizedEvolution.jl:81-155 (fast_cycle = false)."""
    o, rng = S.options, isl.rng
    num_evals = 0.0
    pop = isl.pop
    for _ in range(round(len(pop) / o.tournament_selection_n)):
        if rng.random() > o.crossover_probability:
            allstar = best_of_sample(isl, S, freqs)
            baby, accepted, ev = yield from next_generation(isl, S, allstar, temperature, curmaxsize, freqs)
            num_evals += ev
            if not accepted and o.skip_mutation_failures:
                continue
            pop[_oldest(pop)] = baby
        else:
            a1 = best_of_sample(isl, S, freqs)
            a2 = best_of_sample(isl, S, freqs)
            b1, b2, accepted, ev = yield from crossover_generation(isl, S, a1, a2, curmaxsize)
            num_evals += ev
            if not accepted and o.skip_mutation_failures:
                continue
            pop[_oldest(pop)] = b1
            pop[_oldest(pop)] = b2
    return num_evals


def s_r_cycle(isl: Island, S: Search, ncycles: int, curmaxsize: int, freqs: np.ndarray):
    """SingleIteration.jl:17-61: returns the island's best-seen hall of fame."""
    o, T = S.options, S.T
    temps = np.linspace(1.0, 0.0 if o.annealing else 1.0, ncycles).astype(T) if ncycles > 0 else []
    best = HallOfFame(o, T)
    num_evals = 0.0
    for temperature in temps:
        num_evals += yield from reg_evol_cycle(isl, S, temperature, curmaxsize, freqs)
        for m in isl.pop:
            size = minfo(m, o)[0]
            if 0 < size <= o.maxsize and (not best.exists[size - 1] or m.score < best.members[size - 1].score):
                best.exists[size - 1] = True
                best.members[size - 1] = copy_member(m)
    return best, num_evals


def start_noise(trees: Sequence[Node], nrestarts: int, rng) -> np.ndarray:
    """`randn(T, nconst)` per restart per tree with constants (ConstantOptimization.jl:46-54)."""
    parts = []
    for t in trees:
        n = count_constants(t)
        for _ in range(nrestarts if n else 0):
            parts.append(rng.standard_normal(n))
    return np.concatenate(parts) if parts else np.zeros(0)


def optimize_members(isl: Island, S: Search, members: List[PopMember]):
    """optimize_constants for each member (ConstantOptimization.jl:22-65): the
    trees are updated in place; a converged member is re-scored and re-born."""
    o = S.options
    todo = [m for m in members if minfo(m, o)[2] > 0]
    if not todo:
        return 0.0
    noise = start_noise([m.tree for m in todo], o.optimizer_nrestarts, isl.rng)
    ans = yield Optimize([m.tree for m in todo], noise)
    conv = [m for m, ok in zip(todo, ans.converged) if ok]
    if conv:
        # `member.score, member.loss = score_func(...)` (:58; counted in num_evals)
        losses = yield Score([m.tree for m in conv])
        for m, l in zip(conv, losses):
            m.loss = float(l)
            m.score = S.score_of(m.loss, minfo(m, o)[0])
            m.birth = isl.born()
    return float(np.sum(ans.num_evals))


def optimize_and_simplify_population(isl: Island, S: Search, curmaxsize: int):
    """SingleIteration.jl:63-127 (+ finalize_scores, Population.jl:134-148)."""
    o, rng, T = S.options, isl.rng, S.T
    pop = isl.pop
    do_opt = rng.random(len(pop)) < o.optimizer_probability
    for m in pop:
        m.tree = simplify_tree(m.tree, o, T)
        m.tree = combine_operators(m.tree, o, T)
        m.info = None
    num_evals = 0.0
    if o.should_optimize_constants:
        num_evals += yield from optimize_members(isl, S, [m for m, d in zip(pop, do_opt) if d])
    if o.batching:  # finalize_scores
        losses = yield Score([m.tree for m in pop])
        for m, l in zip(pop, losses):
            m.loss = float(l)
            m.score = S.score_of(l, minfo(m, o)[0])
        num_evals += len(pop) * (o.batch_size / S.n)
    for m in pop:  # new references
        m.parent = m.ref
        m.ref = int(rng.integers(0, 2 ** 62))
    return num_evals


def island_init(isl: Island, S: Search):
    """Population(dataset; npop, nlength=3) (Population.jl:31-46)."""
    o = S.options
    trees = [gen_random_tree(3, o, S.nfeatures, S.T, isl.rng) for _ in range(o.npop)]
    losses = yield Score(trees)
    isl.pop = [PopMember(t, S.score_of(l, compute_complexity(t, o)), float(l), isl.born(),
                         int(isl.rng.integers(0, 2 ** 62))) for t, l in zip(trees, losses)]
    isl.num_evals = float(o.npop)


def island_iteration(isl: Island, S: Search, curmaxsize: int, freqs: np.ndarray, first: bool):
    """One spawned job of SymbolicRegression.jl:588-627 / :794-832."""
    o = S.options
    best, ev = yield from s_r_cycle(isl, S, o.ncycles_per_iteration, curmaxsize, freqs)
    ev += yield from optimize_and_simplify_population(isl, S, curmaxsize)
    if o.batching:
        idx = [i for i in range(len(best.members)) if first or best.exists[i]]
        losses = yield Score([best.members[i].tree for i in idx])
        for i, l in zip(idx, losses):
            best.members[i].loss = float(l)
            best.members[i].score = S.score_of(l, minfo(best.members[i], o)[0])
        ev += len(idx)
    isl.best_seen = best
    isl.num_evals = ev


# ------------------------------------------------------------- drivers
class Stats:
    def __init__(self):
        self.launches = 0
        self.trees_scored = 0
        self.optimize_calls = 0
        self.engine_seconds = 0.0


def _answer(kind, reqs, evaluator, stats: Stats):
    """One evaluator call for all requests of one kind; returns per-request answers."""
    t0 = time.perf_counter()
    if kind is Score:
        trees = [t for r in reqs for t in r.trees]
        out = np.asarray(evaluator.losses(trees), dtype=np.float64) if trees else np.zeros(0)
        stats.launches += 1
        stats.trees_scored += len(trees)
    elif kind is ScoreRows:
        trees = [t for r in reqs for t in r.trees]
        rows = [x for r in reqs for x in r.rows]
        losses, ok = evaluator.losses_rows(trees, rows)
        out = np.stack([np.asarray(losses, dtype=np.float64), np.asarray(ok, dtype=np.float64)], axis=1)
        stats.launches += 1
        stats.trees_scored += len(trees)
    else:
        trees = [t for r in reqs for t in r.trees]
        noise = np.concatenate([r.noise for r in reqs]) if reqs else np.zeros(0)
        res = evaluator.optimize(trees, noise)
        stats.optimize_calls += 1
        stats.engine_seconds += time.perf_counter() - t0
        answers, k = [], 0
        for r in reqs:
            n = len(r.trees)
            answers.append(OptimizeAnswer(res.losses[k:k + n], res.converged[k:k + n], res.num_evals[k:k + n]))
            k += n
        return answers
    stats.engine_seconds += time.perf_counter() - t0
    answers, k = [], 0
    for r in reqs:
        n = len(r.trees)
        answers.append(out[k:k + n])
        k += n
    return answers


def run_lockstep(jobs: Dict[int, Iterator], evaluator, stats: Stats) -> None:
    """Advance every island job to its next request; answer all pending
    requests with one evaluator call per request kind; repeat."""
    pending = {}
    for i, g in jobs.items():
        try:
            pending[i] = next(g)
        except StopIteration:
            pass
    while pending:
        by_kind: Dict[type, List[int]] = {}
        for i, r in pending.items():
            by_kind.setdefault(type(r), []).append(i)
        answers = {}
        for kind in (Score, ScoreRows, Optimize):
            ids = by_kind.get(kind)
            if ids:
                for i, a in zip(ids, _answer(kind, [pending[i] for i in ids], evaluator, stats)):
                    answers[i] = a
        nxt = {}
        for i in pending:
            try:
                nxt[i] = jobs[i].send(answers[i])
            except StopIteration:
                pass
        pending = nxt


def run_serial(jobs: Dict[int, Iterator], evaluator, stats: Stats) -> None:
    """The reference's schedule: one island after the other, one call per request."""
    for i, g in jobs.items():
        try:
            r = next(g)
            while True:
                r = g.send(_answer(type(r), [r], evaluator, stats)[0])
        except StopIteration:
            pass


# ------------------------------------------------------------- evaluators
class EngineEvaluator:
    """The engine behind the three request kinds (one launch each)."""

    def __init__(self, dataset, options, device=None):
        self.dataset, self.options, self.device = dataset, options, device

    def losses(self, trees):
        from .interface import eval_loss_batch

        return eval_loss_batch(trees, self.dataset, self.options, device=self.device)

    def losses_rows(self, trees, rows):
        from .interface import eval_loss_batch_rowsets

        return eval_loss_batch_rowsets(trees, self.dataset, self.options, rows, device=self.device)

    def optimize(self, trees, noise):
        from .constant_optimization import optimize_constants_batch

        return optimize_constants_batch(self.dataset, trees, self.options, noise=noise, device=self.device)


# ------------------------------------------------------------- head node
@dataclass
class SearchResult:
    hall_of_fame: HallOfFame
    populations: List[List[PopMember]]
    stats: dict = field(default_factory=dict)


def _migrate(candidates: List[PopMember], isl: Island, frac: float, rng) -> None:
    """Migration.jl:16-35."""
    npop = len(isl.pop)
    num = round(npop * frac)
    if num <= 0 or not candidates:
        return
    locations = rng.integers(0, npop, size=num)
    picks = rng.integers(0, len(candidates), size=num)
    for loc, k in zip(locations, picks):
        m = copy_member(candidates[int(k)])
        m.birth = isl.born()  # copy_pop_member_reset_birth
        isl.pop[int(loc)] = m


def equation_search_default(dataset, options, niterations: int, evaluator, seed: int = 0, lockstep: bool = True,
                            rank: int = 0, world: int = 1, group=None, verbose: bool = False) -> SearchResult:
    with np.errstate(all="ignore"):  # Julia's IEEE arithmetic: Inf / NaN scores are values, not errors
        return _equation_search_default(dataset, options, niterations, evaluator, seed, lockstep, rank, world,
                                        group, verbose)


def _equation_search_default(dataset, options, niterations, evaluator, seed, lockstep, rank, world, group,
                             verbose) -> SearchResult:
    """_EquationSearch (SymbolicRegression.jl:439-935) for one output, islands
    in lockstep. `dataset` needs n, nfeatures, T and baseline_loss set."""
    o = options
    T = np.dtype(dataset.T).type
    S = Search(o, dataset.nfeatures, dataset.n, T, float(dataset.baseline_loss))
    npops = o.npopulations
    mine = [i for i in range(npops) if i % world == rank]
    islands = {i: Island(i, seed) for i in range(npops)}
    head = np.random.default_rng(np.random.SeedSequence([seed, 0]))
    stats_rs = RunningSearchStatistics(o)
    hof = HallOfFame(o, T)
    curmaxsize = o.maxsize if o.warmup_maxsize_by == 0.0 else 3
    st = Stats()
    run = run_lockstep if lockstep else run_serial
    t0 = time.perf_counter()

    def gather():
        """Every rank receives every island's state (sharded search only)."""
        if world == 1:
            return
        import torch.distributed as dist

        out = [None] * world
        dist.all_gather_object(out, {i: (islands[i].pop, islands[i].best_seen, islands[i].clock,
                                         islands[i].num_evals) for i in mine}, group=group)
        for part in out:
            for i, (pop, best, clock, ev) in part.items():
                isl = islands[i]
                isl.pop, isl.best_seen, isl.clock, isl.num_evals = pop, best, clock, ev

    # dummy best sub-populations (SearchUtils.jl:47-57), on the head
    dtrees = [gen_random_tree(3, o, S.nfeatures, T, head) for _ in range(npops)]
    dl = _answer(Score, [Score(dtrees)], evaluator, st)[0]
    best_sub = [[PopMember(t, S.score_of(l, compute_complexity(t, o)), float(l), 0)] for t, l in zip(dtrees, dl)]
    # initial populations and the first spawn (:539-630): every island, frequencies uniform
    run({i: island_init(islands[i], S) for i in mine}, evaluator, st)
    freqs0 = stats_rs.snapshot()
    spawned = {i: (curmaxsize, freqs0) for i in mine}
    total_evals = {i: float(o.npop) for i in range(npops)}
    all_idx = list(range(npops))
    head.shuffle(all_idx)
    first = True
    for it in range(niterations):
        run({i: island_iteration(islands[i], S, spawned[i][0], spawned[i][1], first) for i in mine}, evaluator, st)
        gather()
        first = False
        last_round = it == niterations - 1
        spawned = {}
        for pos, i in enumerate(all_idx):  # the head node, SymbolicRegression.jl:695-866
            isl = islands[i]
            total_evals[i] += isl.num_evals
            order = sorted(range(len(isl.pop)), key=lambda k: (math.isnan(isl.pop[k].score), isl.pop[k].score))
            best_sub[i] = [copy_member(isl.pop[k]) for k in order[:o.topn]]
            best_pops = [m for sub in best_sub for m in sub]
            cand = list(isl.pop) + [m for m, e in zip(isl.best_seen.members, isl.best_seen.exists) if e]
            for k, m in enumerate(cand):
                size = minfo(m, o)[0]
                if k < len(isl.pop):
                    stats_rs.update_frequencies(size)
                if 0 < size < o.maxsize + MAX_DEGREE:
                    if not hof.exists[size - 1] or m.score < hof.members[size - 1].score:
                        hof.members[size - 1] = copy_member(m)
                        hof.exists[size - 1] = True
            dominating = hof.pareto()
            if o.migration:
                _migrate(best_pops, isl, o.fraction_replaced, head)
            if o.hof_migration and dominating:
                _migrate(dominating, isl, o.fraction_replaced_hof, head)
            if last_round and pos == len(all_idx) - 1:
                break  # cycles_remaining == 0 (:781-784)
            if not last_round:
                spawned[i] = (curmaxsize, stats_rs.snapshot())
            cycles_elapsed = it * npops + pos + 1
            if o.warmup_maxsize_by > 0:
                frac = np.float32(cycles_elapsed) / np.float32(npops * niterations)
                if frac > o.warmup_maxsize_by:
                    curmaxsize = o.maxsize
                else:
                    curmaxsize = 3 + int(math.floor((o.maxsize - 3) * frac / o.warmup_maxsize_by))
            stats_rs.move_window()
        spawned = {i: v for i, v in spawned.items() if i in mine}
        if verbose and rank == 0:
            front = hof.pareto()
            print(f"iteration {it + 1}: best loss {min(m.loss for m in front) if front else math.inf:.4g}, "
                  f"{time.perf_counter() - t0:.1f} s, {st.launches} launches", flush=True)
    secs = time.perf_counter() - t0
    evals = float(sum(total_evals.values()))
    stats = dict(evals=evals, seconds=secs, evals_per_s=evals / max(secs, 1e-12),
                 seconds_per_iteration=secs / max(niterations, 1), iterations=niterations,
                 launches=st.launches, trees_scored=st.trees_scored, optimize_calls=st.optimize_calls,
                 engine_seconds=st.engine_seconds, engine_share=st.engine_seconds / max(secs, 1e-12))
    return SearchResult(hof, [islands[i].pop for i in range(npops)], stats)
