"""Random trees: ports of the reference's generators (src/MutationFunctions.jl)
used for synthetic workloads (BASELINE.json configs) and tests.

The reference draws from Julia's global RNG; here a numpy Generator is
passed explicitly (distributions are the same, streams are not).
"""
from __future__ import annotations

from typing import List

import numpy as np

from .node import Node, count_nodes


def make_random_leaf(nfeatures: int, T, rng: np.random.Generator) -> Node:
    """MutationFunctions.jl:151-157: constant randn(T) or a uniform feature."""
    if rng.random() > 0.5:
        return Node(val=T(rng.standard_normal()))
    return Node(feature=int(rng.integers(1, nfeatures + 1)))


def _leaves(tree: Node) -> List[Node]:
    out, stack = [], [tree]
    while stack:
        t = stack.pop()
        if t.degree == 0:
            out.append(t)
        else:
            stack.append(t.l)
            if t.degree == 2:
                stack.append(t.r)
    return out


def _set_node(dst: Node, src: Node) -> None:
    for k in Node.__slots__:
        setattr(dst, k, getattr(src, k))


def append_random_op(tree: Node, options, nfeatures: int, T, rng: np.random.Generator,
                     make_new_bin_op=None) -> Node:
    """MutationFunctions.jl:82-114: replace a uniformly chosen leaf
    (random_node until degree == 0) by op(leaf[, leaf])."""
    leaves = _leaves(tree)
    node = leaves[int(rng.integers(0, len(leaves)))]
    if make_new_bin_op is None:
        make_new_bin_op = rng.random() < options.nbin / (options.nuna + options.nbin)
    if make_new_bin_op:
        new = Node(int(rng.integers(1, options.nbin + 1)), make_random_leaf(nfeatures, T, rng),
                   make_random_leaf(nfeatures, T, rng))
    else:
        new = Node(int(rng.integers(1, options.nuna + 1)), make_random_leaf(nfeatures, T, rng))
    _set_node(node, new)
    return tree


def gen_random_tree_fixed_size(node_count: int, options, nfeatures: int, T,
                               rng: np.random.Generator) -> Node:
    """MutationFunctions.jl:248-263."""
    tree = make_random_leaf(nfeatures, T, rng)
    cur = count_nodes(tree)
    while cur < node_count:
        if cur == node_count - 1:
            if options.nuna == 0:
                break
            tree = append_random_op(tree, options, nfeatures, T, rng, make_new_bin_op=False)
        else:
            tree = append_random_op(tree, options, nfeatures, T, rng)
        cur = count_nodes(tree)
    return tree


def gen_random_tree(length: int, options, nfeatures: int, T, rng: np.random.Generator) -> Node:
    """MutationFunctions.jl:236-246."""
    tree = Node(val=T(1))
    for _ in range(length):
        tree = append_random_op(tree, options, nfeatures, T, rng)
    return tree


def random_population(ntrees: int, options, nfeatures: int, T, seed: int = 0,
                      maxsize: int = 30) -> List[Node]:
    """Config #2's synthetic batch: sizes ~ U{1..maxsize} (Mutate.jl:131-132)."""
    rng = np.random.default_rng(seed)
    return [gen_random_tree_fixed_size(int(rng.integers(1, maxsize + 1)), options, nfeatures, T, rng)
            for _ in range(ntrees)]
