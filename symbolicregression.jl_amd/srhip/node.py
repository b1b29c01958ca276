"""Expression trees: a Python mirror of DynamicExpressions' `Node{T}` as used
by SymbolicRegression.jl (src/SymbolicRegression.jl:68-86), plus the
flattener to the postfix node streams of include/srhip.h.

Node fields follow the reference: `degree` (0, 1, 2), `constant`, `val`,
`feature` (1-based), `op` (1-based index into options.unary_operators /
binary_operators), `l`, `r`.
"""
from __future__ import annotations

from typing import Iterable, List, Optional, Sequence

import numpy as np

from . import constants as K


class Node:
    __slots__ = ("degree", "constant", "val", "feature", "op", "l", "r")

    def __init__(self, *args, val=None, feature=None, op=None, l=None, r=None):
        self.degree = 0
        self.constant = False
        self.val = 0.0
        self.feature = 0
        self.op = 0
        self.l: Optional[Node] = None
        self.r: Optional[Node] = None
        if args:
            if len(args) == 1 and isinstance(args[0], str):  # Node("x3")
                name = args[0]
                if not (name.startswith("x") and name[1:].isdigit()):
                    raise ValueError(f"feature name must be x<i>, got {name!r}")
                feature = int(name[1:])
            elif isinstance(args[0], (int, np.integer)) and len(args) in (2, 3):
                op = int(args[0])  # Node(op, l[, r])
                l = args[1]
                r = args[2] if len(args) == 3 else None
            else:
                raise TypeError("Node(op, l[, r]), Node('x1'), Node(val=c) or Node(feature=i)")
        if val is not None:
            self.constant = True
            self.val = val
        elif feature is not None:
            if int(feature) < 1:
                raise ValueError("features are 1-based")
            self.feature = int(feature)
        elif op is not None:
            if l is None:
                raise ValueError("operator node needs a child")
            self.op = int(op)
            self.l = l
            self.r = r
            self.degree = 2 if r is not None else 1
        else:
            raise TypeError("Node needs val, feature, or op with children")

    # -- operator overloading (mirrors @extend_operators, InterfaceDynamicExpressions.jl:206-215)
    def _bin(self, other, name, swap=False):
        from .options import _default_options

        opts = _default_options()
        if opts is None:
            raise RuntimeError("call extend_operators(options) before building trees with operators")
        o = other if isinstance(other, Node) else Node(val=other)
        a, b = (o, self) if swap else (self, o)
        return opts.make_binary(name, a, b)

    def __add__(self, o): return self._bin(o, "+")
    def __radd__(self, o): return self._bin(o, "+", True)
    def __sub__(self, o): return self._bin(o, "-")
    def __rsub__(self, o): return self._bin(o, "-", True)
    def __mul__(self, o): return self._bin(o, "*")
    def __rmul__(self, o): return self._bin(o, "*", True)
    def __truediv__(self, o): return self._bin(o, "/")
    def __rtruediv__(self, o): return self._bin(o, "/", True)
    def __pow__(self, o): return self._bin(o, "^")
    def __rpow__(self, o): return self._bin(o, "^", True)

    def copy(self) -> "Node":
        """copy_node: a deep copy (shared children become separate copies)."""
        if self.degree == 0:
            return Node(val=self.val) if self.constant else Node(feature=self.feature)
        if self.degree == 1:
            return Node(self.op, self.l.copy())
        return Node(self.op, self.l.copy(), self.r.copy())

    def __repr__(self) -> str:
        if self.degree == 0:
            return f"Node(val={self.val!r})" if self.constant else f"Node('x{self.feature}')"
        if self.degree == 1:
            return f"Node({self.op}, {self.l!r})"
        return f"Node({self.op}, {self.l!r}, {self.r!r})"


def count_nodes(tree: Node) -> int:
    """count_nodes (DynamicExpressions); shared children count per reference."""
    n, stack = 0, [tree]
    while stack:
        t = stack.pop()
        n += 1
        if t.degree >= 1:
            stack.append(t.l)
        if t.degree == 2:
            stack.append(t.r)
    return n


def _postorder(tree: Node) -> List[Node]:
    out, stack = [], [(tree, False)]
    while stack:
        t, seen = stack.pop()
        if t.degree == 0 or seen:
            out.append(t)
            continue
        stack.append((t, True))
        if t.degree == 2:
            stack.append((t.r, False))
        stack.append((t.l, False))
    return out


def get_constants(tree: Node) -> list:
    """Constants in DynamicExpressions' get_constants order (leaf order, left
    to right; test/test_derivatives.jl:126-150)."""
    return [t.val for t in _postorder(tree) if t.degree == 0 and t.constant]


def set_constants(tree: Node, values: Sequence) -> None:
    it = iter(values)
    for t in _postorder(tree):
        if t.degree == 0 and t.constant:
            t.val = next(it)


def has_constants(tree: Node) -> bool:
    return any(t.degree == 0 and t.constant for t in _postorder(tree))


def string_tree(tree: Node, options) -> str:
    if tree.degree == 0:
        return repr(float(tree.val)) if tree.constant else f"x{tree.feature}"
    if tree.degree == 1:
        return f"{options.unary_operators[tree.op - 1]}({string_tree(tree.l, options)})"
    name = options.binary_operators[tree.op - 1]
    a, b = string_tree(tree.l, options), string_tree(tree.r, options)
    if name in ("+", "-", "*", "/", "^"):
        return f"({a} {name} {b})"
    return f"{name}({a}, {b})"


class FlatTrees:
    """A batch of trees as the postfix node streams of include/srhip.h."""

    def __init__(self, node_off, kind, arg, const_off, consts, nodes):
        self.node_off = node_off
        self.kind = kind
        self.arg = arg
        self.const_off = const_off
        self.consts = consts
        self.nodes = nodes  # count_nodes per tree

    @property
    def ntrees(self) -> int:
        return len(self.node_off) - 1

    def tree(self, t: int):
        b, e = self.node_off[t], self.node_off[t + 1]
        cb, ce = self.const_off[t], self.const_off[t + 1]
        return self.kind[b:e], self.arg[b:e], self.consts[cb:ce]

    def take(self, idx, consts=None) -> "FlatTrees":
        """The trees idx (repeats allowed) as a new batch; `consts` replaces
        their concatenated constants (default: the trees' own)."""
        idx = np.asarray(idx, dtype=np.int64)

        def gather(off, arr):
            lens = np.diff(off)[idx]
            new_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
            pos = np.repeat(off[:-1][idx] - new_off[:-1], lens) + np.arange(new_off[-1])
            return new_off, arr[pos]

        node_off, kind = gather(self.node_off, self.kind)
        _, arg = gather(self.node_off, self.arg)
        const_off, cs = gather(self.const_off, self.consts)
        if consts is not None:
            cs = np.asarray(consts, dtype=self.consts.dtype)
            if cs.shape != (const_off[-1],):
                raise ValueError("constant vector has the wrong length")
        return FlatTrees(node_off, kind, arg, const_off, cs, self.nodes[idx])


def flatten(trees: Iterable[Node], options, dtype=np.float32) -> FlatTrees:
    """Post-order flattening. Operator indices are mapped through the
    options' operator tables to engine ids (raises Unsupported for an
    operator the engine does not implement)."""
    bin_ids, una_ids = options.engine_operator_ids()
    kinds: List[int] = []
    args: List[int] = []
    consts: List[float] = []
    node_off = [0]
    const_off = [0]
    nodes = []
    kapp, aapp, capp = kinds.append, args.append, consts.append
    NC, NF, NU, NB = K.NODE_CONST, K.NODE_FEATURE, K.NODE_UNARY, K.NODE_BINARY

    def emit(t):  # post-order
        d = t.degree
        if d == 0:
            if t.constant:
                kapp(NC)
                aapp(0)
                capp(t.val)
            else:
                kapp(NF)
                aapp(t.feature - 1)
        elif d == 1:
            emit(t.l)
            kapp(NU)
            aapp(una_ids[t.op - 1])
        else:
            emit(t.l)
            emit(t.r)
            kapp(NB)
            aapp(bin_ids[t.op - 1])

    for tree in trees:
        before = len(kinds)
        emit(tree)
        node_off.append(len(kinds))
        const_off.append(len(consts))
        nodes.append(len(kinds) - before)
    return FlatTrees(
        np.asarray(node_off, dtype=np.int32),
        np.asarray(kinds, dtype=np.uint8),
        np.asarray(args, dtype=np.uint16),
        np.asarray(const_off, dtype=np.int32),
        np.asarray(consts, dtype=dtype),
        np.asarray(nodes, dtype=np.int64),
    )
