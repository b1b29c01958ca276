"""Batched constant optimisation: the Python mirror
of `optimize_constants` (src/ConstantOptimization.jl:22-65) for a whole
population, over libsrhip's lockstep optimiser (csrc/constopt.cpp).

The reference optimises one PopMember at a time: Optim.Newton (one
constant) or Optim.BFGS — or NelderMead (:35-36) — with
LineSearches.BackTracking, `optimizer_iterations` = 8 (src/Options.jl:607-621),
from x0 and from `optimizer_nrestarts` = 2 perturbed starts x0 .* (1 + randn/2)
(:46-54); the best run is kept if Optim reports convergence, else the
constants go back to x0 (:56-63).

Here every start of every tree is a candidate and all candidates advance in
lockstep inside libsrhip (srhip_optimize_constants_batch): each phase of an
iteration is ONE launch over all of them (srhip_program_set_constants +
srhip_eval_loss_grad / srhip_eval_loss). The per-candidate algebra runs in
C++ next to the engine; this module draws the start noise (from the caller's
numpy Generator, tree by tree, restart by restart — where the reference
calls randn) and writes the results back into the trees.

`evaluator_factory` plugs any other evaluator into the same C++ driver
through srhip_optimize_constants_cb (a row-sharded dataset whose partials
are all-reduced, the oracle in tests): factory(candidates) returns an object
with loss_grad(consts) -> (f, g) and loss_only(consts) -> f. No part of the
optimiser runs in Python; tests/constopt_reference.py restates it as the
checker.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Callable, Optional, Sequence

import numpy as np

from ._lib import CONSTOPT_EVAL_FN, ConstOptOptions, check, lib
from .dataset import Dataset
from .engine import _trees_struct
from .node import Node, flatten, set_constants
from .options import Options

ALGORITHMS = {"BFGS": 0, "NelderMead": 1}  # SRHIP_OPT_*


@dataclass
class ConstOptResult:
    """Per input tree: the loss after optimisation (the reference re-scores a
    converged member, :56-60; else the loss at x0), Optim's convergence flag of
    the best start, and the number of loss evaluations (num_evals)."""

    losses: np.ndarray
    converged: np.ndarray
    num_evals: np.ndarray


def _finish(sums, wsum, ok) -> np.ndarray:
    """Loss of each candidate from engine partials (:12-19): Σw·ℓ/Σw, +Inf on failure."""
    with np.errstate(invalid="ignore", divide="ignore"):
        f = sums / wsum
    return np.where(ok & np.isfinite(f), f, np.inf)


def _grad_finish(grads, wsum, ok, const_off) -> np.ndarray:
    """∂L/∂c of each constant from engine partials, NaN for failed candidates."""
    g = grads / wsum
    g[np.repeat(~ok, np.diff(const_off))] = np.nan
    return g


def start_noise(flat, nrestarts: int, rng: np.random.Generator) -> np.ndarray:
    """The standard normal draws of the perturbed starts in the C ABI's order
    (tree by tree, restart by restart, :46-54)."""
    co = flat.const_off
    parts = []
    for i in range(flat.ntrees):
        n = int(co[i + 1] - co[i])
        for _ in range(nrestarts if n else 0):
            parts.append(rng.standard_normal(n))
    return np.concatenate(parts) if parts else np.zeros(0)


def optimize_constants_batch(dataset: Dataset, trees: Sequence[Node], options: Options,
                             rng: Optional[np.random.Generator] = None, device: Optional[int] = None,
                             evaluator_factory: Optional[Callable] = None,
                             noise: Optional[np.ndarray] = None) -> ConstOptResult:
    """`optimize_constants` for many trees at once. Trees are updated in place
    (constants of the best start when it converged, else left at x0).
    `noise` (default: drawn from `rng`) is the standard normal draws of the
    perturbed starts in start_noise's order, for callers that draw them
    where the reference does (srhip.evolution: from each island's stream)."""
    algorithm = getattr(options, "optimizer_algorithm", "BFGS")
    if algorithm not in ALGORITHMS:
        raise ValueError("Optimization function not implemented.")  # :39-41
    T = np.dtype(dataset.T).type
    flat = flatten(trees, options, dtype=T)
    nrestarts = int(getattr(options, "optimizer_nrestarts", 2))
    if noise is None:
        noise = start_noise(flat, nrestarts, rng or np.random.default_rng())
    noise = np.ascontiguousarray(noise, dtype=np.float64)
    need = int(sum(nrestarts * int(flat.const_off[i + 1] - flat.const_off[i]) for i in range(flat.ntrees)))
    if noise.shape != (need,):
        raise ValueError(f"start noise has {noise.size} values, the trees' restarts need {need}")
    loss = options.elementwise_loss
    par = None if loss.params is None else np.ascontiguousarray(loss.params, dtype=np.float64)
    opts = ConstOptOptions(ALGORITHMS[algorithm], int(getattr(options, "optimizer_iterations", 8)), nrestarts,
                           int(loss.kind), None if par is None else par.ctypes.data_as(C.POINTER(C.c_double)),
                           noise.ctypes.data_as(C.POINTER(C.c_double)), 0)
    consts = np.ascontiguousarray(flat.consts, dtype=T)
    tr = _trees_struct(flat, consts)
    nt = len(trees)
    out_c = np.zeros(max(consts.size, 1), dtype=T)
    out_l = np.zeros(max(nt, 1))
    out_k = np.zeros(max(nt, 1), dtype=np.uint8)
    out_n = np.zeros(max(nt, 1))
    ptrs = [a.ctypes.data_as(C.c_void_p) for a in (out_c, out_l, out_k, out_n)]
    if evaluator_factory is None:
        dev = dataset.device(device)
        check(lib().srhip_optimize_constants_batch(dev.ctx.handle, dev.handle, C.byref(tr), C.byref(opts), *ptrs))
    else:
        cb = _Callback(trees, evaluator_factory)
        rc = lib().srhip_optimize_constants_cb(C.byref(tr), 0 if T == np.float32 else 1, C.byref(opts),
                                               cb.fn, None, *ptrs)
        if cb.error is not None:
            raise cb.error
        check(rc)
    conv = out_k[:nt].astype(bool)
    co = flat.const_off
    for i in np.flatnonzero(conv):
        set_constants(trees[i], [T(v) for v in out_c[co[i]:co[i + 1]]])
    return ConstOptResult(out_l[:nt].copy(), conv, out_n[:nt].copy())


class _Callback:
    """srhip_constopt_eval_fn over evaluator_factory: one evaluator per member
    list the driver asks for (candidates, simplex vertices, line-search
    stragglers, the final trees), built from copies of the input trees."""

    def __init__(self, trees, factory):
        self.trees, self.factory = trees, factory
        self.cache = {}
        self.error = None
        self.fn = CONSTOPT_EVAL_FN(self._eval)

    def _eval(self, _user, n, idx, consts, grad, out_f, out_g):
        try:
            members = np.ctypeslib.as_array(idx, shape=(n,)).copy() if n else np.zeros(0, dtype=np.int32)
            key = members.tobytes()
            ev = self.cache.get(key)
            if ev is None:
                ev = self.factory([self.trees[int(i)].copy() for i in members])
                self.cache[key] = ev
            nconst = sum(len(_consts_of(self.trees[int(i)])) for i in members)
            x = np.ctypeslib.as_array(consts, shape=(nconst,)).copy() if nconst else np.zeros(0)
            if grad:
                f, g = ev.loss_grad(x)
                if nconst:
                    np.ctypeslib.as_array(out_g, shape=(nconst,))[:] = np.asarray(g, dtype=np.float64)
            else:
                f = ev.loss_only(x)
            if n:
                np.ctypeslib.as_array(out_f, shape=(n,))[:] = np.asarray(f, dtype=np.float64)
            return 0
        except BaseException as e:  # reported after the C call returns
            self.error = e
            return 1


def _consts_of(tree: Node):
    from .node import get_constants

    return get_constants(tree)


def last_profile() -> dict:
    """Where the last optimize_constants_batch call of this thread spent its
    time (srhip_constopt_profile): seconds and call counts."""
    out = (C.c_double * 12)()
    check(lib().srhip_constopt_profile(out, 12))
    keys = ("total_s", "create_s", "set_constants_s", "loss_s", "grad_s", "kernel_s", "n_create", "n_loss", "n_grad",
            "n_rebuilt", "jit_codegen_s", "jit_load_s")
    d = dict(zip(keys, (float(v) for v in out)))
    d["host_s"] = d["total_s"] - d["create_s"] - d["set_constants_s"] - d["loss_s"] - d["grad_s"]
    return d

