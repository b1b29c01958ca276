"""TEST-ONLY CHECKER (not product code): the Python restatement of the
lockstep constant optimiser that libsrhip's srhip_optimize_constants_batch /
srhip_optimize_constants_cb (csrc/constopt.cpp) implement. tests/
test_constopt_abi.py drives both over the same evaluator (the CPU oracle)
with the same start noise and requires identical trajectories: constants,
losses, convergence flags and evaluation counts bit for bit.

Reference: optimize_constants, src/ConstantOptimization.jl:22-65 (Optim.Newton
for one constant, else BFGS or NelderMead, LineSearches.BackTracking;
optimizer_iterations iterations from x0 and optimizer_nrestarts starts
x0 .* (1 .+ randn/2), :46-54; the best start kept only if it converged,
:56-63). Every start of every tree is a candidate, all advance in lockstep,
each phase of an iteration is one evaluation of all candidates.

Summation order: every reduction (segment sums, matrix-vector products, the
simplex statistics) is a sequential loop, as in constopt.cpp, so the two
round alike; the start noise is indexed per tree in the input order
(nrestarts * const_off[i] + r * n_i + j), as srhip_constopt_options
.start_noise is. Deviations from Optim, shared with constopt.cpp: analytic
gradients instead of finite differences; Newton's Hessian as the central
difference of the gradient, made positive as PositiveFactorizations does
for 1x1; f_calls counts loss evaluations (a loss + gradient counts once).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from srhip.node import FlatTrees, Node, flatten, get_constants, set_constants

# Optim.Options defaults the reference inherits (g_abstol = 1e-8; x/f tolerances 0).
G_TOL = 1e-8
# LineSearches.BackTracking defaults (c_1, ρ_hi, ρ_lo, order = 3, iterations = 1000).
# Its iterations = 1000 is replaced by 60 shrinks: each shrink multiplies α by at
# most ρ_hi, so after 60 the step is below 2⁻⁶⁰ of the search direction and no
# longer changes x in Float64; a candidate still failing Armijo then is a failed
# line search (LineSearchException → Optim stops, not converged).
C1, RHO_HI, RHO_LO, LS_ITERATIONS = 1e-4, 0.5, 0.1, 60


@dataclass
class ConstOptResult:
    """Per input tree: the loss after optimisation (the reference re-scores a
    converged member, :56-60; else the loss at x0), Optim's convergence flag of
    the best start, and the number of loss evaluations (num_evals)."""

    losses: np.ndarray
    converged: np.ndarray
    num_evals: np.ndarray


def _finish(sums, wsum, ok) -> np.ndarray:
    with np.errstate(invalid="ignore", divide="ignore"):
        f = sums / wsum
    f = np.where(ok & np.isfinite(f), f, np.inf)
    return f


def _grad_finish(grads, wsum, ok, const_off) -> np.ndarray:
    g = grads / wsum
    bad = np.repeat(~ok, np.diff(const_off))
    g[bad] = np.nan
    return g


def _backtrack_step(a1, a2, phi0, dphi0, phix0, phix1, first: bool) -> float:
    """One BackTracking shrink (LineSearches.jl, order 3): quadratic
    interpolation on the first shrink, cubic after, safeguarded to
    [ρ_lo·α, ρ_hi·α]. Published algorithm: Nocedal & Wright §3.5."""
    if first:
        den = 2.0 * (phix1 - phi0 - dphi0 * a2)
        at = -(dphi0 * a2 * a2) / den if den != 0 else np.nan
    else:
        div = 1.0 / (a1 * a1 * a2 * a2 * (a2 - a1))
        r1 = phix1 - phi0 - dphi0 * a2
        r0 = phix0 - phi0 - dphi0 * a1
        a = (a1 * a1 * r1 - a2 * a2 * r0) * div
        b = (-a1 ** 3 * r1 + a2 ** 3 * r0) * div
        if abs(a) <= 1e-12 * max(1.0, abs(b)):
            at = dphi0 / (2.0 * b) if b != 0 else np.nan
        else:
            d = max(b * b - 3.0 * a * dphi0, 0.0)
            at = (-b + np.sqrt(d)) / (3.0 * a)
    hi, lo = a2 * RHO_HI, a2 * RHO_LO
    at = hi if not np.isfinite(at) else min(at, hi)  # NaNMath.min
    return max(at, lo)


def _backtrack_steps(a1, a2, phi0, dphi0, phix0, phix1, first):
    """_backtrack_step for arrays of candidates (NaN/Inf arithmetic as IEEE)."""
    with np.errstate(all="ignore"):
        den = 2.0 * (phix1 - phi0 - dphi0 * a2)
        at_q = np.where(den != 0, -(dphi0 * a2 * a2) / den, np.nan)
        div = 1.0 / (a1 * a1 * a2 * a2 * (a2 - a1))
        r1 = phix1 - phi0 - dphi0 * a2
        r0 = phix0 - phi0 - dphi0 * a1
        a = (a1 * a1 * r1 - a2 * a2 * r0) * div
        b = (-a1 ** 3 * r1 + a2 ** 3 * r0) * div
        lin = np.abs(a) <= 1e-12 * np.maximum(1.0, np.abs(b))
        at_l = np.where(b != 0, dphi0 / (2.0 * b), np.nan)
        d = np.maximum(b * b - 3.0 * a * dphi0, 0.0)
        at_c = (-b + np.sqrt(d)) / (3.0 * a)
        at = np.where(first, at_q, np.where(lin, at_l, at_c))
        hi, lo = a2 * RHO_HI, a2 * RHO_LO
        at = np.where(np.isfinite(at), np.minimum(at, hi), hi)  # NaNMath.min
        return np.maximum(at, lo)


def optimize_constants_batch(dataset, trees: Sequence[Node], options, noise: np.ndarray,
                             evaluator_factory: Callable) -> ConstOptResult:
    """The checker's optimize_constants for many trees: trees are updated in
    place (the best start's constants where it converged, else x0).
    `noise`: [nrestarts * total constants] standard normal draws (start
    noise, natural tree order); `evaluator_factory(candidates)` returns an
    object with loss_grad(consts) -> (f, g) and loss_only(consts) -> f."""
    with np.errstate(all="ignore"):  # NaN/Inf losses and gradients are data here
        return _optimize(dataset, trees, options, np.asarray(noise, dtype=np.float64), evaluator_factory)


def _optimize(dataset, trees, options, noise, factory) -> ConstOptResult:
    T = np.dtype(dataset.T).type
    algorithm = getattr(options, "optimizer_algorithm", "BFGS")
    if algorithm not in ("BFGS", "NelderMead"):
        raise ValueError("Optimization function not implemented.")  # :39-41
    flat = flatten(trees, options, dtype=T)
    ntrees = len(trees)
    acc = dict(num_evals=np.zeros(ntrees), converged=np.zeros(ntrees, dtype=bool),
               consts=np.asarray(flat.consts, dtype=T).copy())
    nconst = np.diff(flat.const_off)
    # one constant: Newton whatever the option says (:32-33); more: NelderMead (:35-36)
    multi = (nconst > 1) if algorithm == "NelderMead" else np.zeros(ntrees, dtype=bool)
    _optimize_gradient(dataset, trees, flat, np.flatnonzero(~multi), options, noise, factory, acc)
    _optimize_nelder_mead(dataset, trees, flat, np.flatnonzero(multi), options, noise, factory, acc)
    for i in np.flatnonzero(acc["converged"]):
        vals = acc["consts"][flat.const_off[i]:flat.const_off[i + 1]]
        set_constants(trees[i], [T(v) for v in vals])
    losses = factory([t for t in trees]).loss_only(acc["consts"].astype(np.float64)) if ntrees else np.zeros(0)
    return ConstOptResult(np.asarray(losses, dtype=np.float64), acc["converged"], acc["num_evals"])


def _starts(flat: FlatTrees, sel, T, nrestarts, noise):
    """Candidates: x0 and `nrestarts` perturbed copies x0 .* (1 + randn/2) per
    selected tree with constants (:42-54); tree i, restart r draws
    noise[nrestarts * const_off[i] + r * n_i : ... + n_i]."""
    cand_tree: List[int] = []
    cand_x: List[np.ndarray] = []
    co = flat.const_off
    for i in sel:
        x0 = np.asarray(flat.consts[co[i]:co[i + 1]], dtype=T)
        if x0.size == 0:
            continue
        cand_tree.append(int(i))
        cand_x.append(x0.copy())
        for r in range(nrestarts):  # :47
            cand_tree.append(int(i))
            z = noise[nrestarts * co[i] + r * x0.size: nrestarts * co[i] + (r + 1) * x0.size]
            cand_x.append((x0 * (T(1) + T(0.5) * z.astype(T))).astype(T))
    return cand_tree, cand_x


def _seqsum_seg(v, starts, sizes):
    """Per-segment sums, each a sequential loop from 0.0 (constopt.cpp)."""
    acc = np.zeros(len(starts))
    for j in range(int(sizes.max()) if len(sizes) else 0):
        m = sizes > j
        acc[m] = acc[m] + v[starts[m] + j]
    return acc


def _matvec(H, g):
    """[m, n, n] x [m, n] -> [m, n], the sum over j sequential."""
    acc = np.zeros(g.shape)
    for j in range(g.shape[1]):
        acc = acc + H[:, :, j] * g[:, None, j]
    return acc


def _dot(a, b):
    acc = np.zeros(a.shape[0])
    for j in range(a.shape[1]):
        acc = acc + a[:, j] * b[:, j]
    return acc


def _pick_best(flat, cand_tree, fbest, xbest, conv, f_calls, acc, T):
    """The best start of every tree (:51-53), kept if it converged (:56-63)."""
    best = {}
    for k, i in enumerate(cand_tree):
        acc["num_evals"][i] += f_calls[k]
        if i not in best or fbest[k] < fbest[best[i]]:
            best[i] = k
    for i, k in best.items():
        if conv[k]:
            acc["consts"][flat.const_off[i]:flat.const_off[i + 1]] = np.asarray(xbest[k], dtype=T)
            acc["converged"][i] = True
            acc["num_evals"][i] += 1


def _optimize_gradient(dataset, trees, flat, sel, options, noise, factory, acc):
    """BFGS (Newton for one constant) with BackTracking, all starts in lockstep."""
    T = np.dtype(dataset.T).type
    iterations = int(getattr(options, "optimizer_iterations", 8))
    nrestarts = int(getattr(options, "optimizer_nrestarts", 2))
    cand_tree, cand_x = _starts(flat, sel, T, nrestarts, noise)
    if not cand_tree:
        return
    ev = _make_evaluator(trees, cand_tree, cand_x, factory)

    nc = len(cand_tree)
    sizes = np.array([x.size for x in cand_x])
    off = np.concatenate([[0], np.cumsum(sizes)])
    starts = off[:-1]
    X = np.concatenate(cand_x).astype(T)
    newton = sizes == 1
    f_calls = np.zeros(nc)
    # candidates grouped by constant count: the BFGS algebra runs batched per group
    groups = {int(sz): np.nonzero(sizes == sz)[0] for sz in np.unique(sizes) if sz > 1}
    gidx = {sz: starts[ks][:, None] + np.arange(sz)[None, :] for sz, ks in groups.items()}  # flat positions
    invH = {sz: np.repeat(np.eye(sz)[None], len(ks), axis=0) for sz, ks in groups.items()}

    def segsum(v):
        return _seqsum_seg(v, starts, sizes)

    def segmax_abs(v):
        return np.maximum.reduceat(np.abs(v), starts)

    f, G = ev.loss_grad(X)
    f_calls += 1
    active = np.isfinite(f)
    with np.errstate(invalid="ignore"):
        conv = active & (segmax_abs(G) <= G_TOL)  # converged at x0
    active &= ~conv

    for _ in range(iterations):
        if not active.any():
            break
        # search directions
        S = np.zeros_like(X, dtype=np.float64)
        nw = newton & active
        if nw.any():
            step = np.where(nw, np.cbrt(np.finfo(T).eps) * np.maximum(1.0, np.abs(X[starts].astype(np.float64))), 0)
            Xp, Xm = X.astype(np.float64), X.astype(np.float64)
            Xp[starts[nw]] += step[nw]
            Xm[starts[nw]] -= step[nw]
            _, Gp = ev.loss_grad(Xp.astype(T))
            _, Gm = ev.loss_grad(Xm.astype(T))
            h = (Gp[starts] - Gm[starts]) / np.where(nw, 2 * step, 1.0)
            hk = np.where(np.isfinite(h) & (np.abs(h) > np.finfo(T).eps), np.abs(h), 1.0)
            S[starts[nw]] = -G[starts[nw]] / hk[nw]
        for sz, ks in groups.items():
            act = active[ks]
            if not act.any():
                continue
            g = G[gidx[sz]]
            sd = -_matvec(invH[sz], g)
            bad = ~(_dot(g, sd) < 0)  # not a descent direction: restart from I
            if (bad & act).any():
                invH[sz][bad & act] = np.eye(sz)
                sd[bad] = -g[bad]
            S[gidx[sz][act]] = sd[act]
        with np.errstate(invalid="ignore", over="ignore"):
            dphi0 = np.where(active, segsum(G * S), 0.0)
        # a NaN gradient (or no descent at all) ends the run: Optim's x would turn NaN
        active &= np.isfinite(dphi0) & (dphi0 < 0)

        # BackTracking line search, all candidates in lockstep
        a1 = np.ones(nc)
        a2 = np.ones(nc)
        phix0 = f.copy()
        searching = active.copy()
        Xbase = X.astype(np.float64)
        trial = ev.loss_only((Xbase + S).astype(T))
        f_calls += searching
        phix1 = np.where(searching, trial, f)
        finite_left = np.where(searching, int(-np.log2(np.finfo(T).eps)), 0)
        first = np.ones(nc, dtype=bool)
        ls_iter = np.zeros(nc, dtype=int)
        while True:
            fin = np.isfinite(phix1)
            halve = searching & ~fin & (finite_left > 0)  # halve until the loss is finite
            searching &= fin | halve
            with np.errstate(invalid="ignore"):
                armijo = searching & fin & (phix1 <= f + C1 * a2 * dphi0)
            searching &= ~armijo
            failed = searching & fin & (ls_iter >= LS_ITERATIONS)  # failed line search: stays at x
            searching &= ~failed
            phix1 = np.where(failed, np.inf, phix1)
            step = searching & fin
            finite_left = np.where(halve, finite_left - 1, finite_left)
            ls_iter = np.where(step, ls_iter + 1, ls_iter)
            at = _backtrack_steps(a1, a2, f, dphi0, phix0, phix1, first)
            shrink = halve | step
            a1 = np.where(shrink, a2, a1)
            a2 = np.where(halve, a2 * 0.5, np.where(step, at, a2))
            first = np.where(step, False, first)
            if not shrink.any():
                break
            alpha_full = np.repeat(a2, sizes)
            Xt = np.where(np.repeat(shrink, sizes), Xbase + alpha_full * S, Xbase).astype(T)
            trial = ev.loss_only(Xt)
            f_calls += shrink
            phix0 = np.where(shrink, phix1, phix0)
            phix1 = np.where(shrink, trial, phix1)

        # accept, new gradient (one launch), BFGS update, convergence (Optim.converged)
        moved = active & np.isfinite(phix1)
        Xn = np.where(np.repeat(moved, sizes), Xbase + np.repeat(a2, sizes) * S, Xbase).astype(T)
        fn, Gn = ev.loss_grad(Xn)
        f_calls += moved
        upd = active & moved & np.isfinite(fn)
        active &= upd
        dx_all = Xn.astype(np.float64) - X.astype(np.float64)
        dg_all = Gn - G
        with np.errstate(invalid="ignore", over="ignore"):
            x_conv = segmax_abs(dx_all) <= 0.0
            f_conv = np.abs(fn - f) <= 0.0
            g_conv = segmax_abs(Gn) <= G_TOL
        with np.errstate(all="ignore"):  # IEEE arithmetic: overflow gives Inf, as in Julia
            for sz, ks in groups.items():
                u = upd[ks]
                if not u.any():
                    continue
                dx, dg = dx_all[gidx[sz]], dg_all[gidx[sz]]
                dxdg = _dot(dx, dg)
                u &= dxdg > 0
                if not u.any():
                    continue
                H = invH[sz][u]
                dxu, dgu, d = dx[u], dg[u], dxdg[u]
                Hdg = _matvec(H, dgu)
                outer_dx = dxu[:, :, None] * dxu[:, None, :]
                coef = (d + _dot(dgu, Hdg)) / (d * d)
                invH[sz][u] = (H + coef[:, None, None] * outer_dx
                               - (Hdg[:, :, None] * dxu[:, None, :] + dxu[:, :, None] * Hdg[:, None, :])
                               / d[:, None, None])
        done = upd & (x_conv | f_conv | g_conv)
        conv |= done
        active &= ~done
        keep = np.repeat(moved, sizes)
        X = np.where(keep, Xn, X).astype(T)
        G = np.where(keep, Gn, G)
        f = np.where(moved & np.isfinite(fn), fn, f)

    xb = [X[off[k]:off[k + 1]] for k in range(nc)]
    _pick_best(flat, cand_tree, f, xb, conv, f_calls, acc, T)


def _make_evaluator(trees, cand_tree, cand_x, factory, repeat=None):
    """The evaluator of the candidates (start k = tree cand_tree[k] with
    constants cand_x[k]); `repeat[k]` copies of each when given."""
    idx = np.asarray(cand_tree) if repeat is None else np.repeat(cand_tree, repeat)
    xs = cand_x if repeat is None else [x for x, r in zip(cand_x, repeat) for _ in range(r)]
    cands = []
    for i, x in zip(idx, xs):
        c = trees[i].copy()
        set_constants(c, list(x))
        cands.append(c)
    return factory(cands)


NM_INITIAL_A, NM_INITIAL_B = 0.025, 0.5  # Optim.AffineSimplexer defaults


def _optimize_nelder_mead(dataset, trees, flat, sel, options, noise, factory, acc):
    """Optim.NelderMead for trees of two or more constants (:35-36), every
    start of every tree in lockstep: the affine initial simplex
    x0 + (a + b·x0_j)·e_j (a = 0.025, b = 0.5), Gao & Han's adaptive
    parameters (α = 1, β = 1 + 2/n, γ = 0.75 - 1/(2n), δ = 1 - 1/n),
    reflection / expansion / outside and inside contraction / shrink,
    convergence when the population standard deviation of the simplex losses
    is <= g_abstol (1e-8), and the final minimiser = the centroid of the best
    n vertices if its loss beats the best vertex."""
    T = np.dtype(dataset.T).type
    iterations = int(getattr(options, "optimizer_iterations", 8))
    nrestarts = int(getattr(options, "optimizer_nrestarts", 2))
    cand_tree, cand_x = _starts(flat, sel, T, nrestarts, noise)
    if not cand_tree:
        return
    nc = len(cand_tree)
    sizes = [x.size for x in cand_x]
    point_ev = _make_evaluator(trees, cand_tree, cand_x, factory)
    simplex_ev = _make_evaluator(trees, cand_tree, cand_x, factory, repeat=[sz + 1 for sz in sizes])

    simplex = []
    for x0 in cand_x:
        v = np.repeat(x0[None, :], x0.size + 1, axis=0).astype(T)
        for j in range(x0.size):
            v[j + 1, j] = T((1.0 + NM_INITIAL_B) * float(v[j + 1, j]) + NM_INITIAL_A)
        simplex.append(v)

    def eval_simplices():
        fl = simplex_ev.loss_only(np.concatenate([v.reshape(-1) for v in simplex]))
        out, o = [], 0
        for k in range(nc):
            out.append(np.asarray(fl[o:o + sizes[k] + 1], dtype=np.float64))
            o += sizes[k] + 1
        return out

    def eval_points(pts):
        return np.asarray(point_ev.loss_only(np.concatenate(pts)), dtype=np.float64)

    def nm_x(fs):  # the population standard deviation, sequential sums
        s = 0.0
        for v in fs:
            s = s + float(v)
        mean = s / len(fs)
        q = 0.0
        for v in fs:
            q = q + (float(v) - mean) * (float(v) - mean)
        return float(np.sqrt(q / len(fs)))

    def centroid(v, h):  # mean of every vertex but h, in vertex order
        rows = [v[i].astype(np.float64) for i in range(v.shape[0]) if i != h]
        m = rows[0].copy()
        for r in rows[1:]:
            m = m + r
        return m / float(len(rows))

    fsx = eval_simplices()
    f_calls = np.array([s + 1.0 for s in sizes])
    order = [np.argsort(f, kind="stable") for f in fsx]
    conv = np.zeros(nc, dtype=bool)
    active = np.ones(nc, dtype=bool)
    params = []
    for n in sizes:
        params.append((1.0, 1.0 + 2.0 / n, 0.75 - 1.0 / (2.0 * n), 1.0 - 1.0 / n))

    for _ in range(iterations):
        if not active.any():
            break
        # 1. reflections
        xc, xh, xr = [None] * nc, [None] * nc, [None] * nc
        for k in range(nc):
            m = sizes[k] + 1
            xc[k] = centroid(simplex[k], order[k][m - 1])
            xh[k] = simplex[k][order[k][m - 1]].astype(np.float64)
            xr[k] = (xc[k] + params[k][0] * (xc[k] - xh[k])).astype(T) if active[k] else simplex[k][0]
        fr = eval_points(xr)
        f_calls += active
        # 2. expansion / contraction points
        second = np.zeros(nc, dtype=int)  # 0 none, 1 expand, 2 outside, 3 inside
        xs = [simplex[k][0] for k in range(nc)]
        shrink = np.zeros(nc, dtype=bool)
        for k in np.nonzero(active)[0]:
            m = sizes[k] + 1
            f, o = fsx[k], order[k]
            al, be, ga, de = params[k]
            xrf = xr[k].astype(np.float64)
            if fr[k] < f[o[0]]:
                second[k], xs[k] = 1, (xc[k] + be * (xrf - xc[k])).astype(T)
            elif fr[k] < f[o[m - 2]]:
                simplex[k][o[m - 1]], f[o[m - 1]] = xr[k], fr[k]
                order[k] = np.argsort(f, kind="stable")
            elif fr[k] < f[o[m - 1]]:
                second[k], xs[k] = 2, (xc[k] + ga * (xrf - xc[k])).astype(T)
            else:
                second[k], xs[k] = 3, (xc[k] - ga * (xrf - xc[k])).astype(T)
        if second.any():
            fs2 = eval_points(xs)
            f_calls += second > 0
            for k in np.nonzero(second)[0]:
                m = sizes[k] + 1
                f, o = fsx[k], order[k]
                h = o[m - 1]
                if second[k] == 1:
                    if fs2[k] < fr[k]:
                        simplex[k][h], f[h] = xs[k], fs2[k]
                    else:
                        simplex[k][h], f[h] = xr[k], fr[k]
                    order[k] = np.concatenate([[h], o[:m - 1]])  # the new vertex is the lowest
                elif (second[k] == 2 and fs2[k] < fr[k]) or (second[k] == 3 and fs2[k] < f[h]):
                    simplex[k][h], f[h] = xs[k], fs2[k]
                    order[k] = np.argsort(f, kind="stable")
                else:
                    shrink[k] = True
        # 3. shrinks towards the lowest vertex: every other vertex re-evaluated
        if shrink.any():
            for k in np.nonzero(shrink)[0]:
                lo = simplex[k][order[k][0]].astype(np.float64)
                de = params[k][3]
                for i in order[k][1:]:
                    simplex[k][i] = (lo + de * (simplex[k][i].astype(np.float64) - lo)).astype(T)
            fall = eval_simplices()
            for k in np.nonzero(shrink)[0]:
                f = fsx[k]
                for i in order[k][1:]:
                    f[i] = fall[k][i]
                f_calls[k] += sizes[k]
                order[k] = np.argsort(f, kind="stable")
        for k in np.nonzero(active)[0]:
            if nm_x(fsx[k]) <= G_TOL:
                conv[k], active[k] = True, False

    # after the loop: the centroid of the best n vertices against the best vertex
    xcen = []
    for k in range(nc):
        order[k] = np.argsort(fsx[k], kind="stable")
        xcen.append(centroid(simplex[k], order[k][-1]).astype(T))
    fcen = eval_points(xcen)
    f_calls += 1
    xmin, fmin = [], np.zeros(nc)
    for k in range(nc):
        i = julia_findmin(fsx[k])
        if fcen[k] < fsx[k][i]:  # False for a NaN minimum: the NaN vertex is kept, as in Optim
            xmin.append(xcen[k])
            fmin[k] = fcen[k]
        else:
            xmin.append(simplex[k][i].copy())
            fmin[k] = fsx[k][i]
    _pick_best(flat, cand_tree, fmin, xmin, conv, f_calls, acc, T)


def julia_findmin(f) -> int:
    """Index Julia's `findmin` picks (Optim's NelderMead after_while!): the
    first NaN if there is one (findmin propagates NaN), else the first
    minimum."""
    f = np.asarray(f)
    nan = np.flatnonzero(np.isnan(f))
    return int(nan[0]) if nan.size else int(np.argmin(f))
