"""CPU model of the tree code's guarded FAST path (no GPU): which trees'
losses leave the north_star's 1e-5 bar when exp / sin / cos are off by an
ulp or two, and which guard rules catch them at what redo cost.

Every tree is evaluated twice in Float32 over the same rows: "precise"
(exp / sin / cos evaluated in Float64 and rounded once: the reference, and
the tree code's PRECISE routines) and "fast" (a stand-in for the FAST
routines: numpy's Float32 SIMD exp / cos / sin, off by up to 2 ulp on 39 % /
17 % / 11 % of arguments, or --noise k: the precise value moved by a random
0..k ulp). Feature-free subtrees are folded (precise, untainted), as the host
compiler does. Guard rules are evaluated on the fast values per row, as the
tree code does; a 256-row tile where any guard fires (or that fails) takes
the precise values. Reports, per rule set: trees outside 1e-5 relative of
the precise loss, and the fraction of (tree, tile) pairs redone.

Usage: python tools/fast_guard_sim.py [--rows N] [--ntrees N] [--seed S] [--noise K]
"""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "symbolicregression.jl_amd")]
import srhip  # noqa: E402

TILE = 256
F32 = np.float32


def ulp_move(v, k, rng):
    if k == 0:
        return v
    d = rng.integers(-k, k + 1, size=v.shape).astype(np.int32)
    b = v.view(np.int32) + d * np.where(v.view(np.int32) < 0, -1, 1).astype(np.int32)
    out = b.view(F32)
    return np.where(np.isfinite(v), out, v)


class Sim:
    def __init__(self, X, y, noise, rng):
        self.X, self.y, self.noise, self.rng = X, y, noise, rng
        self.n = X.shape[1]

    def trans(self, name, a, fast):
        f64 = {"exp": np.exp, "cos": np.cos, "sin": np.sin}[name]
        with np.errstate(all="ignore"):
            p = f64(a.astype(np.float64)).astype(F32)
            if not fast:
                return p
            if self.noise:
                return ulp_move(p, self.noise, self.rng)
            return f64(a).astype(F32)

    def ev(self, nd, opts, zs, guards, rules):
        """-> (vp, vf, taint, const). guards: dict rule -> row mask (fast values)."""
        if nd.degree == 0:
            if nd.constant:
                v = np.full(self.n, F32(nd.val))
                return v, v, False, True
            v = self.X[nd.feature - 1]
            return v, v, False, False
        if nd.degree == 1:
            name = opts.unary_operators[nd.op - 1]
            zs_c = zs and name in ("neg", "abs", "square", "cube", "sin")
            ap, af, at, ac = self.ev(nd.l, opts, zs_c, guards, rules)
            with np.errstate(all="ignore"):
                if name in ("exp", "cos", "sin"):
                    vp = self.trans(name, ap, False)
                    vf = vp if ac else self.trans(name, af, True)
                    taint = not ac
                    for r in rules:
                        r.unary(name, af, vf, at, zs, nd, guards)
                else:
                    fn = {"neg": np.negative, "abs": np.abs, "square": np.square, "cube": lambda a: (a * a) * a}[name]
                    vp, vf, taint = fn(ap), fn(af), at
            return vp, vf, taint, ac
        name = opts.binary_operators[nd.op - 1]
        if name == "/":
            zl, zr = zs, True
        elif name in ("+", "-", "*"):
            zl = zr = zs
        else:
            zl = zr = False
        ap, af, at, ac = self.ev(nd.l, opts, zl, guards, rules)
        bp, bf, bt, bc = self.ev(nd.r, opts, zr, guards, rules)
        fn = {"+": np.add, "-": np.subtract, "*": np.multiply, "/": np.divide}[name]
        with np.errstate(all="ignore"):
            vp, vf = fn(ap, bp), fn(af, bf)
        taint = at or bt
        for r in rules:
            r.binary(name, af, bf, vf, at, bt, zs, guards)
        return vp, vf, taint, ac and bc


class Base:
    """The round-3 guards (jit.cpp analyze / emit_*)."""
    name = "r3"

    def unary(self, name, a, v, at, zs, nd, g):
        if name == "exp":
            self.fire(g, "exp87", ~(np.abs(a) <= 87))
        if name in ("cos", "sin") and at and zs:
            self.fire(g, "trig14", ~(np.abs(a) <= 2.0 ** 14))

    def binary(self, name, a, b, v, at, bt, zs, g):
        if not (at or bt) or not zs:
            return
        if name in ("+", "-"):
            self.fire(g, "can", ~(np.abs(v) > 2.0 ** -14 * (np.abs(a) + np.abs(b))))
        if name in ("*", "/"):
            self.fire(g, "min", ~(np.abs(v) >= 2.0 ** -120))

    @staticmethod
    def fire(g, k, m):
        g[k] = m if k not in g else (g[k] | m)


def run_tree(sim, tree, opts, rules):
    guards = {}
    vp, vf, taint, const = sim.ev(tree, opts, False, guards, rules)
    n = sim.n
    nt = (n + TILE - 1) // TILE
    pad = nt * TILE - n
    with np.errstate(all="ignore"):
        rp = (vp.astype(np.float64) - sim.y) ** 2
        rf = (vf.astype(np.float64) - sim.y) ** 2
    okp = np.isfinite(vp)
    if not okp.all():
        return None  # the reference fails the tree: did_succeed decides, no loss
    fire = ~np.isfinite(vf)
    for m in guards.values():
        fire = fire | m
    fire_t = np.pad(fire, (0, pad)).reshape(nt, TILE).any(1)
    rows_fire = np.repeat(fire_t, TILE)[:n]
    res = np.where(rows_fire, rp, rf)
    Lp, Le = rp.sum(), res.sum()
    rel = abs(Le - Lp) / abs(Lp) if Lp != 0 else abs(Le)
    per_rule = {k: float(np.pad(m, (0, pad)).reshape(nt, TILE).any(1).mean()) for k, m in guards.items()}
    # cost model (FAST tile 1, PRECISE tile P): calls of CALL tiles; once a
    # tile of a call is redone, the call's later tiles run PRECISE directly
    P, CALL = 1.7, 4
    nc = (nt + CALL - 1) // CALL
    ft = np.pad(fire_t, (0, nc * CALL - nt)).reshape(nc, CALL)
    before = np.cumsum(ft, axis=1) - ft > 0  # an earlier tile of the call was redone
    cost_adapt = float(np.where(before, P, 1 + ft * P).sum() / (nc * CALL))
    cost_plain = float((1 + ft * P).sum() / (nc * CALL))
    return rel, float(fire_t.mean()), per_rule, cost_plain, cost_adapt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=262144)
    ap.add_argument("--ntrees", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--noise", type=int, default=0)
    ap.add_argument("--rules", default="r3")
    ap.add_argument("--show", type=int, default=15)
    ap.add_argument("--kc", type=float)
    ap.add_argument("--kt", type=float)
    ap.add_argument("--te", type=float)
    ap.add_argument("--tt", type=float)
    a = ap.parse_args()
    o = srhip.Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    trees = srhip.random_population(a.ntrees, o, 5, np.float32, seed=a.seed)
    rng = np.random.default_rng(1)
    X = rng.standard_normal((5, 1_000_000)).astype(F32)[:, :a.rows].copy()
    y = (F32(2) * np.cos(X[3]) + X[0] * X[0] - F32(2)).astype(F32).astype(np.float64)
    sim = Sim(X, y, a.noise, np.random.default_rng(7))
    rules = [RULES[r]() for r in a.rules.split(",")]
    for r in rules:
        for k in ("KC", "KT", "TE", "TT"):
            v = getattr(a, k.lower(), None)
            if v is not None:
                setattr(r, k, v)
    out, redo, rule_cost, ok, costs = [], [], {}, 0, []
    for i, t in enumerate(trees):
        r = run_tree(sim, t, o, rules)
        if r is None:
            continue
        ok += 1
        rel, fr, pr, cp, ca = r
        redo.append(fr)
        costs.append((cp, ca))
        for k, v in pr.items():
            rule_cost[k] = rule_cost.get(k, 0.0) + v
        if not rel <= 1e-5:
            out.append((rel, i, fr))
    out.sort(reverse=True)
    print(f"rules {a.rules} {[(k, getattr(rules[0], k, None)) for k in ('KC', 'KT', 'TE', 'TT')]} noise {a.noise}: {ok} succeeding trees, {len(out)} outside 1e-5; "
          f"tiles redone {np.mean(redo):.4%}; by rule " +
          ", ".join(f"{k} {v / max(ok, 1):.4%}" for k, v in sorted(rule_cost.items())))
    rd = np.asarray(redo)
    cs = np.asarray(costs)
    print(f"  per-tree redo fraction: =0 {np.mean(rd == 0):.3f}, <5% {np.mean(rd < .05):.3f}, >50% {np.mean(rd > .5):.3f}, "
          f">90% {np.mean(rd > .9):.3f}; cost vs all-FAST (PRECISE 1.7x): plain {cs[:, 0].mean():.4f}, "
          f"rest-of-call PRECISE after a redo {cs[:, 1].mean():.4f}; all PRECISE 1.7")
    for rel, i, fr in out[:a.show]:
        print(f"  tree {i}: rel {rel:.3g}, redo {fr:.3f}: {srhip.string_tree(trees[i], o)}")


class V4(Base):
    """Candidate round-4 rules (parameters from the environment of main):
    the zs-path cancellation guard at 2^-KC, |sin/cos(u)| below 2^-KT·max(1,|u|)
    for a FAST-derived u on a zs path, |u| > TE at exp of a FAST-derived u,
    |u| > TT at sin / cos of a FAST-derived u anywhere."""
    name = "v4"
    KC, KT, TE, TT = 14, 8, 16.0, 64.0

    def unary(self, name, a, v, at, zs, nd, g):
        Base.unary(self, name, a, v, at, zs, nd, g)
        if not at:
            return
        if name == "exp":
            self.fire(g, "exp_arg", ~(np.abs(a) <= self.TE))
        if name in ("cos", "sin"):
            self.fire(g, "trig_arg", ~(np.abs(a) <= self.TT))
            if zs:
                self.fire(g, "trig_small", ~(np.abs(v) > 2.0 ** -self.KT * np.maximum(1, np.abs(a))))

    def binary(self, name, a, b, v, at, bt, zs, g):
        if not (at or bt) or not zs:
            return
        if name in ("+", "-"):
            self.fire(g, "can", ~(np.abs(v) > 2.0 ** -self.KC * (np.abs(a) + np.abs(b))))
        if name in ("*", "/"):
            self.fire(g, "min", ~(np.abs(v) >= 2.0 ** -120))


RULES = {"r3": Base, "v4": V4}

if __name__ == "__main__":
    main()
