// constopt.cpp — the lockstep constant optimiser behind
// srhip_optimize_constants_batch / _cb (include/srhip.h); see constopt.h.
//
// Reference: optimize_constants, src/ConstantOptimization.jl:22-65 — Newton
// for one constant, else BFGS (or NelderMead, :35-36), both with
// LineSearches.BackTracking; `optimizer_iterations` iterations from x0 and
// `optimizer_nrestarts` starts x0 .* (1 .+ randn/2) (:46-54); the best run is
// kept only if Optim reports convergence, else x0 stays (:56-63). Optim and
// LineSearches are not vendored in the reference: their published algorithms
// are restated (Nocedal & Wright §3.5 for the backtracking interpolation,
// Gao & Han's adaptive Nelder-Mead parameters, Optim's AffineSimplexer).
// Deliberate deviations, as in the checker: analytic gradients instead of
// finite differences; Newton's Hessian by a central difference of the
// gradient (made positive as PositiveFactorizations does for 1×1); the line
// search capped at 60 shrinks (a step below 2^-60 of the direction no longer
// moves x); f_calls counts loss evaluations (loss + gradient once).
//
// Built with -ffp-contract=off: every sum and product is rounded as the
// checker's numpy does, so trajectories agree bit for bit.
#include "constopt.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <limits>
#include <map>
#include <random>
#include <stdexcept>

#include "../../include/srhip.h"
#include "compile.h"

namespace srhip {
namespace copt {
namespace {

constexpr double G_TOL = 1e-8;                   // Optim.Options g_abstol
constexpr double C1 = 1e-4, RHO_HI = 0.5, RHO_LO = 0.1;  // BackTracking defaults
constexpr int LS_ITERATIONS = 60;
constexpr int SUBSET_FRACTION = 10;              // stragglers below 1/10 get a set of their own
constexpr double NM_A = 0.025, NM_B = 0.5;       // Optim.AffineSimplexer defaults
const double kInf = std::numeric_limits<double>::infinity();
const double kNaN = std::numeric_limits<double>::quiet_NaN();

struct Num {
  bool f32;
  double rt(double v) const { return f32 ? (double)(float)v : v; }
  double eps() const { return f32 ? (double)FLT_EPSILON : DBL_EPSILON; }
  double cbrt_eps() const { return f32 ? (double)cbrtf(FLT_EPSILON) : std::cbrt(DBL_EPSILON); }
  int log2_eps() const { return f32 ? 23 : 52; }
  // x0 .* (1 .+ randn(T)/2) in T (:47)
  double perturb(double x0, double n) const {
    if (f32) {
      float t = 0.5f * (float)n;
      t = 1.0f + t;
      return (double)((float)x0 * t);
    }
    double t = 0.5 * n;
    t = 1.0 + t;
    return x0 * t;
  }
};

// the candidates: x0 and the perturbed starts of every selected tree with constants
struct Cands {
  std::vector<int32_t> tree;
  std::vector<int64_t> off{0};
  std::vector<double> x;
  int nc() const { return (int)tree.size(); }
  int size(int k) const { return (int)(off[k + 1] - off[k]); }
  void add(int32_t t, const double* v, int n) {
    tree.push_back(t);
    x.insert(x.end(), v, v + n);
    off.push_back((int64_t)x.size());
  }
};

Cands make_starts(const Problem& pb, const std::vector<int>& sel, int nrestarts, const std::vector<double>& noise,
                  const Num& num) {
  Cands c;
  std::vector<double> tmp;
  for (int i : sel) {
    const int64_t a = pb.const_off[i], n = pb.const_off[i + 1] - a;
    if (n == 0) continue;
    c.add(i, &pb.consts[a], (int)n);
    for (int r = 0; r < nrestarts; ++r) {
      tmp.resize(n);
      const double* z = &noise[(size_t)nrestarts * a + (size_t)r * n];
      for (int64_t j = 0; j < n; ++j) tmp[j] = num.perturb(pb.consts[a + j], z[j]);
      c.add(i, tmp.data(), (int)n);
    }
  }
  return c;
}

double seg_max_abs(const std::vector<double>& v, int64_t a, int64_t b) {
  double m = std::fabs(v[a]);
  for (int64_t j = a + 1; j < b; ++j) {
    const double x = std::fabs(v[j]);
    m = (std::isnan(m) || std::isnan(x)) ? kNaN : std::max(m, x);
  }
  return m;
}

// One BackTracking shrink (LineSearches.jl order 3): quadratic interpolation
// on the first shrink, cubic after, safeguarded to [ρ_lo·α, ρ_hi·α]
double backtrack(double a1, double a2, double phi0, double dphi0, double phix0, double phix1, bool first) {
  double at;
  if (first) {
    const double den = 2.0 * (phix1 - phi0 - dphi0 * a2);
    at = den != 0.0 ? -(dphi0 * a2 * a2) / den : kNaN;
  } else {
    const double div = 1.0 / (a1 * a1 * a2 * a2 * (a2 - a1));
    const double r1 = phix1 - phi0 - dphi0 * a2;
    const double r0 = phix0 - phi0 - dphi0 * a1;
    const double a = (a1 * a1 * r1 - a2 * a2 * r0) * div;
    const double b = (-std::pow(a1, 3.0) * r1 + std::pow(a2, 3.0) * r0) * div;
    if (std::fabs(a) <= 1e-12 * std::max(1.0, std::fabs(b))) {
      at = b != 0.0 ? dphi0 / (2.0 * b) : kNaN;
    } else {
      const double d = std::max(b * b - 3.0 * a * dphi0, 0.0);
      at = (-b + std::sqrt(d)) / (3.0 * a);
    }
  }
  const double hi = a2 * RHO_HI, lo = a2 * RHO_LO;
  at = std::isfinite(at) ? std::min(at, hi) : hi;  // NaNMath.min
  return std::max(at, lo);
}

struct Acc {  // per input tree
  std::vector<double>& num_evals;
  std::vector<uint8_t>& converged;
  std::vector<double>& consts;
};

// the best start of every tree (:51-53), kept if it converged (:56-63)
void pick_best(const Problem& pb, const Cands& c, const std::vector<double>& fbest,
               const std::vector<std::vector<double>>& xbest, const std::vector<uint8_t>& conv,
               const std::vector<double>& f_calls, Acc& acc) {
  std::map<int, int> best;
  for (int k = 0; k < c.nc(); ++k) {
    const int i = c.tree[k];
    acc.num_evals[i] += f_calls[k];
    auto it = best.find(i);
    if (it == best.end()) best[i] = k;
    else if (fbest[k] < fbest[it->second]) it->second = k;
  }
  for (const auto& [i, k] : best) {
    if (!conv[k]) continue;
    const int64_t a = pb.const_off[i];
    for (size_t j = 0; j < xbest[k].size(); ++j) acc.consts[a + j] = xbest[k][j];
    acc.converged[i] = 1;
    acc.num_evals[i] += 1;
  }
}

// BFGS (Newton for one constant) with BackTracking, every start in lockstep
void run_gradient(const Problem& pb, const std::vector<int>& sel, const Options& opt, const std::vector<double>& noise,
                  const Num& num, Factory& fac, Acc& acc) {
  Cands c = make_starts(pb, sel, opt.nrestarts, noise, num);
  const int nc = c.nc();
  if (nc == 0) return;
  std::unique_ptr<Set> ev = fac.make(c.tree);
  const int64_t nx = c.off[nc];
  std::vector<double> X(c.x.size());
  for (int64_t j = 0; j < nx; ++j) X[j] = num.rt(c.x[j]);
  std::vector<double> f_calls(nc, 0.0);
  std::vector<std::vector<double>> invH(nc);
  for (int k = 0; k < nc; ++k) {
    const int sz = c.size(k);
    if (sz > 1) {
      invH[k].assign((size_t)sz * sz, 0.0);
      for (int i = 0; i < sz; ++i) invH[k][(size_t)i * sz + i] = 1.0;
    }
  }
  std::vector<double> f, G;
  ev->eval(X, true, f, G);
  for (int k = 0; k < nc; ++k) f_calls[k] += 1;
  std::vector<uint8_t> active(nc), conv(nc);
  for (int k = 0; k < nc; ++k) {
    active[k] = std::isfinite(f[k]);
    conv[k] = active[k] && seg_max_abs(G, c.off[k], c.off[k + 1]) <= G_TOL;  // converged at x0
    if (conv[k]) active[k] = 0;
  }
  auto any = [](const std::vector<uint8_t>& v) { return std::find(v.begin(), v.end(), 1) != v.end(); };
  std::vector<double> S(nx), dphi0(nc), a1(nc), a2(nc), phix0(nc), phix1(nc), Xbase(nx), Xt(nx), trial, fn, Gn,
      Gp, Gm, fdum;
  std::vector<uint8_t> searching(nc), first(nc), moved(nc), upd(nc);
  std::vector<int> finite_left(nc), ls_iter(nc);
  std::vector<double> sd, gv, Hdg;
  // Newton's central differences need ∂L/∂c of the one-constant candidates
  // only: when they are a minority, a set of just them (built once, at the
  // first Newton step, with every one-constant candidate) takes those two
  // gradient calls per iteration instead of the whole set
  std::unique_ptr<Set> nev;
  std::vector<int> newton_ks;
  std::vector<double> nx_p, nx_m, nf, nGp, nGm;
  for (int it = 0; it < opt.iterations; ++it) {
    if (!any(active)) break;
    // search directions
    std::fill(S.begin(), S.end(), 0.0);
    bool any_newton = false;
    for (int k = 0; k < nc; ++k) any_newton = any_newton || (c.size(k) == 1 && active[k]);
    if (any_newton) {
      std::vector<double> Xp(X), Xm(X), step(nc, 0.0);
      for (int k = 0; k < nc; ++k) {
        if (!(c.size(k) == 1 && active[k])) continue;
        step[k] = num.cbrt_eps() * std::max(1.0, std::fabs(X[c.off[k]]));
        Xp[c.off[k]] += step[k];
        Xm[c.off[k]] -= step[k];
      }
      for (int64_t j = 0; j < nx; ++j) { Xp[j] = num.rt(Xp[j]); Xm[j] = num.rt(Xm[j]); }
      if (!nev && fac.has_subset()) {
        std::vector<int32_t> mem;
        for (int k = 0; k < nc; ++k)
          if (c.size(k) == 1) newton_ks.push_back(k);
        if ((int64_t)newton_ks.size() * 2 < nc) {
          for (int k : newton_ks) mem.push_back(c.tree[k]);
          nev = fac.make(mem);
        } else {
          newton_ks.clear();
        }
      }
      if (nev) {
        const size_t nn = newton_ks.size();
        nx_p.resize(nn);
        nx_m.resize(nn);
        for (size_t q = 0; q < nn; ++q) {
          nx_p[q] = Xp[c.off[newton_ks[q]]];
          nx_m[q] = Xm[c.off[newton_ks[q]]];
        }
        nev->eval(nx_p, true, nf, nGp);
        nev->eval(nx_m, true, nf, nGm);
        Gp.assign(nx, 0.0);
        Gm.assign(nx, 0.0);
        for (size_t q = 0; q < nn; ++q) {
          Gp[c.off[newton_ks[q]]] = nGp[q];
          Gm[c.off[newton_ks[q]]] = nGm[q];
        }
      } else {
        ev->eval(Xp, true, fdum, Gp);
        ev->eval(Xm, true, fdum, Gm);
      }
      for (int k = 0; k < nc; ++k) {
        if (!(c.size(k) == 1 && active[k])) continue;
        const int64_t s0 = c.off[k];
        const double h = (Gp[s0] - Gm[s0]) / (2.0 * step[k]);
        const double hk = (std::isfinite(h) && std::fabs(h) > num.eps()) ? std::fabs(h) : 1.0;
        S[s0] = -G[s0] / hk;
      }
    }
    for (int k = 0; k < nc; ++k) {
      const int sz = c.size(k);
      if (sz <= 1 || !active[k]) continue;
      const int64_t s0 = c.off[k];
      std::vector<double>& H = invH[k];
      sd.assign(sz, 0.0);
      for (int i = 0; i < sz; ++i) {
        double acc_ = 0.0;
        for (int j = 0; j < sz; ++j) acc_ += H[(size_t)i * sz + j] * G[s0 + j];
        sd[i] = -acc_;
      }
      double gs = 0.0;
      for (int i = 0; i < sz; ++i) gs += G[s0 + i] * sd[i];
      if (!(gs < 0.0)) {  // not a descent direction: restart from the identity
        std::fill(H.begin(), H.end(), 0.0);
        for (int i = 0; i < sz; ++i) H[(size_t)i * sz + i] = 1.0;
        for (int i = 0; i < sz; ++i) sd[i] = -G[s0 + i];
      }
      for (int i = 0; i < sz; ++i) S[s0 + i] = sd[i];
    }
    for (int k = 0; k < nc; ++k) {
      double d = 0.0;
      if (active[k]) {
        for (int64_t j = c.off[k]; j < c.off[k + 1]; ++j) d += G[j] * S[j];
      }
      dphi0[k] = d;
      // a NaN gradient (or no descent at all) ends the run: Optim's x would turn NaN
      active[k] = active[k] && std::isfinite(d) && d < 0.0;
    }

    // BackTracking line search, all candidates in lockstep
    Xbase = X;
    for (int k = 0; k < nc; ++k) {
      a1[k] = a2[k] = 1.0;
      phix0[k] = f[k];
      searching[k] = active[k];
      first[k] = 1;
      ls_iter[k] = 0;
      finite_left[k] = searching[k] ? num.log2_eps() : 0;
    }
    for (int64_t j = 0; j < nx; ++j) Xt[j] = num.rt(Xbase[j] + S[j]);
    ev->eval(Xt, false, trial, fdum);
    for (int k = 0; k < nc; ++k) {
      f_calls[k] += searching[k];
      phix1[k] = searching[k] ? trial[k] : f[k];
    }
    std::unique_ptr<Set> sev;
    std::vector<int> sub_ks;
    std::vector<int64_t> sub_pos;
    // the candidates still searching: a candidate that stops never resumes,
    // and one that does not shrink only has its trial point reset to x
    std::vector<int> live;
    for (int k = 0; k < nc; ++k)
      if (searching[k]) live.push_back(k);
    std::vector<uint8_t> shrink(nc, 0);
    for (;;) {
      bool any_shrink = false;
      int nshrink = 0;
      for (int k : live) {
        const bool fin = std::isfinite(phix1[k]);
        const bool halve = searching[k] && !fin && finite_left[k] > 0;  // halve until the loss is finite
        bool s = searching[k] && (fin || halve);
        const bool armijo = s && fin && (phix1[k] <= f[k] + C1 * a2[k] * dphi0[k]);
        s = s && !armijo;
        const bool failed = s && fin && ls_iter[k] >= LS_ITERATIONS;  // a failed line search stays at x
        s = s && !failed;
        searching[k] = s;
        if (failed) phix1[k] = kInf;
        const bool step = s && fin;
        if (halve) finite_left[k] -= 1;
        if (step) ls_iter[k] += 1;
        shrink[k] = halve || step;
        if (shrink[k]) {
          const double at = step ? backtrack(a1[k], a2[k], f[k], dphi0[k], phix0[k], phix1[k], first[k]) : 0.0;
          a1[k] = a2[k];
          a2[k] = halve ? a2[k] * 0.5 : at;
        }
        if (step) first[k] = 0;
        any_shrink = any_shrink || shrink[k];
        nshrink += shrink[k];
      }
      if (!any_shrink) break;
      for (int k : live)
        for (int64_t j = c.off[k]; j < c.off[k + 1]; ++j)
          Xt[j] = num.rt(shrink[k] ? Xbase[j] + a2[k] * S[j] : Xbase[j]);
      if (!sev && fac.has_subset() && (int64_t)nshrink * SUBSET_FRACTION < nc) {
        // the stragglers (a line search that keeps shrinking) continue on their own set
        std::vector<int32_t> mem;
        for (int k : live)
          if (shrink[k]) {
            sub_ks.push_back(k);
            mem.push_back(c.tree[k]);
            for (int64_t j = c.off[k]; j < c.off[k + 1]; ++j) sub_pos.push_back(j);
          }
        sev = fac.make(mem);
      }
      if (sev) {
        std::vector<double> xs(sub_pos.size()), ts;
        for (size_t q = 0; q < sub_pos.size(); ++q) xs[q] = Xt[sub_pos[q]];
        sev->eval(xs, false, ts, fdum);
        trial.assign(nc, kInf);
        for (size_t q = 0; q < sub_ks.size(); ++q) trial[sub_ks[q]] = ts[q];
      } else {
        ev->eval(Xt, false, trial, fdum);
      }
      for (int k : live) {
        f_calls[k] += shrink[k];
        if (shrink[k]) {
          phix0[k] = phix1[k];
          phix1[k] = trial[k];
        }
      }
      // who did not shrink this round has stopped searching
      size_t w = 0;
      for (int k : live)
        if (shrink[k]) live[w++] = k;
      live.resize(w);
    }

    // accept, the new gradient (one evaluation), BFGS update, convergence (Optim.converged)
    std::vector<double> Xn(nx);
    for (int k = 0; k < nc; ++k) {
      moved[k] = active[k] && std::isfinite(phix1[k]);
      for (int64_t j = c.off[k]; j < c.off[k + 1]; ++j) Xn[j] = num.rt(moved[k] ? Xbase[j] + a2[k] * S[j] : Xbase[j]);
    }
    ev->eval(Xn, true, fn, Gn);
    for (int k = 0; k < nc; ++k) {
      f_calls[k] += moved[k];
      upd[k] = active[k] && moved[k] && std::isfinite(fn[k]);
      active[k] = active[k] && upd[k];
    }
    for (int k = 0; k < nc; ++k) {
      const int sz = c.size(k);
      const int64_t s0 = c.off[k];
      double xmax = 0.0, gmax = 0.0;
      {
        std::vector<double> dx(sz), gn(sz);
        for (int i = 0; i < sz; ++i) { dx[i] = Xn[s0 + i] - X[s0 + i]; gn[i] = Gn[s0 + i]; }
        xmax = seg_max_abs(dx, 0, sz);
        gmax = seg_max_abs(gn, 0, sz);
      }
      const bool x_conv = xmax <= 0.0, f_conv = std::fabs(fn[k] - f[k]) <= 0.0, g_conv = gmax <= G_TOL;
      if (sz > 1 && upd[k]) {
        std::vector<double> dx(sz), dg(sz);
        for (int i = 0; i < sz; ++i) { dx[i] = Xn[s0 + i] - X[s0 + i]; dg[i] = Gn[s0 + i] - G[s0 + i]; }
        double d = 0.0;
        for (int i = 0; i < sz; ++i) d += dx[i] * dg[i];
        if (d > 0.0) {
          std::vector<double>& H = invH[k];
          Hdg.assign(sz, 0.0);
          for (int i = 0; i < sz; ++i) {
            double a_ = 0.0;
            for (int j = 0; j < sz; ++j) a_ += H[(size_t)i * sz + j] * dg[j];
            Hdg[i] = a_;
          }
          double dgHdg = 0.0;
          for (int i = 0; i < sz; ++i) dgHdg += dg[i] * Hdg[i];
          const double coef = (d + dgHdg) / (d * d);
          for (int i = 0; i < sz; ++i)
            for (int j = 0; j < sz; ++j) {
              const double outer = dx[i] * dx[j];
              H[(size_t)i * sz + j] = H[(size_t)i * sz + j] + coef * outer - (Hdg[i] * dx[j] + dx[i] * Hdg[j]) / d;
            }
        }
      }
      if (upd[k] && (x_conv || f_conv || g_conv)) {
        conv[k] = 1;
        active[k] = 0;
      }
    }
    for (int k = 0; k < nc; ++k) {
      if (moved[k])
        for (int64_t j = c.off[k]; j < c.off[k + 1]; ++j) { X[j] = Xn[j]; G[j] = Gn[j]; }
      if (moved[k] && std::isfinite(fn[k])) f[k] = fn[k];
    }
  }
  std::vector<std::vector<double>> xb(nc);
  for (int k = 0; k < nc; ++k) xb[k].assign(X.begin() + c.off[k], X.begin() + c.off[k + 1]);
  pick_best(pb, c, f, xb, conv, f_calls, acc);
}

// argsort, stable, NaN last (numpy)
std::vector<int> argsort(const std::vector<double>& f) {
  std::vector<int> o(f.size());
  for (size_t i = 0; i < o.size(); ++i) o[i] = (int)i;
  std::stable_sort(o.begin(), o.end(), [&](int a, int b) {
    const double x = f[a], y = f[b];
    if (std::isnan(x)) return false;
    if (std::isnan(y)) return true;
    return x < y;
  });
  return o;
}
// Julia's findmin: the first NaN if any, else the first minimum
int julia_findmin(const std::vector<double>& f) {
  for (size_t i = 0; i < f.size(); ++i)
    if (std::isnan(f[i])) return (int)i;
  int b = 0;
  for (size_t i = 1; i < f.size(); ++i)
    if (f[i] < f[b]) b = (int)i;
  return b;
}

// Optim.NelderMead for trees of two or more constants (:35-36), every start in
// lockstep: the affine initial simplex, Gao-Han adaptive parameters,
// reflection / expansion / outside and inside contraction / shrink, convergence
// when the simplex losses' population standard deviation is <= 1e-8, and the
// final minimiser = the centroid of the best n vertices if it beats the best
// vertex. Evaluations per iteration: reflections, expansion / contraction
// points, shrinks (all vertices of every simplex).
void run_nelder_mead(const Problem& pb, const std::vector<int>& sel, const Options& opt,
                     const std::vector<double>& noise, const Num& num, Factory& fac, Acc& acc) {
  Cands c = make_starts(pb, sel, opt.nrestarts, noise, num);
  const int nc = c.nc();
  if (nc == 0) return;
  std::vector<int32_t> rep;
  for (int k = 0; k < nc; ++k)
    for (int v = 0; v <= c.size(k); ++v) rep.push_back(c.tree[k]);
  std::unique_ptr<Set> point_ev = fac.make(c.tree), simplex_ev = fac.make(rep);
  // simplex[k]: (n+1) x n vertices, row-major, values of T
  std::vector<std::vector<double>> simplex(nc), fsx(nc);
  for (int k = 0; k < nc; ++k) {
    const int n = c.size(k);
    simplex[k].resize((size_t)(n + 1) * n);
    for (int v = 0; v <= n; ++v)
      for (int j = 0; j < n; ++j) simplex[k][(size_t)v * n + j] = num.rt(c.x[c.off[k] + j]);
    for (int j = 0; j < n; ++j) {
      double& e = simplex[k][(size_t)(j + 1) * n + j];
      e = num.rt((1.0 + NM_B) * e + NM_A);
    }
  }
  std::vector<double> fdum;
  auto eval_simplices = [&]() {
    std::vector<double> X, fl;
    for (int k = 0; k < nc; ++k) X.insert(X.end(), simplex[k].begin(), simplex[k].end());
    simplex_ev->eval(X, false, fl, fdum);
    std::vector<std::vector<double>> out(nc);
    size_t o = 0;
    for (int k = 0; k < nc; ++k) {
      out[k].assign(fl.begin() + o, fl.begin() + o + c.size(k) + 1);
      o += c.size(k) + 1;
    }
    return out;
  };
  auto eval_points = [&](const std::vector<std::vector<double>>& pts) {
    std::vector<double> X, fl;
    for (const auto& p : pts) X.insert(X.end(), p.begin(), p.end());
    point_ev->eval(X, false, fl, fdum);
    return fl;
  };
  auto vertex = [&](int k, int v) {
    const int n = c.size(k);
    return std::vector<double>(simplex[k].begin() + (size_t)v * n, simplex[k].begin() + (size_t)(v + 1) * n);
  };
  auto set_vertex = [&](int k, int v, const std::vector<double>& x) {
    const int n = c.size(k);
    std::copy(x.begin(), x.end(), simplex[k].begin() + (size_t)v * n);
  };
  auto centroid = [&](int k, int h) {  // mean of every vertex but h, in vertex order
    const int n = c.size(k);
    std::vector<double> m(n, 0.0);
    bool firstv = true;
    for (int v = 0; v <= n; ++v) {
      if (v == h) continue;
      for (int j = 0; j < n; ++j) m[j] = firstv ? simplex[k][(size_t)v * n + j] : m[j] + simplex[k][(size_t)v * n + j];
      firstv = false;
    }
    for (int j = 0; j < n; ++j) m[j] = m[j] / (double)n;
    return m;
  };
  auto nm_x = [&](const std::vector<double>& fs) {  // population standard deviation
    double s = 0.0;
    for (double v : fs) s += v;
    const double mean = s / (double)fs.size();
    double q = 0.0;
    for (double v : fs) q += (v - mean) * (v - mean);
    return std::sqrt(q / (double)fs.size());
  };
  auto rt_vec = [&](std::vector<double> v) {
    for (double& e : v) e = num.rt(e);
    return v;
  };

  fsx = eval_simplices();
  std::vector<double> f_calls(nc);
  std::vector<std::vector<int>> order(nc);
  std::vector<uint8_t> conv(nc, 0), active(nc, 1);
  struct P { double al, be, ga, de; };
  std::vector<P> par(nc);
  for (int k = 0; k < nc; ++k) {
    const double n = c.size(k);
    f_calls[k] = n + 1.0;
    order[k] = argsort(fsx[k]);
    par[k] = {1.0, 1.0 + 2.0 / n, 0.75 - 1.0 / (2.0 * n), 1.0 - 1.0 / n};
  }
  for (int it = 0; it < opt.iterations; ++it) {
    if (std::find(active.begin(), active.end(), 1) == active.end()) break;
    // 1. reflections
    std::vector<std::vector<double>> xc(nc), xr(nc);
    for (int k = 0; k < nc; ++k) {
      const int m = c.size(k) + 1;
      if (active[k]) {
        xc[k] = centroid(k, order[k][m - 1]);
        const std::vector<double> xh = vertex(k, order[k][m - 1]);
        std::vector<double> r(xc[k].size());
        for (size_t j = 0; j < r.size(); ++j) r[j] = xc[k][j] + par[k].al * (xc[k][j] - xh[j]);
        xr[k] = rt_vec(r);
      } else {
        xc[k] = centroid(k, order[k][m - 1]);
        xr[k] = vertex(k, 0);
      }
    }
    const std::vector<double> fr = eval_points(xr);
    for (int k = 0; k < nc; ++k) f_calls[k] += active[k];
    // 2. expansion / contraction points
    std::vector<int> second(nc, 0);  // 0 none, 1 expand, 2 outside, 3 inside
    std::vector<std::vector<double>> xs(nc);
    std::vector<uint8_t> shrink(nc, 0);
    for (int k = 0; k < nc; ++k) xs[k] = vertex(k, 0);
    for (int k = 0; k < nc; ++k) {
      if (!active[k]) continue;
      const int m = c.size(k) + 1;
      std::vector<double>& f = fsx[k];
      const std::vector<int>& o = order[k];
      const P& p = par[k];
      auto pt = [&](double coef) {
        std::vector<double> r(xc[k].size());
        for (size_t j = 0; j < r.size(); ++j) r[j] = xc[k][j] + coef * (xr[k][j] - xc[k][j]);
        return rt_vec(r);
      };
      if (fr[k] < f[o[0]]) {
        second[k] = 1;
        xs[k] = pt(p.be);
      } else if (fr[k] < f[o[m - 2]]) {
        set_vertex(k, o[m - 1], xr[k]);
        f[o[m - 1]] = fr[k];
        order[k] = argsort(f);
      } else if (fr[k] < f[o[m - 1]]) {
        second[k] = 2;
        xs[k] = pt(p.ga);
      } else {
        second[k] = 3;
        std::vector<double> r(xc[k].size());
        for (size_t j = 0; j < r.size(); ++j) r[j] = xc[k][j] - p.ga * (xr[k][j] - xc[k][j]);
        xs[k] = rt_vec(r);
      }
    }
    if (std::any_of(second.begin(), second.end(), [](int s) { return s > 0; })) {
      const std::vector<double> fs2 = eval_points(xs);
      for (int k = 0; k < nc; ++k) {
        if (!second[k]) continue;
        f_calls[k] += 1;
        const int m = c.size(k) + 1;
        std::vector<double>& f = fsx[k];
        const std::vector<int> o = order[k];
        const int h = o[m - 1];
        if (second[k] == 1) {
          if (fs2[k] < fr[k]) { set_vertex(k, h, xs[k]); f[h] = fs2[k]; }
          else { set_vertex(k, h, xr[k]); f[h] = fr[k]; }
          std::vector<int> no{h};  // the new vertex is the lowest
          no.insert(no.end(), o.begin(), o.begin() + (m - 1));
          order[k] = no;
        } else if ((second[k] == 2 && fs2[k] < fr[k]) || (second[k] == 3 && fs2[k] < f[h])) {
          set_vertex(k, h, xs[k]);
          f[h] = fs2[k];
          order[k] = argsort(f);
        } else {
          shrink[k] = 1;
        }
      }
    }
    // 3. shrinks towards the lowest vertex: every other vertex re-evaluated
    if (std::find(shrink.begin(), shrink.end(), 1) != shrink.end()) {
      for (int k = 0; k < nc; ++k) {
        if (!shrink[k]) continue;
        const int n = c.size(k);
        const std::vector<double> lo = vertex(k, order[k][0]);
        for (size_t q = 1; q < order[k].size(); ++q) {
          const int v = order[k][q];
          for (int j = 0; j < n; ++j) {
            double& e = simplex[k][(size_t)v * n + j];
            e = num.rt(lo[j] + par[k].de * (e - lo[j]));
          }
        }
      }
      const std::vector<std::vector<double>> fall = eval_simplices();
      for (int k = 0; k < nc; ++k) {
        if (!shrink[k]) continue;
        for (size_t q = 1; q < order[k].size(); ++q) fsx[k][order[k][q]] = fall[k][order[k][q]];
        f_calls[k] += c.size(k);
        order[k] = argsort(fsx[k]);
      }
    }
    for (int k = 0; k < nc; ++k)
      if (active[k] && nm_x(fsx[k]) <= G_TOL) { conv[k] = 1; active[k] = 0; }
  }
  // the centroid of the best n vertices against the best vertex
  std::vector<std::vector<double>> xcen(nc);
  for (int k = 0; k < nc; ++k) {
    order[k] = argsort(fsx[k]);
    xcen[k] = rt_vec(centroid(k, order[k].back()));
  }
  const std::vector<double> fcen = eval_points(xcen);
  std::vector<double> fmin(nc);
  std::vector<std::vector<double>> xmin(nc);
  for (int k = 0; k < nc; ++k) {
    f_calls[k] += 1;
    const int i = julia_findmin(fsx[k]);
    if (fcen[k] < fsx[k][i]) {  // false for a NaN minimum: the NaN vertex is kept, as in Optim
      xmin[k] = xcen[k];
      fmin[k] = fcen[k];
    } else {
      xmin[k] = vertex(k, i);
      fmin[k] = fsx[k][i];
    }
  }
  pick_best(pb, c, fmin, xmin, conv, f_calls, acc);
}

}  // namespace

Result optimize(const Problem& pb, const Options& opt, Factory& fac) {
  const int nt = pb.ntrees();
  if (nt < 0) throw Error(SRHIP_ERR_INVALID, "no trees");
  if (opt.iterations < 0 || opt.nrestarts < 0) throw Error(SRHIP_ERR_INVALID, "negative iterations / restarts");
  if (opt.algorithm != SRHIP_OPT_BFGS && opt.algorithm != SRHIP_OPT_NELDERMEAD)
    throw Error(SRHIP_ERR_UNSUPPORTED, "Optimization function not implemented.");  // :39-41
  const Num num{pb.dtype == SRHIP_F32};
  const size_t nconst = pb.consts.size();
  std::vector<double> noise;
  if (opt.noise) {
    noise.assign(opt.noise, opt.noise + (size_t)opt.nrestarts * nconst);
  } else {
    std::mt19937_64 gen(opt.seed);
    std::normal_distribution<double> nd;
    noise.resize((size_t)opt.nrestarts * nconst);
    for (double& z : noise) z = nd(gen);
  }
  Result r;
  r.consts = pb.consts;
  r.converged.assign(nt, 0);
  r.num_evals.assign(nt, 0.0);
  Acc acc{r.num_evals, r.converged, r.consts};
  std::vector<int> single, multi;
  for (int i = 0; i < nt; ++i) {
    const int n = pb.const_off[i + 1] - pb.const_off[i];
    if (opt.algorithm == SRHIP_OPT_NELDERMEAD && n > 1) multi.push_back(i);
    else single.push_back(i);  // one constant: Newton whatever the option says (:32-33)
  }
  run_gradient(pb, single, opt, noise, num, fac, acc);
  run_nelder_mead(pb, multi, opt, noise, num, fac, acc);
  // the trees as they stand: one evaluation (the reference's score_func re-score, :58)
  std::vector<int32_t> all(nt);
  for (int i = 0; i < nt; ++i) all[i] = i;
  std::vector<double> g;
  if (nt > 0) fac.make(all)->eval(r.consts, false, r.loss, g);
  return r;
}

}  // namespace copt
}  // namespace srhip
