// constopt.h — batched constant optimisation (optimize_constants,
// src/ConstantOptimization.jl:22-65, for a whole population at once).
//
// Every start (x0 and optimizer_nrestarts perturbed copies, :42-54) of every
// tree is one candidate; all candidates advance in lockstep and each phase of
// an iteration is ONE evaluation of all of them (one launch on the engine):
// BFGS (Newton for one constant) with LineSearches.BackTracking (order 3), or
// Nelder-Mead for trees of two or more constants. The per-candidate algebra
// (inverse-Hessian updates, backtracking interpolation, simplex moves) is a
// few flops per constant and runs here on the host, in the order of the
// checker (tests/constopt_reference.py) so both trajectories are identical
// for the same evaluator and start noise. DESIGN.md §3.5.
#pragma once

#include <cstdint>
#include <memory>
#include <vector>

namespace srhip {
namespace copt {

// One evaluation set: a fixed list of members (input tree indices, with
// repetition); eval() scores every member at the given constants (members'
// constants concatenated in member order, values of the dtype held in
// double). f: loss per member (+Inf when the evaluation fails or is not
// finite); g (grad only): ∂L/∂c per constant, NaN for failed members.
struct Set {
  virtual ~Set() = default;
  virtual void eval(const std::vector<double>& X, bool grad, std::vector<double>& f, std::vector<double>& g) = 0;
};
struct Factory {
  virtual ~Factory() = default;
  virtual std::unique_ptr<Set> make(const std::vector<int32_t>& members) = 0;
  // small sets for the line-search stragglers (the engine: a program of their own)
  virtual bool has_subset() const { return true; }
};

struct Problem {
  int dtype = 0;                  // SRHIP_F32 / SRHIP_F64
  std::vector<int32_t> const_off; // [ntrees + 1]
  std::vector<double> consts;     // x0 of every tree (values of the dtype)
  int ntrees() const { return (int)const_off.size() - 1; }
};

struct Options {
  int algorithm = 0;   // SRHIP_OPT_BFGS / SRHIP_OPT_NELDERMEAD
  int iterations = 8;  // optimizer_iterations (src/Options.jl:607-621)
  int nrestarts = 2;   // optimizer_nrestarts
  const double* noise = nullptr;  // [nrestarts * const_off[ntrees]] standard normal draws, or null
  uint64_t seed = 0;   // draws of an internal generator when noise is null
};

struct Result {
  std::vector<double> consts;     // the input constants, the best start's where it converged
  std::vector<double> loss;       // loss of every tree at those constants (one final evaluation)
  std::vector<uint8_t> converged;
  std::vector<double> num_evals;  // loss evaluations (a loss + gradient counts once)
};

Result optimize(const Problem& pb, const Options& opt, Factory& fac);

}  // namespace copt
}  // namespace srhip
