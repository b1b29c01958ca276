// host_ops.h — scalar operator semantics on the host, used by the program
// compiler to fold feature-free subtrees into one constant, exactly as
// DynamicExpressions' `is_constant(tree)` path does on the CPU
// (`_eval_constant_tree`: scalar evaluation, every operator output checked
// with isfinite, constant leaves unchecked).
//
// Semantics: src/Operators.jl:8-111 after src/Options.jl:86-120. Float32
// transcendentals are evaluated in double and rounded once (Julia evaluates
// Float32 trig/exp/log with Float64 kernels; SpecialFunctions promotes).
#pragma once
#include <cmath>
#include <cstdint>

#include "srhip_internal.h"

namespace srhip {
namespace host {

template <typename T>
inline T rd(double v) { return (T)v; }

template <typename T>
inline T safe_pow(T x, T y) {
  if (y == std::trunc(y)) {
    if (y < T(0) && x == T(0)) return T(NAN);
  } else {
    if (y > T(0) && x < T(0)) return T(NAN);
    if (y < T(0) && x <= T(0)) return T(NAN);
  }
  return rd<T>(std::pow((double)x, (double)y));
}

template <typename T>
inline T jl_mod(T x, T y) {
  T r = std::fmod(x, y);
  if (r == T(0)) return std::copysign(r, y);
  if ((r > T(0)) != (y > T(0))) return r + y;
  return r;
}

template <typename T>
inline T binop(int op, T x, T y) {
  switch (op) {
    case SRHIP_BOP_ADD: return x + y;
    case SRHIP_BOP_SUB: return x - y;
    case SRHIP_BOP_MUL: return x * y;
    case SRHIP_BOP_DIV: return x / y;
    case SRHIP_BOP_POW: return safe_pow(x, y);
    case SRHIP_BOP_GREATER: return x > y ? T(1) : T(0);
    case SRHIP_BOP_LOGICAL_OR: return (x > T(0) || y > T(0)) ? T(1) : T(0);
    case SRHIP_BOP_LOGICAL_AND: return (x > T(0) && y > T(0)) ? T(1) : T(0);
    case SRHIP_BOP_MOD: return jl_mod(x, y);
    case SRHIP_BOP_MAX:
      if (x != x || y != y) return x - y;
      if (x > y) return x;
      if (y > x) return y;
      return std::signbit(x) ? y : x;
    case SRHIP_BOP_MIN:
      if (x != x || y != y) return x - y;
      if (x < y) return x;
      if (y < x) return y;
      return std::signbit(x) ? x : y;
  }
  return T(NAN);
}

template <typename T>
inline T unop(int op, T x) {
  const double d = (double)x;
  switch (op) {
    case SRHIP_UOP_NEG: return -x;
    case SRHIP_UOP_SQUARE: return x * x;
    case SRHIP_UOP_CUBE: return (x * x) * x;
    case SRHIP_UOP_EXP: return rd<T>(std::exp(d));
    case SRHIP_UOP_ABS: return std::fabs(x);
    case SRHIP_UOP_LOG: return x <= T(0) ? T(NAN) : rd<T>(std::log(d));
    case SRHIP_UOP_LOG2: return x <= T(0) ? T(NAN) : rd<T>(std::log2(d));
    case SRHIP_UOP_LOG10: return x <= T(0) ? T(NAN) : rd<T>(std::log10(d));
    case SRHIP_UOP_LOG1P: return x <= T(-1) ? T(NAN) : rd<T>(std::log1p(d));
    case SRHIP_UOP_SQRT: return x < T(0) ? T(NAN) : std::sqrt(x);
    case SRHIP_UOP_SIN: return rd<T>(std::sin(d));
    case SRHIP_UOP_COS: return rd<T>(std::cos(d));
    case SRHIP_UOP_TAN: return rd<T>(std::tan(d));
    case SRHIP_UOP_SINH: return rd<T>(std::sinh(d));
    case SRHIP_UOP_COSH: return rd<T>(std::cosh(d));
    case SRHIP_UOP_TANH: return rd<T>(std::tanh(d));
    case SRHIP_UOP_ATAN: return rd<T>(std::atan(d));
    case SRHIP_UOP_ASINH: return rd<T>(std::asinh(d));
    case SRHIP_UOP_ACOSH: return x < T(1) ? T(NAN) : rd<T>(std::acosh(d));
    case SRHIP_UOP_ATANH_CLIP: return rd<T>(std::atanh((double)(jl_mod<T>(x + T(1), T(2)) - T(1))));
    case SRHIP_UOP_ERF: return rd<T>(std::erf(d));
    case SRHIP_UOP_ERFC: return rd<T>(std::erfc(d));
    case SRHIP_UOP_GAMMA: {
      T g = rd<T>(std::tgamma(d));
      return std::isinf(g) ? T(NAN) : g;
    }
    case SRHIP_UOP_RELU: return (x + std::fabs(x)) / T(2);
    case SRHIP_UOP_ROUND: return std::rint(x);
    case SRHIP_UOP_FLOOR: return std::floor(x);
    case SRHIP_UOP_CEIL: return std::ceil(x);
    case SRHIP_UOP_SIGN: return x > T(0) ? T(1) : (x < T(0) ? T(-1) : x);
    case SRHIP_UOP_INV: return T(1) / x;
  }
  return T(NAN);
}

}  // namespace host
}  // namespace srhip
