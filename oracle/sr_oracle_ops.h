/*
 * sr_oracle_ops.h — scalar operator semantics, instantiated for T = float and
 * T = double by sr_oracle.c (TEST INFRASTRUCTURE ONLY; see sr_oracle.h).
 *
 * Follows src/Operators.jl:8-111 after the mapping of src/Options.jl:86-120.
 * Float32 transcendentals are evaluated in double and rounded once, which is
 * what Julia's Base does for Float32 trig/exp/log (Float64 kernels) and what
 * SpecialFunctions does for Float32 gamma/erf (promote, evaluate, convert).
 *
 * Expected macros: T, SFX (suffix token), and TNOISE(v): the identity, except
 * in the float64 build while a test has set a rounding-noise amplitude
 * (oracle_set_noise, sr_oracle.c) to estimate a tree's condition.
 */

static inline T CAT(b_add, SFX)(T x, T y) { return x + y; }
static inline T CAT(b_sub, SFX)(T x, T y) { return x - y; }
static inline T CAT(b_mul, SFX)(T x, T y) { return x * y; }
static inline T CAT(b_div, SFX)(T x, T y) { return x / y; }

/* safe_pow, Operators.jl:38-46 */
static inline T CAT(b_pow, SFX)(T x, T y) {
  if (y == TRUNC(y)) { /* isinteger(y) */
    if (y < (T)0 && x == (T)0) return (T)NAN;
  } else {
    if (y > (T)0 && x < (T)0) return (T)NAN;
    if (y < (T)0 && x <= (T)0) return (T)NAN;
  }
  return TNOISE((T)pow((double)x, (double)y));
}
/* greater / logical_or / logical_and, Operators.jl:94-111 */
static inline T CAT(b_greater, SFX)(T x, T y) { return x > y ? (T)1 : (T)0; }
static inline T CAT(b_or, SFX)(T x, T y) { return (x > (T)0 || y > (T)0) ? (T)1 : (T)0; }
static inline T CAT(b_and, SFX)(T x, T y) { return (x > (T)0 && y > (T)0) ? (T)1 : (T)0; }
/* Base.mod(x::T, y::T) for floats: r = rem(x, y); r == 0 → copysign(r, y);
 * sign mismatch → r + y; else r. rem is C fmod (exact). */
static inline T CAT(b_mod, SFX)(T x, T y) {
  T r = FMOD(x, y);
  if (r == (T)0) return COPYSIGN(r, y);
  if ((r > (T)0) != (y > (T)0)) return r + y;
  return r;
}
/* Base.max / Base.min for floats: NaN-propagating, -0.0 < +0.0 */
static inline T CAT(b_max, SFX)(T x, T y) {
  if (x != x || y != y) return x - y; /* NaN */
  if (x > y) return x;
  if (y > x) return y;
  return SIGNBIT(x) ? y : x;
}
static inline T CAT(b_min, SFX)(T x, T y) {
  if (x != x || y != y) return x - y;
  if (x < y) return x;
  if (y < x) return y;
  return SIGNBIT(x) ? x : y;
}

static inline T CAT(u_neg, SFX)(T x) { return -x; }
static inline T CAT(u_square, SFX)(T x) { return x * x; }
static inline T CAT(u_cube, SFX)(T x) { return (x * x) * x; } /* literal_pow x^3 = x*x*x */
static inline T CAT(u_exp, SFX)(T x) { return TNOISE((T)exp((double)x)); }
static inline T CAT(u_abs, SFX)(T x) { return FABS(x); }
static inline T CAT(u_log, SFX)(T x) { return x <= (T)0 ? (T)NAN : TNOISE((T)log((double)x)); }
static inline T CAT(u_log2, SFX)(T x) { return x <= (T)0 ? (T)NAN : TNOISE((T)log2((double)x)); }
static inline T CAT(u_log10, SFX)(T x) { return x <= (T)0 ? (T)NAN : TNOISE((T)log10((double)x)); }
static inline T CAT(u_log1p, SFX)(T x) { return x <= (T)-1 ? (T)NAN : TNOISE((T)log1p((double)x)); }
static inline T CAT(u_sqrt, SFX)(T x) { return x < (T)0 ? (T)NAN : SQRT(x); }
static inline T CAT(u_sin, SFX)(T x) { return TNOISE((T)sin((double)x)); }
static inline T CAT(u_cos, SFX)(T x) { return TNOISE((T)cos((double)x)); }
static inline T CAT(u_tan, SFX)(T x) { return TNOISE((T)tan((double)x)); }
static inline T CAT(u_sinh, SFX)(T x) { return TNOISE((T)sinh((double)x)); }
static inline T CAT(u_cosh, SFX)(T x) { return TNOISE((T)cosh((double)x)); }
static inline T CAT(u_tanh, SFX)(T x) { return TNOISE((T)tanh((double)x)); }
static inline T CAT(u_atan, SFX)(T x) { return TNOISE((T)atan((double)x)); }
static inline T CAT(u_asinh, SFX)(T x) { return TNOISE((T)asinh((double)x)); }
static inline T CAT(u_acosh, SFX)(T x) { return x < (T)1 ? (T)NAN : TNOISE((T)acosh((double)x)); }
/* atanh_clip(x) = atanh(mod(x + 1, 2) - 1), Operators.jl:14 */
static inline T CAT(u_atanh_clip, SFX)(T x) {
  T m = CAT(b_mod, SFX)(x + (T)1, (T)2) - (T)1;
  return TNOISE((T)atanh((double)m));
}
static inline T CAT(u_erf, SFX)(T x) { return TNOISE((T)erf((double)x)); }
static inline T CAT(u_erfc, SFX)(T x) { return TNOISE((T)erfc((double)x)); }
/* gamma: Inf → NaN, Operators.jl:8-11 (check made on the T result) */
static inline T CAT(u_gamma, SFX)(T x) {
  T g = (T)tgamma((double)x);
  return ISINF(g) ? (T)NAN : TNOISE(g);
}
static inline T CAT(u_relu, SFX)(T x) { return (x + FABS(x)) / (T)2; } /* :100-102 */
static inline T CAT(u_round, SFX)(T x) { return RINT(x); }             /* RoundNearest */
static inline T CAT(u_floor, SFX)(T x) { return FLOOR(x); }
static inline T CAT(u_ceil, SFX)(T x) { return CEIL(x); }
static inline T CAT(u_sign, SFX)(T x) {
  if (x > (T)0) return (T)1;
  if (x < (T)0) return (T)-1;
  return x; /* ±0 and NaN */
}
static inline T CAT(u_inv, SFX)(T x) { return (T)1 / x; }

/* dispatch helpers: the macro runs STMT(fn) with the per-operator function so
 * that the row loops are specialised per operator (the reference compiles one
 * loop per operator, too). */
#define CAT3(a, b) a##b
#define FN(name, sfx) CAT3(name, sfx)

/* derivatives (forward mode) — ∂op/∂x, ∂op/∂y in T */
static inline void CAT(db, SFX)(int op, T x, T y, T* dx, T* dy) {
  switch (op) {
    case SRHIP_BOP_ADD: *dx = 1; *dy = 1; break;
    case SRHIP_BOP_SUB: *dx = 1; *dy = -1; break;
    case SRHIP_BOP_MUL: *dx = y; *dy = x; break;
    case SRHIP_BOP_DIV: *dx = (T)1 / y; *dy = -x / (y * y); break;
    case SRHIP_BOP_POW: {
      T p = CAT(b_pow, SFX)(x, y);
      *dx = y * CAT(b_pow, SFX)(x, y - (T)1);
      *dy = (x > (T)0) ? p * (T)log((double)x) : (T)0;
      break;
    }
    case SRHIP_BOP_MAX: *dx = (x >= y) ? (T)1 : (T)0; *dy = (x >= y) ? (T)0 : (T)1; break;
    case SRHIP_BOP_MIN: *dx = (x <= y) ? (T)1 : (T)0; *dy = (x <= y) ? (T)0 : (T)1; break;
    case SRHIP_BOP_MOD: *dx = 1; *dy = -FLOOR(x / y); break;
    default: *dx = 0; *dy = 0; break;
  }
}
static inline T CAT(du, SFX)(int op, T x) {
  switch (op) {
    case SRHIP_UOP_NEG: return -1;
    case SRHIP_UOP_SQUARE: return (T)2 * x;
    case SRHIP_UOP_CUBE: return (T)3 * x * x;
    case SRHIP_UOP_EXP: return (T)exp((double)x);
    case SRHIP_UOP_ABS: return x > (T)0 ? (T)1 : (x < (T)0 ? (T)-1 : (T)0);
    case SRHIP_UOP_LOG: return (T)1 / x;
    case SRHIP_UOP_LOG2: return (T)(1.0 / ((double)x * 0.69314718055994530942));
    case SRHIP_UOP_LOG10: return (T)(1.0 / ((double)x * 2.30258509299404568402));
    case SRHIP_UOP_LOG1P: return (T)1 / ((T)1 + x);
    case SRHIP_UOP_SQRT: return (T)0.5 / SQRT(x);
    case SRHIP_UOP_SIN: return (T)cos((double)x);
    case SRHIP_UOP_COS: return -(T)sin((double)x);
    case SRHIP_UOP_TAN: { T c = (T)cos((double)x); return (T)1 / (c * c); }
    case SRHIP_UOP_SINH: return (T)cosh((double)x);
    case SRHIP_UOP_COSH: return (T)sinh((double)x);
    case SRHIP_UOP_TANH: { T t = (T)tanh((double)x); return (T)1 - t * t; }
    case SRHIP_UOP_ATAN: return (T)1 / ((T)1 + x * x);
    case SRHIP_UOP_ASINH: return (T)(1.0 / sqrt((double)x * x + 1.0));
    case SRHIP_UOP_ACOSH: return (T)(1.0 / sqrt((double)x * x - 1.0));
    case SRHIP_UOP_ERF: return (T)(1.1283791670955126 * exp(-(double)x * x));
    case SRHIP_UOP_ERFC: return (T)(-1.1283791670955126 * exp(-(double)x * x));
    case SRHIP_UOP_RELU: return x > (T)0 ? (T)1 : (T)0;
    case SRHIP_UOP_INV: return (T)-1 / (x * x);
    default: return 0;
  }
}
