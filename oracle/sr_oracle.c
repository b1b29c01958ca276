/*
 * sr_oracle.c — CPU restatement of the SymbolicRegression.jl scoring hot
 * path (TEST INFRASTRUCTURE ONLY; see sr_oracle.h for scope and pinning).
 *
 * Built twice by oracle/Makefile from this one source:
 *   liboracle_scalar.so  -O2 -fno-tree-vectorize   ~ Options(turbo=false)
 *   liboracle_simd.so    -O3 -march=x86-64-v3      ~ Options(turbo=true)
 * both with -ffp-contract=off (no fused multiply-add: Julia does not contract
 * `a*b + c`), no fast-math, and OpenMP over trees for the batched entry.
 */
#include "sr_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/srhip.h"

int oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

#define CAT_(a, b) a##b
#define CAT(a, b) CAT_(a, b)

/* Rounding-noise model for the parity tests' condition estimates (TEST
 * INFRASTRUCTURE, default off): with eps > 0 every transcendental value of
 * the float64 evaluator is multiplied by (1 + eps u), u in [-1, 1) a hash of
 * the operand bits and the seed. Two correct evaluations of one tree may
 * differ by each operator's error bound (<= 4 ulp for transcendentals), and
 * a tree can amplify that far beyond what input perturbations show (cos of a
 * cancellation); the tests take the spread of such noisy evaluations as the
 * tolerance of a whole-tree comparison. */
static double g_noise_eps = 0.0;
static uint64_t g_noise_seed = 0;
void oracle_set_noise(double eps, uint64_t seed) {
  g_noise_eps = eps;
  g_noise_seed = seed;
}
static inline double oracle_noise_f64(double v) {
  if (g_noise_eps == 0.0) return v;
  uint64_t h;
  memcpy(&h, &v, 8);
  h ^= g_noise_seed;
  h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ull; h ^= h >> 33;
  const double u = (double)(h >> 11) * (1.0 / 4503599627370496.0) - 1.0; /* [-1, 1) */
  return v * (1.0 + g_noise_eps * u);
}

/* |r|^n of LPDistLoss{n} with an integer n (SRHIP_LOSS_LPINT): Julia's
 * ^(::Float32, ::Integer) and ^(::Float64, ::Integer), Base math.jl (Julia
 * 1.9+: Float32 keeps literal_pow's x*x*x for n = 3 and (1/x)^2 for n = -2,
 * else Base.power_by_squaring in Float64 rounded once; Float64 by pow_body,
 * power by squaring with each product's error carried by fma). Not in
 * /root/reference (Julia's Base); restated from its published source, parity
 * unpinned. */
static double oracle_pbs(double x, long long p) {
  if (p == 0) return 1.0;
  if (p == 1) return x;
  if (p == 2) return x * x;
  int t = __builtin_ctzll((unsigned long long)p) + 1;
  p >>= t;
  while ((t -= 1) > 0) x = x * x;
  double y = x;
  while (p > 0) {
    t = __builtin_ctzll((unsigned long long)p) + 1;
    p >>= t;
    while ((t -= 1) >= 0) x = x * x;
    y = y * x;
  }
  return y;
}
static float ipow_f32(float x, long long n) {
  if (n == -2) { float i = 1.0f / x; return i * i; }
  if (n == 3) return x * x * x;
  if (n < 0) return (float)oracle_pbs(1.0 / (double)x, -n);
  return (float)oracle_pbs((double)x, n);
}
static double ipow_f64(double x, long long n) {
  double y = 1.0, xnlo = 0.0, ynlo = 0.0;
  if (n == 0) return 1.0;
  if (n == 3) return x * x * x;
  if (n < 0) {
    double rx = 1.0 / x;
    if (n == -2) return rx * rx;
    if (isfinite(x)) xnlo = -fma(x, rx, -1.0) * rx;
    x = rx;
    n = -n;
  }
  while (n > 1) {
    if (n & 1) {
      double err = fma(y, xnlo, x * ynlo);
      double xy = x * y;
      ynlo = fma(x, y, -xy);
      y = xy;
      ynlo += err;
    }
    double err = x * 2 * xnlo;
    double xx = x * x;
    xnlo = fma(x, x, -xx);
    x = xx;
    xnlo += err;
    n >>= 1;
  }
  double err = fma(y, xnlo, x * ynlo);
  return (isfinite(x) && isfinite(err)) ? fma(x, y, err) : x * y;
}

/* ---------------- T = float ---------------- */
#define T float
#define TNOISE(v) (v)
#define SFX _f32
#define TRUNC truncf
#define FMOD fmodf
#define COPYSIGN copysignf
#define SIGNBIT signbit
#define FABS fabsf
#define SQRT sqrtf
#define RINT rintf
#define FLOOR floorf
#define CEIL ceilf
#define ISINF isinf
#define ISFINITE isfinite
#include "sr_oracle_ops.h"
#include "sr_oracle_eval.h"
#undef ONODE
#undef ECTX
#undef XAT
#undef BOP_CASE
#undef FOR_EACH_BOP
#undef UOP_CASE
#undef FOR_EACH_UOP
#undef T
#undef TNOISE
#undef SFX
#undef TRUNC
#undef FMOD
#undef COPYSIGN
#undef FABS
#undef SQRT
#undef RINT
#undef FLOOR
#undef CEIL

/* ---------------- T = double ---------------- */
#define T double
#define TNOISE(v) oracle_noise_f64(v)
#define SFX _f64
#define TRUNC trunc
#define FMOD fmod
#define COPYSIGN copysign
#define FABS fabs
#define SQRT sqrt
#define RINT rint
#define FLOOR floor
#define CEIL ceil
#include "sr_oracle_ops.h"
#include "sr_oracle_eval.h"

float oracle_binop_f32(int op, float x, float y) { return apply_b_f32(op, x, y); }
double oracle_binop_f64(int op, double x, double y) { return apply_b_f64(op, x, y); }
float oracle_unop_f32(int op, float x) { return apply_u_f32(op, x); }
double oracle_unop_f64(int op, double x) { return apply_u_f64(op, x); }

double oracle_elem_loss_f64(int loss, const double* params, double yhat, double y) {
  return elem_loss_f64(loss, params, yhat, y);
}
float oracle_elem_loss_f32(int loss, const double* params, float yhat, float y) {
  return elem_loss_f32(loss, params, yhat, y);
}

/* one body for both precisions: the Float32 gradient is what the reference
 * computes for Float32 trees (every intermediate rounded to Float32) */
#define GRAD_CONSTS_BODY(T, SFX_)                                                                  \
  if (nnodes <= 0) return 0;                                                                       \
  CAT(onode, SFX_)* nd = (CAT(onode, SFX_)*)malloc(sizeof(CAT(onode, SFX_)) * nnodes);            \
  int root = CAT(parse, SFX_)(kind, arg, consts, nnodes, nd);                                      \
  if (root < 0) { free(nd); return 0; }                                                            \
  int nc = 0;                                                                                      \
  for (int i = 0; i < nnodes; ++i) nc += (kind[i] == SRHIP_NODE_CONST);                            \
  CAT(ectx, SFX_) c = {nd, X, n, nfeat};                                                           \
  int cidx = 0;                                                                                    \
  T* val = (T*)malloc(sizeof(T) * (size_t)(n > 0 ? n : 1));                                        \
  T* tan = (T*)malloc(sizeof(T) * (size_t)(nc > 0 ? nc : 1) * (size_t)(n > 0 ? n : 1));            \
  int ok = CAT(grad_rec, SFX_)(&c, root, nc, &cidx, val, tan);                                     \
  if (out) memcpy(out, val, sizeof(T) * (size_t)n);                                                \
  if (grad) memcpy(grad, tan, sizeof(T) * (size_t)nc * (size_t)n);                                 \
  free(val); free(tan); free(nd);                                                                  \
  return ok;

int oracle_eval_grad_consts_f64(const uint8_t* kind, const uint16_t* arg,
                                const double* consts, int32_t nnodes,
                                const double* X, int64_t n, int32_t nfeat,
                                double* out, double* grad) {
  GRAD_CONSTS_BODY(double, _f64)
}

int oracle_eval_grad_consts_f32(const uint8_t* kind, const uint16_t* arg,
                                const float* consts, int32_t nnodes,
                                const float* X, int64_t n, int32_t nfeat,
                                float* out, float* grad) {
  GRAD_CONSTS_BODY(float, _f32)
}
