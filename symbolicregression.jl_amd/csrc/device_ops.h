// device_ops.h — operator and loss semantics on the device (gfx950).
//
// Semantics: src/Operators.jl:8-111 after the mapping of
// src/Options.jl:86-120; Base.mod / max / min for floats; LossFunctions.jl
// distance losses (docs/src/losses.md). `+ - * /` and sqrt are IEEE
// correctly rounded (built with -ffp-contract=off, no fast-math, f32
// denormals kept), so they are bit-identical to Julia; transcendentals use
// OCML's full-precision routines (never the __expf-style intrinsics).
#pragma once
#include <hip/hip_runtime.h>

#include "srhip_internal.h"

namespace srhip {
namespace dev {

// ---- thin overload set over OCML ----------------------------------------------
// Heavy or branchy routines (trig range reduction, tgamma, pow, fmod, ...)
// are called out of line: inlined into the interpreter's dispatch switch,
// their divergent internal branches make the register allocator split the
// accumulator's live ranges and insert a copy of every accumulator register
// into EVERY dispatch. A call costs two v_mov and an s_swappc per value.
// exp, log and sqrt are short and branch-free and stay inline.
#define SR_M1(name, f32, f64)                                              \
  __device__ __forceinline__ float name(float x) { return f32(x); }        \
  __device__ __forceinline__ double name(double x) { return f64(x); }
// SRHIP_INLINE_ALL (the threaded interpreter's handler snippets,
// gen_asm_interp.py): everything inline, a handler body cannot call.
#ifdef SRHIP_INLINE_ALL
#define SR_NOINLINE __attribute__((always_inline))
#else
#define SR_NOINLINE __attribute__((noinline))
#endif
#define SR_M1_OOL(name, f32, f64)                                                       \
  __device__ SR_NOINLINE float name##_ool(float x) { return f32(x); }      \
  __device__ SR_NOINLINE double name##_ool(double x) { return f64(x); }    \
  __device__ __forceinline__ float name(float x) { return name##_ool(x); }              \
  __device__ __forceinline__ double name(double x) { return name##_ool(x); }
// f32 exp: OCML's expf is a 2^x kernel plus over/underflow selects; here the
// argument is clamped first (exp(89) = Inf and exp(-104) rounds to 0 like the
// unclamped value; NaN/Inf operands fail the tree before the value is used,
// exp being checked as lossy) and the selects go. e = rint(x log2 e); the
// reduced argument a = x log2(e) - e comes from two FMAs (log2 e as hi + lo,
// |error| <= 2^-25), then v_exp_f32(a) and v_ldexp by e: 8 VALU. Validated
// exhaustively against the correctly rounded value on MI355X: <= 1 ulp over
// every float (tools/check_fast_exp.hip), as OCML's expf.
__device__ __forceinline__ float fast_exp_f32(float x) {
  x = __builtin_amdgcn_fmed3f(x, -104.0f, 89.0f);
  const float e = __builtin_rintf(x * 1.44269502e+00f);
  float a = __builtin_fmaf(x, 1.44269502e+00f, -e);
  a = __builtin_fmaf(x, 1.92596299e-08f, a);
  return __builtin_amdgcn_ldexpf(__builtin_amdgcn_exp2f(a), (int)e);
}
// SR_PRECISE_TRANSC (default 1): Float32 exp / sin / cos are evaluated in
// Float64 and rounded once, as Julia does for Float32 arguments and as the
// oracle does. A 1-ulp difference in one of them decides did_succeed when a
// divisor cancels to exactly 0 on some row (4 of 4096 config #2
// trees with the f32 routines); with one rounding of a ~2^-52-accurate value
// the engine returns the correctly rounded Float32 except within ~2^-28 of a
// rounding boundary. SR_PRECISE_TRANSC=0 builds the all-f32 routines.
#ifndef SR_PRECISE_TRANSC
#define SR_PRECISE_TRANSC 1
#endif
// e^x = 2^n e^r, n = rint(x log2 e), r = x - n ln2 (two-part ln2, exact
// products for |n| <= 151), e^r by a degree-10 minimax polynomial (|r| <=
// 0.347: relative error 2^-51.6; the Taylor series to r^11 of rounds 1-4 had
// 2^-47 with one more FMA), one v_ldexp_f64, one rounding to Float32. Every
// float of [-104, 89] rounds as the oracle's (float)exp((double)x) does
// (tools/check_precise.c: 0 differ; the Taylor form 2).
__device__ __forceinline__ float precise_exp_f32(float x) {
  x = __builtin_amdgcn_fmed3f(x, -104.0f, 89.0f);
  const double xd = (double)x;
  const double n = __builtin_rint(xd * 1.4426950408889634);
  double r = __builtin_fma(n, -6.93147180369123816490e-01, xd);
  r = __builtin_fma(n, -1.90821492927058770002e-10, r);
  double p = 2.74715993357489975e-07;
  p = __builtin_fma(p, r, 2.76351209779822652e-06);
  p = __builtin_fma(p, r, 2.48019464013407408e-05);
  p = __builtin_fma(p, r, 1.98411849339436464e-04);
  p = __builtin_fma(p, r, 1.38888885022706824e-03);
  p = __builtin_fma(p, r, 8.33333337108620349e-03);
  p = __builtin_fma(p, r, 4.16666666681865250e-02);
  p = __builtin_fma(p, r, 1.66666666666110797e-01);
  p = __builtin_fma(p, r, 4.99999999999982736e-01);
  p = __builtin_fma(p, r, 1.0);
  p = __builtin_fma(p, r, 1.0);
  return (float)__builtin_amdgcn_ldexp(p, (int)n);
}
#if SR_PRECISE_TRANSC
__device__ __forceinline__ float m_exp(float x) { return precise_exp_f32(x); }
#else
__device__ __forceinline__ float m_exp(float x) { return fast_exp_f32(x); }
#endif
__device__ __forceinline__ double m_exp(double x) { return exp(x); }
// log / log2 / log10 and pow of Float32 operands: PRECISE (the default)
// evaluates them in Float64 and rounds once, as Julia's Base does (Float64
// kernels for Float32 log; Float32 ^ promotes) and as the oracle does; OCML's
// logf / powf are within 1 ulp but not correctly rounded, and an ill-
// conditioned tree (cos(safe_log(x)) near a zero of cos) turns that ulp into
// a visible loss / gradient difference (round 5, config #3's operators).
#if SR_PRECISE_TRANSC
__device__ __forceinline__ float m_log(float x) { return (float)log((double)x); }
__device__ SR_NOINLINE float m_log2_ool(float x) { return (float)log2((double)x); }
__device__ SR_NOINLINE float m_log10_ool(float x) { return (float)log10((double)x); }
#else
__device__ __forceinline__ float m_log(float x) { return logf(x); }
__device__ SR_NOINLINE float m_log2_ool(float x) { return log2f(x); }
__device__ SR_NOINLINE float m_log10_ool(float x) { return log10f(x); }
#endif
__device__ __forceinline__ double m_log(double x) { return log(x); }
__device__ SR_NOINLINE double m_log2_ool(double x) { return log2(x); }
__device__ SR_NOINLINE double m_log10_ool(double x) { return log10(x); }
__device__ __forceinline__ float m_log2(float x) { return m_log2_ool(x); }
__device__ __forceinline__ double m_log2(double x) { return m_log2_ool(x); }
__device__ __forceinline__ float m_log10(float x) { return m_log10_ool(x); }
__device__ __forceinline__ double m_log10(double x) { return m_log10_ool(x); }
SR_M1_OOL(m_log1p, log1pf, log1p)
SR_M1(m_sqrt, sqrtf, sqrt)
SR_M1_OOL(m_sin_ocml, sinf, sin)
SR_M1_OOL(m_cos_ocml, cosf, cos)
SR_M1_OOL(m_tan, tanf, tan)
SR_M1_OOL(m_sinh, sinhf, sinh)
SR_M1_OOL(m_cosh, coshf, cosh)
SR_M1_OOL(m_tanh, tanhf, tanh)
SR_M1_OOL(m_atan, atanf, atan)
SR_M1_OOL(m_asinh, asinhf, asinh)
SR_M1_OOL(m_acosh, acoshf, acosh)
SR_M1_OOL(m_atanh, atanhf, atanh)
SR_M1_OOL(m_erf, erff, erf)
SR_M1_OOL(m_erfc, erfcf, erfc)
SR_M1_OOL(m_tgamma, tgammaf, tgamma)
SR_M1(m_rint, rintf, rint)
SR_M1(m_floor, floorf, floor)
SR_M1(m_ceil, ceilf, ceil)
SR_M1(m_trunc, truncf, trunc)
SR_M1(m_fabs, fabsf, fabs)
#undef SR_M1
#undef SR_M1_OOL
#if SR_PRECISE_TRANSC
__device__ SR_NOINLINE float m_pow(float x, float y) { return (float)pow((double)x, (double)y); }
#else
__device__ SR_NOINLINE float m_pow(float x, float y) { return powf(x, y); }
#endif
__device__ SR_NOINLINE double m_pow(double x, double y) { return pow(x, y); }
__device__ SR_NOINLINE float m_fmod(float x, float y) { return fmodf(x, y); }
__device__ SR_NOINLINE double m_fmod(double x, double y) { return fmod(x, y); }
__device__ __forceinline__ float m_copysign(float x, float y) { return copysignf(x, y); }
__device__ __forceinline__ double m_copysign(double x, double y) { return copysign(x, y); }
__device__ __forceinline__ bool m_isinf(float x) { return __builtin_isinf(x); }
__device__ __forceinline__ bool m_isinf(double x) { return __builtin_isinf(x); }
__device__ __forceinline__ bool m_signbit(float x) { return __builtin_signbit(x); }
__device__ __forceinline__ bool m_signbit(double x) { return __builtin_signbit(x); }
// ---- fast single-precision sin / cos ------------------------------------------
// Branch-free, one polynomial: reduction by pi to r in [-pi/2, pi/2],
//   sin x = (-1)^n sin(x - n pi),             n = rint(x / pi),
//   cos x = (-1)^(n+1) sin(x - (n + 1/2) pi),  n = rint(x / pi - 1/2),
// r = x - m pi/2 with m = 2n (sin) or 2n + 1 (cos) by a 3-part Cody–Waite
// split of pi/2 with FMA (exact enough for |x| <= 105615), then
// sin r = r + r^3 P(r^2), P a degree-3 minimax fit (tools/fit_sin.py, 6e-9
// relative), and the sign from n's parity as one XOR (cos folds its extra
// minus into the last FMA). 16 VALU per value for cos, where evaluating both
// quadrant polynomials and selecting took 22. Validated exhaustively on the
// CPU against correctly rounded values: <= 2 ulp over all floats with
// |x| <= 105615 (tools/check_fast_trig.c). Larger finite arguments are
// recomputed with OCML behind a wave-uniform branch (taken only if some lane
// needs it); `nabs` = |n| feeds that test.
__device__ __forceinline__ float fast_sincos_f32(float x, int want_cos, float& nabs) {
  const float n = want_cos ? __builtin_rintf(__builtin_fmaf(x, 0.318309873f, -0.5f))
                           : __builtin_rintf(x * 0.318309873f);
  nabs = __builtin_fabsf(n);
  const float m = want_cos ? __builtin_fmaf(n, 2.0f, 1.0f) : n + n;
#if SR_PRECISE_TRANSC
  // Same reduction in Float64: r = x - m pi/2 (pi/2 = HI + LO, HI with 33
  // significant bits so m*HI is exact for |m| < 2^20; |r| <= pi/2 + tiny),
  // sin r = r + r^3 P(r^2) with P a 7-term minimax fit (relative error
  // 2^-50.4 on |r| <= pi/2; the Taylor series to r^17 of rounds 1-4 had one
  // more FMA and 2^-44), one rounding to Float32, then the sign of n's
  // parity. Over every float with |x| <= 105615, sin rounds as the oracle's
  // (float)sin((double)x) on all but 2, cos on all (tools/check_precise.c;
  // the Taylor form: sin 0, cos 114).
  {
    const double md = (double)m;
    double r = __builtin_fma(md, -1.57079632673412561417e+00, (double)x);
    r = __builtin_fma(md, -6.07710050650619224932e-11, r);
    const double s2 = r * r;
    double p = -7.34673622570819757e-13;
    p = __builtin_fma(p, s2, 1.60458129180763398e-10);
    p = __builtin_fma(p, s2, -2.50518043886916424e-08);
    p = __builtin_fma(p, s2, 2.75573153848002669e-06);
    p = __builtin_fma(p, s2, -1.98412698157051834e-04);
    p = __builtin_fma(p, s2, 8.33333333325722396e-03);
    p = __builtin_fma(p, s2, -1.66666666666660662e-01);  // sin r = r + r^3 p
    const double v = __builtin_fma(p * s2, r, r);
    const float f = (float)(want_cos ? -v : v);
    return __int_as_float(__float_as_int(f) ^ ((int)n << 31));
  }
#endif
  float r = __builtin_fmaf(m, -1.57079601e+00f, x);
  r = __builtin_fmaf(m, -3.13916473e-07f, r);
  r = __builtin_fmaf(m, -5.39030253e-15f, r);
  const float s = r * r;
  float p = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(2.606342605e-06f, s, -1.980987436e-04f), s,
                                          8.333070204e-03f), s, -1.666665971e-01f);
  p = p * s;
  const float v = want_cos ? __builtin_fmaf(p, -r, -r) : __builtin_fmaf(p, r, r);
  return __int_as_float(__float_as_int(v) ^ ((int)n << 31));
}

__device__ __forceinline__ float fast_sincos_f32(float x, int want_cos) {
  float na;
  return fast_sincos_f32(x, want_cos, na);
}
// Fast-path domain test from n: |n| <= kTrigQMax implies |x| < 105250 (inside
// the validated range). max() ignores NaN rows (their result is NaN either
// way); an Inf argument gives n = Inf and takes OCML.
constexpr float kTrigQMax = 33500.0f;

// ---- sin / cos beyond the fast reduction (|x| > 105615) ------------------------
// Payne–Hanek reduction with the bits of 2/pi as instruction literals (no
// table in memory, so the tree compiler's routines can hold it, gen_jit.py):
// |x| = M 2^(e-23) with a 24-bit M; the 96 bits of 2/pi from bit e-24 on
// (one leading zero word covers small e) times M give |x| 2/pi mod 4 with 64
// fraction bits (truncation < 2^-70, far below the closest approach of a
// float to a multiple of pi/2); rounding to the nearest quadrant leaves
// r = f pi/2, |r| <= pi/4, in Float64; the Float64 Taylor polynomials of sin
// and cos (to r^17 / r^16) and one rounding to Float32 give the value the
// oracle's Float64 sin/cos rounds to (except within ~2^-45 of a rounding
// boundary).
// Out of line in the interpreters (rarely taken, behind a ballot; inline it
// would cost the dispatch loop registers), inline in the tree compiler's
// routines (SRHIP_INLINE_ALL: a routine cannot call).
__device__ SR_NOINLINE float big_sincos_f32(float x, int want_cos) {
  const uint32_t ax = __float_as_uint(x) & 0x7fffffffu;
  const int e = (int)(ax >> 23) - 127;  // >= 16 on this path
  const uint64_t M = (ax & 0x7fffffu) | 0x800000u;
  const int p0 = e + 7;                  // first window bit in the table below
  const int k = p0 >> 5, sh = p0 & 31;
  // scalars made opaque: a select chain, never an array in memory or LDS
  uint32_t t1 = 0xA2F9836Eu, t2 = 0x4E441529u, t3 = 0xFC2757D1u, t4 = 0xF534DDC0u, t5 = 0xDB629599u,
           t6 = 0x3C439041u, t7 = 0xFE5163ABu;
  asm volatile("" : "+s"(t1), "+s"(t2), "+s"(t3), "+s"(t4), "+s"(t5), "+s"(t6), "+s"(t7));
  auto word = [&](int j) {
    uint32_t r = j == 1 ? t1 : 0u;
    r = j == 2 ? t2 : r;
    r = j == 3 ? t3 : r;
    r = j == 4 ? t4 : r;
    r = j == 5 ? t5 : r;
    r = j == 6 ? t6 : r;
    return j == 7 ? t7 : r;
  };
  const uint32_t a0 = word(k), a1 = word(k + 1), a2 = word(k + 2), a3 = word(k + 3);
  auto funnel = [&](uint32_t hi, uint32_t lo) { return sh ? (hi << sh) | (lo >> (32 - sh)) : hi; };
  const uint64_t q2 = M * funnel(a2, a3), q1 = M * funnel(a1, a2), q0 = M * funnel(a0, a1);
  // P = q0 2^64 + q1 2^32 + q2 has 94 fraction bits: quadrant = P[95:94], fraction = P[93:30]
  const uint64_t t = q1 + (q2 >> 32);
  const uint64_t u = q0 + (t >> 32);
  uint32_t q = (uint32_t)(u >> 30) & 3u;
  const uint64_t frac = ((u & 0x3fffffffull) << 34) | ((t & 0xffffffffull) << 2) | ((q2 & 0xffffffffull) >> 30);
  const int64_t f = (int64_t)frac;  // >= 1/2 reads negative: the next quadrant, r < 0
  if (f < 0) q = (q + 1u) & 3u;
  const double r = (double)f * (1.5707963267948966 * 0x1p-64);  // f * pi/2 * 2^-64
  const double s2 = r * r;
  double ps = -2.81145725434552076320e-15;
  ps = __builtin_fma(ps, s2, 7.64716373181981647590e-13);
  ps = __builtin_fma(ps, s2, -1.60590438368216145994e-10);
  ps = __builtin_fma(ps, s2, 2.50521083854417187751e-08);
  ps = __builtin_fma(ps, s2, -2.75573192239858906526e-06);
  ps = __builtin_fma(ps, s2, 1.98412698412698412698e-04);
  ps = __builtin_fma(ps, s2, -8.33333333333333333333e-03);
  ps = __builtin_fma(ps, s2, 1.66666666666666666667e-01);
  const double sn = __builtin_fma(-ps * s2, r, r);
  double pc = 4.77947733238738529744e-14;           // 1/16!
  pc = __builtin_fma(pc, s2, -1.14707455977297247139e-11);  // -1/14!
  pc = __builtin_fma(pc, s2, 2.08767569878680989792e-09);   // 1/12!
  pc = __builtin_fma(pc, s2, -2.75573192239858906526e-07);  // -1/10!
  pc = __builtin_fma(pc, s2, 2.48015873015873015873e-05);   // 1/8!
  pc = __builtin_fma(pc, s2, -1.38888888888888888889e-03);  // -1/6!
  pc = __builtin_fma(pc, s2, 4.16666666666666666667e-02);   // 1/4!
  pc = __builtin_fma(pc, s2, -0.5);
  const double cs = __builtin_fma(pc, s2, 1.0);
  const uint32_t idx = (q + (want_cos ? 1u : 0u)) & 3u;  // sin(x + pi/2) = cos(x)
  double v = (idx & 1u) ? cs : sn;
  if (idx & 2u) v = -v;
  if (!want_cos && (__float_as_uint(x) >> 31)) v = -v;  // sin is odd, cos even
  return (float)v;
}

// The large-argument path is taken with a wave-uniform branch (ballot) and a
// select, so no divergent region enters the interpreter's dispatch switch.
__device__ __forceinline__ bool trig_big(float x) {
  return !(__builtin_fabsf(x) <= 105615.0f) && __builtin_isfinite(x);
}
__device__ __forceinline__ float m_sin(float x) {
  float v = fast_sincos_f32(x, 0);
  const bool big = trig_big(x);
  if (__builtin_amdgcn_ballot_w64(big) != 0) {
    const float o = big_sincos_f32(x, 0);
    v = big ? o : v;
  }
  return v;
}
__device__ __forceinline__ float m_cos(float x) {
  float v = fast_sincos_f32(x, 1);
  const bool big = trig_big(x);
  if (__builtin_amdgcn_ballot_w64(big) != 0) {
    const float o = big_sincos_f32(x, 1);
    v = big ? o : v;
  }
  return v;
}
// Float32 sin / cos for derivatives: the single-precision path of
// fast_sincos_f32 (<= 2 ulp) whatever SR_PRECISE_TRANSC says — a derivative
// value is not subject to the did_succeed parity that makes the forward
// values Float64-evaluated — with the large-argument path behind a ballot.
__device__ __forceinline__ float d_sincos_f32(float x, int want_cos) {
  const float n = want_cos ? __builtin_rintf(__builtin_fmaf(x, 0.318309873f, -0.5f))
                           : __builtin_rintf(x * 0.318309873f);
  const float m = want_cos ? __builtin_fmaf(n, 2.0f, 1.0f) : n + n;
  float r = __builtin_fmaf(m, -1.57079601e+00f, x);
  r = __builtin_fmaf(m, -3.13916473e-07f, r);
  r = __builtin_fmaf(m, -5.39030253e-15f, r);
  const float s = r * r;
  float p = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(2.606342605e-06f, s, -1.980987436e-04f), s,
                                          8.333070204e-03f), s, -1.666665971e-01f);
  p = p * s;
  float v = want_cos ? __builtin_fmaf(p, -r, -r) : __builtin_fmaf(p, r, r);
  v = __int_as_float(__float_as_int(v) ^ ((int)n << 31));
  const bool big = trig_big(x);
  if (__builtin_amdgcn_ballot_w64(big) != 0) {
    const float o = big_sincos_f32(x, want_cos);
    v = big ? o : v;
  }
  return v;
}
// sin / cos for the gradient tree code's forward pass together with the
// value its reverse pass needs (jit_grad.cpp: the routine u_sin_pd / u_cos_pd
// leaves it in B and the tree keeps it instead of x): d = cos x for sin,
// sin x for cos. The returned value is fast_sincos_f32's, bit for bit. With
// the same reduction r = x - m pi/2 both are (-1)^n cos r, evaluated as
// sin(pi/2 - |r|) from the Float64 r (relative accuracy at d's own zeros)
// with the FAST odd polynomial: <= 2 ulp as d_sincos_f32. nabs as
// fast_sincos_f32 (the caller's large-argument test).
__device__ __forceinline__ float sincos_pd_f32(float x, int want_cos, float& d, float& nabs) {
#if SR_PRECISE_TRANSC
  const float n = want_cos ? __builtin_rintf(__builtin_fmaf(x, 0.318309873f, -0.5f))
                           : __builtin_rintf(x * 0.318309873f);
  nabs = __builtin_fabsf(n);
  const float m = want_cos ? __builtin_fmaf(n, 2.0f, 1.0f) : n + n;
  const double md = (double)m;
  double r = __builtin_fma(md, -1.57079632673412561417e+00, (double)x);
  r = __builtin_fma(md, -6.07710050650619224932e-11, r);
  const double s2 = r * r;
  double p = -7.34673622570819757e-13;
  p = __builtin_fma(p, s2, 1.60458129180763398e-10);
  p = __builtin_fma(p, s2, -2.50518043886916424e-08);
  p = __builtin_fma(p, s2, 2.75573153848002669e-06);
  p = __builtin_fma(p, s2, -1.98412698157051834e-04);
  p = __builtin_fma(p, s2, 8.33333333325722396e-03);
  p = __builtin_fma(p, s2, -1.66666666666660662e-01);
  const double v = __builtin_fma(p * s2, r, r);
  const float f = (float)(want_cos ? -v : v);
  const int sg = (int)n << 31;
  // sin x of a cos node near x = 0 directly (pi/2 - |r| would cancel: x is not bounded away
  // from that zero of sin as floats are from the others, k pi, k != 0)
  const bool small = want_cos && __builtin_fabsf(x) < 0.785398163f;
  const float t = small ? x : (float)(1.5707963267948966 - __builtin_fabs(r));
  const float s = t * t;
  float q = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(2.606342605e-06f, s, -1.980987436e-04f), s,
                                          8.333070204e-03f), s, -1.666665971e-01f);
  q = q * s;
  d = __int_as_float(__float_as_int(__builtin_fmaf(q, t, t)) ^ (small ? 0 : sg));
  return __int_as_float(__float_as_int(f) ^ sg);
#else
  d = d_sincos_f32(x, !want_cos);
  return fast_sincos_f32(x, want_cos, nabs);
#endif
}
__device__ __forceinline__ double m_sin(double x) { return m_sin_ocml(x); }
__device__ __forceinline__ double m_cos(double x) { return m_cos_ocml(x); }

template <typename T>
__device__ __forceinline__ T qnan() { return __builtin_nan(""); }
template <>
__device__ __forceinline__ float qnan<float>() { return __builtin_nanf(""); }

// Base.mod for floats: r = rem(x, y) (= fmod, exact); r == 0 → copysign(r, y);
// sign(r) != sign(y) → r + y; else r. Out of line (fmod loops).
template <typename T>
__device__ SR_NOINLINE T jl_mod(T x, T y) {
  T r = m_fmod(x, y);
  T s = r + y;
  bool flip = (r > T(0)) != (y > T(0));
  T v = flip ? s : r;
  return (r == T(0)) ? m_copysign(r, y) : v;
}

// safe_pow, Operators.jl:38-46. Out of line (pow's special-case branches).
template <typename T>
__device__ SR_NOINLINE T safe_pow(T x, T y) {
  const bool isint = (y == m_trunc(y));
  const bool bad = isint ? (y < T(0) && x == T(0))
                         : ((y > T(0) && x < T(0)) || (y < T(0) && x <= T(0)));
  return bad ? qnan<T>() : m_pow(x, y);
}

// Base.max / min on finite operands, -0.0 < +0.0, branch-free: for equal
// values the bit patterns are equal except for ±0, where AND (max) clears and
// OR (min) keeps the sign bit.
__device__ __forceinline__ float bits_and(float a, float b) { return __int_as_float(__float_as_int(a) & __float_as_int(b)); }
__device__ __forceinline__ float bits_or(float a, float b) { return __int_as_float(__float_as_int(a) | __float_as_int(b)); }
__device__ __forceinline__ double bits_and(double a, double b) {
  return __longlong_as_double(__double_as_longlong(a) & __double_as_longlong(b));
}
__device__ __forceinline__ double bits_or(double a, double b) {
  return __longlong_as_double(__double_as_longlong(a) | __double_as_longlong(b));
}

// ---- binary operators -----------------------------------------------------------
template <int OP, typename T>
__device__ __forceinline__ T bop(T x, T y) {
  if constexpr (OP == SRHIP_BOP_ADD) return x + y;
  else if constexpr (OP == SRHIP_BOP_SUB) return x - y;
  else if constexpr (OP == SRHIP_BOP_MUL) return x * y;
  else if constexpr (OP == SRHIP_BOP_DIV) return x / y;
  else if constexpr (OP == SRHIP_BOP_POW) return safe_pow(x, y);
  else if constexpr (OP == SRHIP_BOP_GREATER) return x > y ? T(1) : T(0);
  else if constexpr (OP == SRHIP_BOP_LOGICAL_OR) return (x > T(0) || y > T(0)) ? T(1) : T(0);
  else if constexpr (OP == SRHIP_BOP_LOGICAL_AND) return (x > T(0) && y > T(0)) ? T(1) : T(0);
  else if constexpr (OP == SRHIP_BOP_MOD) return jl_mod(x, y);
  else if constexpr (OP == SRHIP_BOP_MAX) {
    const T e = bits_and(x, y);
    const T m = (x > y) ? x : y;
    return (x == y) ? e : m;
  } else if constexpr (OP == SRHIP_BOP_MIN) {
    const T e = bits_or(x, y);
    const T m = (x < y) ? x : y;
    return (x == y) ? e : m;
  } else {
    static_assert(OP < SRHIP_NUM_BOPS, "unknown binary op");
    return x;
  }
}

// ---- unary operators --------------------------------------------------------------
template <int OP, typename T>
__device__ __forceinline__ T uop(T x) {
  if constexpr (OP == SRHIP_UOP_NEG) return -x;
  else if constexpr (OP == SRHIP_UOP_SQUARE) return x * x;
  else if constexpr (OP == SRHIP_UOP_CUBE) return (x * x) * x;
  else if constexpr (OP == SRHIP_UOP_EXP) return m_exp(x);
  else if constexpr (OP == SRHIP_UOP_ABS) return m_fabs(x);
  else if constexpr (OP == SRHIP_UOP_LOG) { T v = m_log(x); return x <= T(0) ? qnan<T>() : v; }
  else if constexpr (OP == SRHIP_UOP_LOG2) { T v = m_log2(x); return x <= T(0) ? qnan<T>() : v; }
  else if constexpr (OP == SRHIP_UOP_LOG10) { T v = m_log10(x); return x <= T(0) ? qnan<T>() : v; }
  else if constexpr (OP == SRHIP_UOP_LOG1P) { T v = m_log1p(x); return x <= T(-1) ? qnan<T>() : v; }
  else if constexpr (OP == SRHIP_UOP_SQRT) { T v = m_sqrt(x); return x < T(0) ? qnan<T>() : v; }
  else if constexpr (OP == SRHIP_UOP_SIN) return m_sin(x);
  else if constexpr (OP == SRHIP_UOP_COS) return m_cos(x);
  else if constexpr (OP == SRHIP_UOP_TAN) return m_tan(x);
  else if constexpr (OP == SRHIP_UOP_SINH) return m_sinh(x);
  else if constexpr (OP == SRHIP_UOP_COSH) return m_cosh(x);
  else if constexpr (OP == SRHIP_UOP_TANH) return m_tanh(x);
  else if constexpr (OP == SRHIP_UOP_ATAN) return m_atan(x);
  else if constexpr (OP == SRHIP_UOP_ASINH) return m_asinh(x);
  else if constexpr (OP == SRHIP_UOP_ACOSH) { T v = m_acosh(x); return x < T(1) ? qnan<T>() : v; }
  else if constexpr (OP == SRHIP_UOP_ATANH_CLIP) return m_atanh(jl_mod(x + T(1), T(2)) - T(1));
  else if constexpr (OP == SRHIP_UOP_ERF) return m_erf(x);
  else if constexpr (OP == SRHIP_UOP_ERFC) return m_erfc(x);
  else if constexpr (OP == SRHIP_UOP_GAMMA) { T g = m_tgamma(x); return m_isinf(g) ? qnan<T>() : g; }
  else if constexpr (OP == SRHIP_UOP_RELU) return (x + m_fabs(x)) * T(0.5);  // == /2 exactly
  else if constexpr (OP == SRHIP_UOP_ROUND) return m_rint(x);
  else if constexpr (OP == SRHIP_UOP_FLOOR) return m_floor(x);
  else if constexpr (OP == SRHIP_UOP_CEIL) return m_ceil(x);
  else if constexpr (OP == SRHIP_UOP_SIGN) return x > T(0) ? T(1) : (x < T(0) ? T(-1) : x);
  else if constexpr (OP == SRHIP_UOP_INV) return T(1) / x;
  else {
    static_assert(OP < SRHIP_NUM_UOPS, "unknown unary op");
    return x;
  }
}

// ---- elementwise losses, r = ŷ - y -------------------------------------------------
// r = ŷ - y in T (LossFunctions' DistanceLoss: value(L, output - target)).
// L2, L1, LogCosh and LogitDist have no parameter and stay in T (abs2 / abs of
// the T residual). The parametric losses hold a Float64 field (LPDistLoss's P,
// HuberLoss's d, the ε / τ / k of the others; src/Options.jl:429-435 builds them
// from Float64 literals), so Julia promotes a Float32 residual to Float64 and
// evaluates them in Float64: so do these, with the parameter as given (never
// rounded to T), and the value rounded to T once.
// |r|^p of LPDistLoss for a Float32 residual (p its Float64 field): exp(p ln|r|)
// in Float64, relative error within ~2^-44 for |p ln|r|| < 700 — far inside
// the one rounding of the loss to Float32, which it changes only for values
// within that distance of a Float32 rounding boundary — with pow's values at
// |r| = 0 and 1. The Float32 tree code's loss routine fits its registers
// (gen_jit.py; the general pow does not); Float64 data keep pow.
__device__ __forceinline__ double lp_pow(double ar, double p) {
  if (ar == 1.0) return 1.0;
  if (ar == 0.0) return p > 0.0 ? 0.0 : (p == 0.0 ? 1.0 : __builtin_inf());
  return m_exp(p * m_log(ar));
}
template <typename T>
__device__ __forceinline__ double lp_pow_t(double ar, double p) {
  if constexpr (std::is_same<T, float>::value) return lp_pow(ar, p);
  else return m_pow(ar, p);
}

// cos(x) in Float64 for |x| <= kCwCosMax: x - n·π/2 by Cody-Waite in three
// parts (33 + 33 + 53 bits of π/2, exact products for |n| < 2^20), then the
// quadrant's cos / sin polynomial (Taylor to r^18 / r^19 on |r| <= π/4,
// truncation below 2^-56). A few ulp of a double, so one rounding to Float32
// matches the correctly rounded value but within ~2^-28 of a boundary. No
// large-argument reduction: `big` reports |x| > kCwCosMax (the value is then
// unspecified) — the Float32 Periodic loss routine of the tree code hands
// such a tile back to the interpreter, which takes OCML's cos there.
constexpr double kCwCosMax = 1.6e6;  // < 2^20 · π/2
// qshift 0: cos x; 3: sin x = cos(x - π/2), the quadrant index one lower
__device__ __forceinline__ double cw_trig(double x, bool& big, int qshift) {
  big = !(__builtin_fabs(x) <= kCwCosMax);
  const double n = __builtin_rint(x * 6.36619772367581382433e-01);  // 2/π
  double r = __builtin_fma(-n, 1.57079632673412561417e+00, x);
  r = __builtin_fma(-n, 6.07710050630396597660e-11, r);
  r = __builtin_fma(-n, 2.02226624879595063154e-21, r);
  const double z = r * r;
  double c = 1.5619206968586225e-16;  // 1/18!
  c = __builtin_fma(c, z, -4.7794773323873853e-14);
  c = __builtin_fma(c, z, 1.1470745597729725e-11);
  c = __builtin_fma(c, z, -2.0876756987868099e-09);
  c = __builtin_fma(c, z, 2.7557319223985891e-07);
  c = __builtin_fma(c, z, -2.4801587301587302e-05);
  c = __builtin_fma(c, z, 1.3888888888888889e-03);
  c = __builtin_fma(c, z, -4.1666666666666664e-02);
  c = __builtin_fma(c, z, 0.5);
  c = __builtin_fma(-c, z, 1.0);
  double sn = 8.2206352466243295e-18;  // 1/19!
  sn = __builtin_fma(sn, z, -2.8114572543455206e-15);
  sn = __builtin_fma(sn, z, 7.6471637318198164e-13);
  sn = __builtin_fma(sn, z, -1.6059043836821613e-10);
  sn = __builtin_fma(sn, z, 2.5052108385441720e-08);
  sn = __builtin_fma(sn, z, -2.7557319223985893e-06);
  sn = __builtin_fma(sn, z, 1.9841269841269841e-04);
  sn = __builtin_fma(sn, z, -8.3333333333333332e-03);
  sn = __builtin_fma(sn, z, 1.6666666666666666e-01);
  sn = __builtin_fma(-sn * z, r, r);
  const int q = (int)(((long long)n + qshift) & 3);
  const double v = (q & 1) ? sn : c;
  return (q == 1 || q == 2) ? -v : v;
}
__device__ __forceinline__ double cw_cos(double x, bool& big) { return cw_trig(x, big, 0); }
// Float32 data's PeriodicLoss value, 1 - cos(r·k), k = 2π/c (LossFunctions'
// PeriodicLoss stores k); the interpreter's and, but for a tile with some
// |r·k| > kCwCosMax (handed back), the tree code's
__device__ __forceinline__ double periodic_f32(double r, double p) {
  const double x = r * (6.28318530717958647692 / p);
  bool big;
  const double c = cw_cos(x, big);
  return 1.0 - (big ? m_cos(x) : c);
}

// LPDistLoss's dℓ/dr of Float64 data for the Float64 gradient tree code
// (gen_jit64.py d_lp): elem_dloss's p·|r|^(p-1)·sign(r) bit for bit, written so
// that only the pow's own temporaries are live (r is the routine's operand
// register, p an SGPR pair): ×sign(r) is copysign for r ≠ 0, and ×0 at r = 0
// (NaN when |r|^(p-1) is Inf, as Julia's P * abs(r)^(P-1) * sign(r))
__device__ __forceinline__ double lp_dloss_f64(double a, double p) {
  // p - 1 made wave-uniform (readfirstlane of both halves), so that the pow's exponent stays in SGPRs
  const unsigned long long b = __builtin_bit_cast(unsigned long long, p - 1.0);
  const double pm1 = __builtin_bit_cast(
      double, ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(b >> 32)) << 32) |
                  (unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)b));
  const double v = p * m_pow(__builtin_fabs(a), pm1);
  return a == 0.0 ? v * 0.0 : __builtin_copysign(v, a);
}

// Float32 data's PeriodicLoss for the gradient tree code (jit_grad.cpp, routines
// g_periodic / d_periodic of gen_jit.py): ℓ = 1 - cos(r·k) or ℓ' = k·sin(r·k),
// k = 2π/c, by the Cody-Waite routine (the interpreter's values but within
// ~2^-28 of a Float32 rounding boundary). A row beyond its range (|r·k| >
// kCwCosMax) gives NaN: the tree "fails" in the tree code and the host reruns
// every failed tree of the call in the forward-mode interpreter (api.cpp
// eval_loss_grad_impl), whose OCML sin / cos reduce fl(r·k) exactly — the
// gradient code's form of the loss tree code's hand-back.
__device__ __forceinline__ double periodic_g_f32(double r, double p, bool deriv) {
  const double k = 6.28318530717958647692 / p;
  bool big;
  const double v = cw_trig(r * k, big, deriv ? 3 : 0);
  if (big) return __builtin_nan("");
  return deriv ? k * v : 1.0 - v;
}

// |r|^n of LPDistLoss{n} for an INTEGER n (SRHIP_LOSS_LPINT). Julia's
// ^(::Float32, ::Integer) and ^(::Float64, ::Integer) (Base math.jl, Julia
// 1.9+; earlier Julias differ, so parity is unpinned): Float32 stays in
// Float32 — 1/x squared for n = -2, x*x*x for n = 3 (literal_pow's), otherwise
// Base.power_by_squaring in Float64 (of 1/x for n < 0) rounded once; Float64
// by pow_body: power by squaring carrying each product's error (two_mul by
// fma), x*x*x for n = 3, (1/x)^2 for n = -2.
__device__ __forceinline__ double pow_by_squaring(double x, long long p) {  // p >= 0
  if (p == 0) return 1.0;
  if (p == 1) return x;
  if (p == 2) return x * x;
  int t = __builtin_ctzll((unsigned long long)p) + 1;
  p >>= t;
  while (--t > 0) x = x * x;
  double y = x;
  while (p > 0) {
    t = __builtin_ctzll((unsigned long long)p) + 1;
    p >>= t;
    while (--t >= 0) x = x * x;
    y = y * x;
  }
  return y;
}
__device__ __forceinline__ float ipow(float x, long long n) {
  if (n == -2) { const float i = 1.0f / x; return i * i; }
  if (n == 3) return x * x * x;
  if (n < 0) return (float)pow_by_squaring(1.0 / (double)x, -n);
  return (float)pow_by_squaring((double)x, n);
}
__device__ __forceinline__ double ipow(double x, long long n) {
  if (n == 0) return 1.0;
  if (n == 3) return x * x * x;
  double xlo = 0.0, y = 1.0, ylo = 0.0;
  if (n < 0) {
    const double rx = 1.0 / x;
    if (n == -2) return rx * rx;
    if (__builtin_isfinite(x)) xlo = -__builtin_fma(x, rx, -1.0) * rx;
    x = rx;
    n = -n;
  }
  while (n > 1) {
    if (n & 1) {
      const double err = __builtin_fma(y, xlo, x * ylo);
      const double h = x * y;
      ylo = __builtin_fma(x, y, -h) + err;
      y = h;
    }
    const double err = x * 2.0 * xlo;
    const double h = x * x;
    xlo = __builtin_fma(x, x, -h) + err;
    x = h;
    n >>= 1;
  }
  const double err = __builtin_fma(y, xlo, x * ylo);
  return (__builtin_isfinite(x) && __builtin_isfinite(err)) ? __builtin_fma(x, y, err) : x * y;
}

template <typename T>
__device__ __forceinline__ double elem_loss_param(int kind, double p, double r) {
  const double ar = __builtin_fabs(r);
  switch (kind) {
    case SRHIP_LOSS_LP: return lp_pow_t<T>(ar, p);
    case SRHIP_LOSS_HUBER: return ar <= p ? 0.5 * r * r : p * (ar - 0.5 * p);
    case SRHIP_LOSS_L1EPSINS: return ar > p ? ar - p : 0.0;
    case SRHIP_LOSS_L2EPSINS: { double e = ar > p ? ar - p : 0.0; return e * e; }
    case SRHIP_LOSS_QUANTILE: return r >= 0.0 ? p * r : (p - 1.0) * r;
    // LossFunctions' PeriodicLoss stores k = 2π/c and evaluates 1 - cos(r·k)
    case SRHIP_LOSS_PERIODIC:
      if constexpr (std::is_same<T, float>::value) return periodic_f32(r, p);
      else return 1.0 - m_cos(r * (6.28318530717958647692 / p));
  }
  return qnan<double>();
}
template <typename T>
__device__ __forceinline__ T elem_loss(int kind, double p, T yhat, T y) {
  const T r = yhat - y;
  const T ar = m_fabs(r);
  switch (kind) {
    case SRHIP_LOSS_L2: return r * r;
    case SRHIP_LOSS_L1: return ar;
    case SRHIP_LOSS_LOGCOSH: return ar + m_log1p(m_exp(T(-2) * ar)) - T(0.69314718055994530942);
    case SRHIP_LOSS_LOGITDIST: return ar + T(2) * m_log1p(m_exp(-ar)) - T(1.38629436111989061883);
    case SRHIP_LOSS_LPINT: return ipow(ar, (long long)p);  // T^Integer stays in T
  }
  return (T)elem_loss_param<T>(kind, p, (double)r);
}

// ---- forward-mode partial derivatives (constant gradients) -----------------------
// f = op(x, y) exactly as bop/uop compute it, plus ∂f/∂x, ∂f/∂y. The rules are
// the textbook ones that Zygote/ForwardDiff derive for these functions;
// piecewise-constant operators (greater, logical_*, round, floor, ceil, sign)
// have zero derivative, gamma's (digamma) is not provided (0).
template <int OP, typename T>
__device__ __forceinline__ void bop_d(T x, T y, T& f, T& fx, T& fy) {
  f = bop<OP>(x, y);
  if constexpr (OP == SRHIP_BOP_ADD) { fx = T(1); fy = T(1); }
  else if constexpr (OP == SRHIP_BOP_SUB) { fx = T(1); fy = T(-1); }
  else if constexpr (OP == SRHIP_BOP_MUL) { fx = y; fy = x; }
  else if constexpr (OP == SRHIP_BOP_DIV) {
    if constexpr (sizeof(T) == 4) {  // v_rcp_f32 (1 ulp): derivatives need no IEEE quotient
      const T ry = __builtin_amdgcn_rcpf(y);
      fx = ry;
      fy = -f * ry;
    } else {
      fx = T(1) / y;
      fy = -x / (y * y);
    }
  }
  else if constexpr (OP == SRHIP_BOP_POW) {
    fx = y * safe_pow(x, y - T(1));
    fy = x > T(0) ? f * m_log(x) : T(0);
  } else if constexpr (OP == SRHIP_BOP_MOD) { fx = T(1); fy = -m_floor(x / y); }
  else if constexpr (OP == SRHIP_BOP_MAX) { fx = x >= y ? T(1) : T(0); fy = x >= y ? T(0) : T(1); }
  else if constexpr (OP == SRHIP_BOP_MIN) { fx = x <= y ? T(1) : T(0); fy = x <= y ? T(0) : T(1); }
  else { fx = T(0); fy = T(0); }
}

template <int OP, typename T>
__device__ __forceinline__ void uop_d(T x, T& f, T& fx) {
  f = uop<OP>(x);
  if constexpr (OP == SRHIP_UOP_NEG) fx = T(-1);
  else if constexpr (OP == SRHIP_UOP_SQUARE) fx = T(2) * x;
  else if constexpr (OP == SRHIP_UOP_CUBE) fx = T(3) * x * x;
  else if constexpr (OP == SRHIP_UOP_EXP) fx = f;
  else if constexpr (OP == SRHIP_UOP_ABS) fx = x > T(0) ? T(1) : (x < T(0) ? T(-1) : T(0));
  else if constexpr (OP == SRHIP_UOP_LOG) fx = T(1) / x;
  else if constexpr (OP == SRHIP_UOP_LOG2) fx = T(1) / (x * T(0.69314718055994530942));
  else if constexpr (OP == SRHIP_UOP_LOG10) fx = T(1) / (x * T(2.30258509299404568402));
  else if constexpr (OP == SRHIP_UOP_LOG1P) fx = T(1) / (T(1) + x);
  else if constexpr (OP == SRHIP_UOP_SQRT) fx = T(0.5) / f;
  else if constexpr (OP == SRHIP_UOP_SIN) {
    if constexpr (sizeof(T) == 4) fx = d_sincos_f32(x, 1);
    else fx = m_cos(x);
  } else if constexpr (OP == SRHIP_UOP_COS) {
    if constexpr (sizeof(T) == 4) fx = -d_sincos_f32(x, 0);
    else fx = -m_sin(x);
  }
  else if constexpr (OP == SRHIP_UOP_TAN) { T c = m_cos(x); fx = T(1) / (c * c); }
  else if constexpr (OP == SRHIP_UOP_SINH) fx = m_cosh(x);
  else if constexpr (OP == SRHIP_UOP_COSH) fx = m_sinh(x);
  else if constexpr (OP == SRHIP_UOP_TANH) fx = T(1) - f * f;
  else if constexpr (OP == SRHIP_UOP_ATAN) fx = T(1) / (T(1) + x * x);
  else if constexpr (OP == SRHIP_UOP_ASINH) fx = T(1) / m_sqrt(x * x + T(1));
  else if constexpr (OP == SRHIP_UOP_ACOSH) fx = T(1) / m_sqrt(x * x - T(1));
  else if constexpr (OP == SRHIP_UOP_ERF) fx = T(1.1283791670955126) * m_exp(-x * x);
  else if constexpr (OP == SRHIP_UOP_ERFC) fx = T(-1.1283791670955126) * m_exp(-x * x);
  else if constexpr (OP == SRHIP_UOP_RELU) fx = x > T(0) ? T(1) : T(0);
  else if constexpr (OP == SRHIP_UOP_INV) fx = T(-1) / (x * x);
  else fx = T(0);
}

// dℓ/dŷ of the elementwise losses (r = ŷ - y); the parametric ones in
// Float64 like their values (elem_loss)
template <typename T>
__device__ __forceinline__ T elem_dloss(int kind, double p, T yhat, T y) {
  const T r = yhat - y;
  const T sg = r > T(0) ? T(1) : (r < T(0) ? T(-1) : T(0));
  switch (kind) {
    case SRHIP_LOSS_L2: return T(2) * r;
    case SRHIP_LOSS_L1: return sg;
    case SRHIP_LOSS_LOGCOSH: return m_tanh(r);
    case SRHIP_LOSS_LOGITDIST: return m_tanh(T(0.5) * r);
    case SRHIP_LOSS_LPINT: {  // LossFunctions' deriv: P * abs(r)^(P-1) * sign(r), in T
      const long long n = (long long)p;
      return T(n) * ipow(m_fabs(r), n - 1) * sg;
    }
  }
  const double rd = (double)r, ar = __builtin_fabs(rd), sd = (double)sg;
  switch (kind) {
    case SRHIP_LOSS_LP: return (T)(p * lp_pow_t<T>(ar, p - 1.0) * sd);
    case SRHIP_LOSS_HUBER: return (T)(ar <= p ? rd : p * sd);
    case SRHIP_LOSS_L1EPSINS: return (T)(ar > p ? sd : 0.0);
    case SRHIP_LOSS_L2EPSINS: return (T)(ar > p ? 2.0 * (ar - p) * sd : 0.0);
    case SRHIP_LOSS_QUANTILE: return (T)(rd >= 0.0 ? p : p - 1.0);
    case SRHIP_LOSS_PERIODIC: { const double k = 6.28318530717958647692 / p; return (T)(k * m_sin(k * rd)); }
  }
  return qnan<T>();
}

}  // namespace dev
}  // namespace srhip
