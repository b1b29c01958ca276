// grad_interp.h — forward-mode (dual number) version of the interpreter, for
// constant gradients (eval_grad_tree_array(...; variable=false),
// src/InterfaceDynamicExpressions.jl:105-107).
//
// Every register carries a value and G tangents: the derivatives with respect
// to the constants c_{g0} .. c_{g0+G-1} of the tree (one "tangent group"; a
// tree with more constants is evaluated once per group). Programs are compiled
// without constant folding and with each constant's index in the slot field
// of the instruction, so a constant operand seeds tangent (index - g0).
#pragma once
#include "interp.h"

namespace srhip {
namespace interp {

template <typename T, int R, int G>
struct Dual {
  T v[R];
  T d[G][R];
};

enum Src : int { S_ACC = 0, S_TMP, S_X, S_X2, S_C };

constexpr int src_l(int v) {
  return v == V_AX ? S_ACC : v == V_XA ? S_X : v == V_AC ? S_ACC : v == V_CA ? S_C
       : v == V_AT ? S_ACC : v == V_TA ? S_TMP : v == V_XX ? S_X : v == V_XC ? S_X : S_C;
}
constexpr int src_r(int v) {
  return v == V_AX ? S_X : v == V_XA ? S_ACC : v == V_AC ? S_C : v == V_CA ? S_ACC
       : v == V_AT ? S_TMP : v == V_TA ? S_ACC : v == V_XX ? S_X2 : v == V_XC ? S_C : S_X;
}
constexpr bool computed(int s) { return s == S_ACC || s == S_TMP; }

template <int U, typename T, int R, int G>
__device__ __forceinline__ void un_grad(Dual<T, R, G>& a, T& chk) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if constexpr (uop_lossy(U)) chk = mark(a.v[r], chk);
    T f, fx;
    dev::uop_d<U>(a.v[r], f, fx);
    a.v[r] = f;
#pragma unroll
    for (int j = 0; j < G; ++j) a.d[j][r] = fx * a.d[j][r];
  }
}

template <int V, int B, typename T, int R, int G>
__device__ __forceinline__ void bin_grad(Dual<T, R, G>& a, const Dual<T, R, G>& t,
                                         const T* __restrict__ sXt, int rs, int lane, int f,
                                         T imm, int jc, T& chk) {
  constexpr int SL = src_l(V), SR = src_r(V);
  constexpr bool LL = bop_lossy_lhs(B), LR = bop_lossy_rhs(B);
  T xa[R], xb[R];
  if constexpr (SL == S_X || SR == S_X) lds_rows<T, R>(sXt + f * rs, lane, xa);
  if constexpr (SR == S_X2) lds_rows<T, R>(sXt + imm_int(imm) * rs, lane, xb);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    T lv, rv;
    if constexpr (SL == S_ACC) lv = a.v[r];
    else if constexpr (SL == S_TMP) lv = t.v[r];
    else if constexpr (SL == S_X) lv = xa[r];
    else lv = imm;
    if constexpr (SR == S_ACC) rv = a.v[r];
    else if constexpr (SR == S_TMP) rv = t.v[r];
    else if constexpr (SR == S_X) rv = xa[r];
    else if constexpr (SR == S_X2) rv = xb[r];
    else rv = imm;
    if constexpr (LL && computed(SL)) chk = mark(lv, chk);
    if constexpr (LR && computed(SR)) chk = mark(rv, chk);
    T fv, fx, fy;
    dev::bop_d<B>(lv, rv, fv, fx, fy);
#pragma unroll
    for (int j = 0; j < G; ++j) {
      T nd = T(0);
      if constexpr (SL == S_ACC) nd = fx * a.d[j][r];
      else if constexpr (SL == S_TMP) nd = fx * t.d[j][r];
      else if constexpr (SL == S_C) nd = (j == jc) ? fx : T(0);
      if constexpr (SR == S_ACC) nd = nd + fy * a.d[j][r];
      else if constexpr (SR == S_TMP) nd = nd + fy * t.d[j][r];
      else if constexpr (SR == S_C) nd = (j == jc) ? nd + fy : nd;
      a.d[j][r] = nd;
    }
    a.v[r] = fv;
  }
}

#define SRG_PUSH(K)                                                      \
  case OP_PUSH0 + K:                                                     \
    if constexpr (K < D) slot[K] = a;                                    \
    break;
#define SRG_POP(K)                                                       \
  case OP_POP0 + K:                                                      \
    if constexpr (K < D) t = slot[K];                                    \
    break;
#define SRG_UN(U) \
  case OP_UN0 + U: if constexpr (opset_has_uop(SET, U)) un_grad<U, T, R, G>(a, chk); break;
#define SRG_BV(V, B) \
  case bin_opcode(V, B): if constexpr (opset_has_bop(SET, B)) bin_grad<V, B, T, R, G>(a, t, sXt, rs, lane, f, imm, jc, chk); break;
#define SRG_BIN(B) SRG_BV(V_AX, B) SRG_BV(V_XA, B) SRG_BV(V_AC, B) SRG_BV(V_CA, B) \
  SRG_BV(V_AT, B) SRG_BV(V_TA, B) SRG_BV(V_XX, B) SRG_BV(V_XC, B) SRG_BV(V_CX, B)

// Run one tree's program over one row tile with tangents for constants
// g0 .. g0+G-1; the result is left in a.
template <typename T, int R, int D, int G, int SET>
__device__ __forceinline__ void run_program_grad(CIns<T>* __restrict__ p,
                                                 const T* __restrict__ sXt, int rs, int lane,
                                                 int g0, Dual<T, R, G>& a, T& chk) {
  Dual<T, R, G> t;
  Dual<T, R, G> slot[D];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    a.v[r] = T(0);
    t.v[r] = T(0);
#pragma unroll
    for (int j = 0; j < G; ++j) { a.d[j][r] = T(0); t.d[j][r] = T(0); }
  }
  Ins<T> cur = fetch<T>(p);
  for (;;) {
    const Ins<T> nxt = fetch<T>(p + 1);
    const uint32_t code = (uint32_t)__builtin_amdgcn_readfirstlane((int)cur.code);
    const T imm = uni(cur.imm);
    const int f = (int)(code >> 16);
    const int jc = (int)((code >> 8) & 0xffu) - g0;  // tangent seeded by a constant operand
    switch (code & 0xffu) {
      case OP_END: return;
      case OP_LDX:
        lds_rows<T, R>(sXt + f * rs, lane, a.v);
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
          for (int j = 0; j < G; ++j) a.d[j][r] = T(0);
        break;
      case OP_LDC:
#pragma unroll
        for (int r = 0; r < R; ++r) {
          a.v[r] = imm;
#pragma unroll
          for (int j = 0; j < G; ++j) a.d[j][r] = (j == jc) ? T(1) : T(0);
        }
        break;
      SRG_PUSH(0) SRG_PUSH(1) SRG_PUSH(2) SRG_PUSH(3) SRG_PUSH(4) SRG_PUSH(5) SRG_PUSH(6) SRG_PUSH(7)
      SRG_PUSH(8) SRG_PUSH(9) SRG_PUSH(10) SRG_PUSH(11) SRG_PUSH(12) SRG_PUSH(13) SRG_PUSH(14) SRG_PUSH(15)
      SRG_POP(0) SRG_POP(1) SRG_POP(2) SRG_POP(3) SRG_POP(4) SRG_POP(5) SRG_POP(6) SRG_POP(7)
      SRG_POP(8) SRG_POP(9) SRG_POP(10) SRG_POP(11) SRG_POP(12) SRG_POP(13) SRG_POP(14) SRG_POP(15)
      SRG_UN(0) SRG_UN(1) SRG_UN(2) SRG_UN(3) SRG_UN(4) SRG_UN(5) SRG_UN(6) SRG_UN(7) SRG_UN(8)
      SRG_UN(9) SRG_UN(10) SRG_UN(11) SRG_UN(12) SRG_UN(13) SRG_UN(14) SRG_UN(15) SRG_UN(16)
      SRG_UN(17) SRG_UN(18) SRG_UN(19) SRG_UN(20) SRG_UN(21) SRG_UN(22) SRG_UN(23) SRG_UN(24)
      SRG_UN(25) SRG_UN(26) SRG_UN(27) SRG_UN(28)
      SRG_BIN(0) SRG_BIN(1) SRG_BIN(2) SRG_BIN(3) SRG_BIN(4) SRG_BIN(5) SRG_BIN(6) SRG_BIN(7)
      SRG_BIN(8) SRG_BIN(9) SRG_BIN(10)
      default: break;
    }
    cur = nxt;
    ++p;
  }
}

}  // namespace interp
}  // namespace srhip
