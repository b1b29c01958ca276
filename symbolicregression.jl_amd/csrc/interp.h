// interp.h — the wave-uniform tree interpreter (device side), shared by the
// evaluation kernels (kernels.hip) and the constant-gradient kernels
// (grad_kernels.hip).
//
// A program is fetched with scalar loads and dispatched with a uniform
// branch tree; each instruction processes R rows per lane held in VGPRs.
// Leaf features are read from the LDS row tile, constants are immediates.
#pragma once
#include <hip/hip_runtime.h>

#include "device_ops.h"
#include "srhip_internal.h"

namespace srhip {
namespace interp {

using dev::bop;
using dev::uop;

// Programs are read through the constant address space so that the uniform
// instruction fetch is a scalar load (s_load) into SGPRs: no vector-memory
// round trip and no readfirstlane on the dispatch path.
template <typename T>
using CIns = const __attribute__((address_space(4))) Ins<T>;
template <typename T>
__device__ __forceinline__ CIns<T>* const_prog(const Ins<T>* p) {
  return (CIns<T>*)(p);
}
template <typename T>
__device__ __forceinline__ Ins<T> fetch(CIns<T>* p) {
  Ins<T> i;
  i.code = p->code;
  i.imm = p->imm;
  return i;
}

template <typename T>
struct V16;
template <>
struct V16<float> {
  using type = float4;
  static constexpr int N = 4;
};
template <>
struct V16<double> {
  using type = double2;
  static constexpr int N = 2;
};

__device__ __forceinline__ float uni(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ double uni(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffll));
  const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ int imm_int(float v) { return __float_as_int(v); }
__device__ __forceinline__ int imm_int(double v) { return (int)(__double_as_longlong(v) & 0xffffffffll); }

// Wave sum without LDS round trips (ds_bpermute): DPP butterflies inside each
// 16-lane row (xor 1, xor 2, half-mirror, mirror), then the four row sums
// read with v_readlane. The result is wave-uniform.
// DPP move of v (lanes of rows outside ROWS get 0, the `old` operand).
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWS, 0xf, false));
}
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ double dpp_f(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTRL, ROWS, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWS, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ float lane_val(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ double lane_val(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
  v += dpp_f<0xB1>(v);         // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);         // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);        // row_half_mirror
  v += dpp_f<0x140>(v);        // row_mirror: every lane holds its row's sum
  v += dpp_f<0x142, 0xa>(v);   // row_bcast:15 -> rows 1, 3: r0+r1, r2+r3
  v += dpp_f<0x143, 0xc>(v);   // row_bcast:31 -> rows 2, 3: lane 63 = r0+r1+r2+r3
  return lane_val(v, 63);
}

// Non-finite marker: fma(v, 0, chk) is NaN iff v is ±Inf or NaN.
__device__ __forceinline__ float mark(float v, float chk) { return __builtin_fmaf(v, 0.0f, chk); }
__device__ __forceinline__ double mark(double v, double chk) { return __builtin_fma(v, 0.0, chk); }

// The R rows of this lane inside one LDS tile row: element e = c*N + i is
// tile row (c*64 + lane)*N + i, so every ds_read_b128 of a wave reads one
// contiguous 1 KiB (conflict-free).
// Vector width used for a lane's R rows: 16 bytes, or R elements if fewer.
template <typename T, int R>
struct RowVec {
  static constexpr int W = (R < V16<T>::N) ? R : V16<T>::N;
};

template <typename T, int R>
__device__ __forceinline__ int row_of(int e, int lane) {
  constexpr int W = RowVec<T, R>::W;
  return ((e / W) * 64 + lane) * W + (e % W);
}

template <typename T, int R>
__device__ __forceinline__ void lds_rows(const T* __restrict__ p, int lane, T (&v)[R]) {
  constexpr int W = RowVec<T, R>::W;
  static_assert(R % W == 0, "R must be a multiple of the row vector width");
#pragma unroll
  for (int c = 0; c < R / W; ++c) {
    const T* q = p + (c * 64 + lane) * W;
    if constexpr (W * sizeof(T) == 16) {
      using V = typename V16<T>::type;
      const V a = *reinterpret_cast<const V*>(q);
      if constexpr (W == 4) {
        v[c * 4 + 0] = a.x; v[c * 4 + 1] = a.y; v[c * 4 + 2] = a.z; v[c * 4 + 3] = a.w;
      } else {
        v[c * 2 + 0] = a.x; v[c * 2 + 1] = a.y;
      }
    } else if constexpr (W == 2) {
      const float2 a = *reinterpret_cast<const float2*>(q);
      v[c * 2 + 0] = a.x; v[c * 2 + 1] = a.y;
    } else {
      v[c] = q[0];
    }
  }
}

template <typename T, int R>
__device__ __forceinline__ void store_rows(T* __restrict__ p, int lane, const T (&v)[R]) {
  constexpr int W = RowVec<T, R>::W;
#pragma unroll
  for (int c = 0; c < R / W; ++c) {
    T* q = p + (c * 64 + lane) * W;
    if constexpr (W * sizeof(T) == 16) {
      using V = typename V16<T>::type;
      V a;
      if constexpr (W == 4) {
        a.x = v[c * 4 + 0]; a.y = v[c * 4 + 1]; a.z = v[c * 4 + 2]; a.w = v[c * 4 + 3];
      } else {
        a.x = v[c * 2 + 0]; a.y = v[c * 2 + 1];
      }
      *reinterpret_cast<V*>(q) = a;
    } else if constexpr (W == 2) {
      *reinterpret_cast<float2*>(q) = make_float2(v[c * 2 + 0], v[c * 2 + 1]);
    } else {
      q[0] = v[c];
    }
  }
}

template <int U, typename T, int R>
__device__ __forceinline__ void un_apply(T (&acc)[R], T& chk) {
  if constexpr ((U == SRHIP_UOP_COS || U == SRHIP_UOP_SIN) && sizeof(T) == 4) {
    // fast f32 sin/cos for all R values, one wave-uniform check for the
    // rare |x| > 105615 that needs the full reduction (device_ops.h
    // big_sincos_f32)
    T v[R];
    float qmax = 0.0f;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float qa;
      v[r] = dev::fast_sincos_f32(acc[r], U == SRHIP_UOP_COS ? 1 : 0, qa);
      qmax = __builtin_fmaxf(qmax, qa);
    }
    if (__builtin_amdgcn_ballot_w64(!(qmax <= dev::kTrigQMax)) != 0) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const T o = dev::big_sincos_f32(acc[r], U == SRHIP_UOP_COS ? 1 : 0);
        v[r] = dev::trig_big(acc[r]) ? o : v[r];
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = v[r];
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if constexpr (uop_lossy(U)) chk = mark(acc[r], chk);
      acc[r] = uop<U>(acc[r]);
    }
  }
}

// x: the instruction's X operand (feature f), already in registers — loaded
// by the driver (prefetched one instruction ahead by run_program_v).
template <int V, int B, typename T, int R>
__device__ __forceinline__ void bin_apply(T (&acc)[R], const T (&tmp)[R], const T (&x)[R],
                                          const T* __restrict__ sXt, int rs,
                                          int lane, T imm, T& chk) {
  constexpr bool LL = bop_lossy_lhs(B);
  constexpr bool LR = bop_lossy_rhs(B);
  if constexpr (V == V_XX) {
    T x2[R];
    lds_rows<T, R>(sXt + imm_int(imm) * rs, lane, x2);
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = bop<B>(x[r], x2[r]);
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if constexpr (V == V_AX) {
        if constexpr (LL) chk = mark(acc[r], chk);
        acc[r] = bop<B>(acc[r], x[r]);
      } else if constexpr (V == V_XA) {
        if constexpr (LR) chk = mark(acc[r], chk);
        acc[r] = bop<B>(x[r], acc[r]);
      } else if constexpr (V == V_XC) {
        acc[r] = bop<B>(x[r], imm);
      } else if constexpr (V == V_CX) {
        acc[r] = bop<B>(imm, x[r]);
      } else if constexpr (V == V_AC) {
        if constexpr (LL) chk = mark(acc[r], chk);
        acc[r] = bop<B>(acc[r], imm);
      } else if constexpr (V == V_CA) {
        if constexpr (LR) chk = mark(acc[r], chk);
        acc[r] = bop<B>(imm, acc[r]);
      } else if constexpr (V == V_AT) {
        if constexpr (LL) chk = mark(acc[r], chk);
        if constexpr (LR) chk = mark(tmp[r], chk);
        acc[r] = bop<B>(acc[r], tmp[r]);
      } else {  // V_TA
        if constexpr (LL) chk = mark(tmp[r], chk);
        if constexpr (LR) chk = mark(acc[r], chk);
        acc[r] = bop<B>(tmp[r], acc[r]);
      }
    }
  }
}

#define SR_UNROLL _Pragma("unroll")
#define SR_PUSH(K)                                                   \
  case OP_PUSH0 + K:                                                 \
    if constexpr (K < D) { SR_UNROLL for (int r = 0; r < R; ++r) slot[K][r] = acc[r]; } \
    break;
#define SR_POP(K)                                                    \
  case OP_POP0 + K:                                                  \
    if constexpr (K < D) { SR_UNROLL for (int r = 0; r < R; ++r) tmp[r] = slot[K][r]; } \
    break;
#define SR_UN(U) \
  case OP_UN0 + U: if constexpr (opset_has_uop(SET, U)) un_apply<U, T, R>(acc, chk); break;
#define SR_BV(V, B) \
  case bin_opcode(V, B): if constexpr (opset_has_bop(SET, B)) bin_apply<V, B, T, R>(acc, tmp, x, sXt, rs, lane, imm, chk); break;
#define SR_BIN(B) SR_BV(V_AX, B) SR_BV(V_XA, B) SR_BV(V_AC, B) SR_BV(V_CA, B) \
  SR_BV(V_AT, B) SR_BV(V_TA, B) SR_BV(V_XX, B) SR_BV(V_XC, B) SR_BV(V_CX, B)

// Execute one instruction (wave-uniform `code`, `imm`); returns false at END.
template <typename T, int R, int D, int SET>
__device__ __forceinline__ bool exec_ins(uint32_t code, T imm, T (&acc)[R], T (&tmp)[R],
                                         T (&slot)[D][R], const T (&x)[R],
                                         const T* __restrict__ sXt, int rs, int lane, T& chk) {
  switch (code & 0xffu) {
    case OP_END: return false;
    case OP_LDX: SR_UNROLL for (int r = 0; r < R; ++r) acc[r] = x[r]; break;
    case OP_LDC: SR_UNROLL for (int r = 0; r < R; ++r) acc[r] = imm; break;
    SR_PUSH(0) SR_PUSH(1) SR_PUSH(2) SR_PUSH(3) SR_PUSH(4) SR_PUSH(5) SR_PUSH(6) SR_PUSH(7)
    SR_PUSH(8) SR_PUSH(9) SR_PUSH(10) SR_PUSH(11) SR_PUSH(12) SR_PUSH(13) SR_PUSH(14) SR_PUSH(15)
    SR_POP(0) SR_POP(1) SR_POP(2) SR_POP(3) SR_POP(4) SR_POP(5) SR_POP(6) SR_POP(7)
    SR_POP(8) SR_POP(9) SR_POP(10) SR_POP(11) SR_POP(12) SR_POP(13) SR_POP(14) SR_POP(15)
    SR_UN(0) SR_UN(1) SR_UN(2) SR_UN(3) SR_UN(4) SR_UN(5) SR_UN(6) SR_UN(7) SR_UN(8) SR_UN(9)
    SR_UN(10) SR_UN(11) SR_UN(12) SR_UN(13) SR_UN(14) SR_UN(15) SR_UN(16) SR_UN(17) SR_UN(18)
    SR_UN(19) SR_UN(20) SR_UN(21) SR_UN(22) SR_UN(23) SR_UN(24) SR_UN(25) SR_UN(26) SR_UN(27)
    SR_UN(28)
    SR_BIN(0) SR_BIN(1) SR_BIN(2) SR_BIN(3) SR_BIN(4) SR_BIN(5) SR_BIN(6) SR_BIN(7) SR_BIN(8)
    SR_BIN(9) SR_BIN(10)
    default: break;
  }
  return true;
}

// Driver 1 (any program length): instructions fetched with scalar loads, one
// ahead; the X operand is read from LDS right before the instruction.
template <typename T, int R, int D, int SET>
__device__ __forceinline__ void run_program(CIns<T>* __restrict__ p,
                                            const T* __restrict__ sXt, int rs,
                                            int lane, T (&acc)[R], T& chk) {
  T tmp[R], x[R];
  T slot[D][R];
#pragma unroll
  for (int r = 0; r < R; ++r) { acc[r] = T(0); tmp[r] = T(0); x[r] = T(0); }
  Ins<T> cur = fetch<T>(p);
  for (;;) {
    const Ins<T> nxt = fetch<T>(p + 1);  // prefetch; every program ends with OP_END + slack
    const uint32_t code = (uint32_t)__builtin_amdgcn_readfirstlane((int)cur.code);
    const T imm = uni(cur.imm);
    if (code & kNeedX) lds_rows<T, R>(sXt + (int)(code >> 16) * rs, lane, x);
    if (!exec_ins<T, R, D, SET>(code, imm, acc, tmp, slot, x, sXt, rs, lane, chk)) return;
    cur = nxt;
    ++p;
  }
}

// A program of at most kVProgMax instructions held in VGPRs: lane j holds
// instruction j (code word and immediate). Loaded once per tree, reused for
// every row tile, read with v_readlane (no memory round trip per dispatch).
template <typename T>
struct VProg;
template <>
struct VProg<float> {
  uint32_t code, imm;
  __device__ __forceinline__ void load(const Ins<float>* p, int lane) {
    const uint2 v = *reinterpret_cast<const uint2*>(p + lane);
    code = v.x; imm = v.y;
  }
  __device__ __forceinline__ uint32_t code_at(int pc) const {
    return (uint32_t)__builtin_amdgcn_readlane((int)code, pc);
  }
  __device__ __forceinline__ float imm_at(int pc) const {
    return __int_as_float(__builtin_amdgcn_readlane((int)imm, pc));
  }
};
template <>
struct VProg<double> {
  uint32_t code, lo, hi;
  __device__ __forceinline__ void load(const Ins<double>* p, int lane) {
    const uint4 v = *reinterpret_cast<const uint4*>(p + lane);
    code = v.x; lo = v.z; hi = v.w;
  }
  __device__ __forceinline__ uint32_t code_at(int pc) const {
    return (uint32_t)__builtin_amdgcn_readlane((int)code, pc);
  }
  __device__ __forceinline__ double imm_at(int pc) const {
    const uint32_t l = (uint32_t)__builtin_amdgcn_readlane((int)lo, pc);
    const uint32_t h = (uint32_t)__builtin_amdgcn_readlane((int)hi, pc);
    return __longlong_as_double((long long)(((uint64_t)h << 32) | l));
  }
};

// Driver 2 (programs of at most kVProgMax instructions): the program is in
// VGPRs and the X operand of the NEXT instruction is read from LDS while the
// dispatch of the current one finishes, so neither the fetch nor the LDS read
// sits on the dispatch path.
template <typename T, int R, int D, int SET>
__device__ __forceinline__ void run_program_v(const VProg<T>& vp, const T* __restrict__ sXt, int rs,
                                              int lane, T (&acc)[R], T& chk) {
  T tmp[R], x[R];
  T slot[D][R];
#pragma unroll
  for (int r = 0; r < R; ++r) { acc[r] = T(0); tmp[r] = T(0); }
  uint32_t code = vp.code_at(0);
  lds_rows<T, R>(sXt + (int)(code >> 16) * rs, lane, x);
  for (int pc = 0;; ++pc) {
    const uint32_t ncode = vp.code_at(pc + 1);
    const T imm = vp.imm_at(pc);
    if (!exec_ins<T, R, D, SET>(code, imm, acc, tmp, slot, x, sXt, rs, lane, chk)) return;
    if (ncode & kNeedX) lds_rows<T, R>(sXt + (int)(ncode >> 16) * rs, lane, x);
    code = ncode;
  }
}
// Driver 3: as driver 2, unrolled by two with ping-pong X buffers so the X
// operand of instruction i+1 is read from LDS before instruction i executes
// (the LDS latency overlaps a whole instruction, not only the dispatch).
template <typename T, int R, int D, int SET>
__device__ __forceinline__ void run_program_v2(const VProg<T>& vp, const T* __restrict__ sXt, int rs,
                                               int lane, T (&acc)[R], T& chk) {
  T tmp[R], xa[R], xb[R];
  T slot[D][R];
#pragma unroll
  for (int r = 0; r < R; ++r) { acc[r] = T(0); tmp[r] = T(0); }
  uint32_t c0 = vp.code_at(0);
  if (c0 & kNeedX) lds_rows<T, R>(sXt + (int)(c0 >> 16) * rs, lane, xa);
  for (int pc = 0;; pc += 2) {
    const uint32_t c1 = vp.code_at(pc + 1);
    if (c1 & kNeedX) lds_rows<T, R>(sXt + (int)(c1 >> 16) * rs, lane, xb);
    if (!exec_ins<T, R, D, SET>(c0, vp.imm_at(pc), acc, tmp, slot, xa, sXt, rs, lane, chk)) return;
    c0 = vp.code_at(pc + 2);
    if (c0 & kNeedX) lds_rows<T, R>(sXt + (int)(c0 >> 16) * rs, lane, xa);
    if (!exec_ins<T, R, D, SET>(c1, vp.imm_at(pc + 1), acc, tmp, slot, xb, sXt, rs, lane, chk)) return;
  }
}
static_assert(SRHIP_NUM_UOPS == 29 && SRHIP_NUM_BOPS == 11, "update the case lists");

}  // namespace interp
}  // namespace srhip
