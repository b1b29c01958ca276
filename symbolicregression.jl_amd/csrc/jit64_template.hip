// jit64_template.hip — the code object that carries Float64 tree code (jit64.cpp).
//
// The Float64 counterpart of jit_template.hip: built once (make) into a
// standalone gfx950 code object, embedded in libsrhip.so, copied and patched
// per program. Kernels:
//   sr_jit64_routines  never launched: the Float64 operator routines of
//                      gen_jit64.py (one region: Float64 has no FAST path);
//   sr_jit64_area      never launched: s_endpgm, then the code area;
//   sr_jit64_eval(_w), sr_jit64_eval_dl(w) (the hand-written tree loop), sr_jit64_out
//                      (per-row outputs)  the driver: one workgroup = (row group, tree group) as
//                      in eval_kernel.h, the row group staged tile-major
//                      ([tile][y, x_0 .. x_{F-1}, w][128 rows of Float64], the
//                      1 KiB per column of the Float32 tiles), each tree one call
//                      of its code.
#include <hip/hip_runtime.h>

#include "interp.h"
#include "kernels.h"
#include "gen/jit64_layout.h"
#include "gen/jit64_routines.inc"

#ifndef SR_JIT64_AREA_WORDS
#define SR_JIT64_AREA_WORDS "1048576"
#endif

using namespace srhip;
using namespace srhip::interp;

extern "C" __global__ void __launch_bounds__(64) sr_jit64_routines() { asm volatile(SR_JIT64_ROUTINES_TEXT); }

extern "C" __global__ void __launch_bounds__(64) sr_jit64_area() {
  asm volatile("s_endpgm\n.globl sr_jit64_code\n.hidden sr_jit64_code\nsr_jit64_code:\n.fill " SR_JIT64_AREA_WORDS
               ", 4, 0xbf810000\n");
}

namespace {
constexpr int R64 = 2;           // rows per lane
constexpr int TILE64 = 64 * R64;  // rows per tile
}  // namespace

struct Jit64Args {
  EvalArgs<double> e;
  const int32_t* code_off;  // [nlist] byte offset of each slot's tree code in the area
  int nraw;                 // feature columns staged (the largest feature the code reads + 1)
};

// OUT: per-row output tree code (srhip_eval_tree_array): no y column is
// staged, no failure flags are read or set (every tile of every tree is
// evaluated, as the interpreter's MODE_OUT does), and each tree's code gets
// its output rows of this row group in s[92:93] (jit64.cpp T_OUT).
template <bool W, bool OUT = false>
__device__ __forceinline__ void jit64_eval_body(const Jit64Args& ja) {
  const EvalArgs<double>& a = ja.e;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* sX = reinterpret_cast<double*>(smem);
  const int narr = 1 + ja.nraw + (W ? 1 : 0);
  const int rows = a.ntiles * TILE64;
  const int rg = blockIdx.x / a.ntg;
  const int g = blockIdx.x - rg * a.ntg;
  const int64_t row0 = (int64_t)rg * rows;
  const int nthreads = __builtin_amdgcn_readfirstlane((int)blockDim.x);
  // 1. stage the row group tile-major: tile t, array k (0 = y, 1 .. nraw = x_{k-1}, last = w)
  {
    constexpr int V = TILE64 / 2;  // double2 per array per tile
    const int total = a.ntiles * narr * V;
    for (int idx = threadIdx.x; idx < total; idx += nthreads) {
      const int v = idx % V;
      const int tk = idx / V;
      const int k = tk % narr;
      const int t = tk / narr;
      if (OUT && k == 0) continue;  // no y
      const double* src = k == 0 ? a.y : (k <= ja.nraw ? a.X + (size_t)(k - 1) * a.n_pad : a.w);
      reinterpret_cast<double2*>(sX + (size_t)tk * TILE64)[v] =
          reinterpret_cast<const double2*>(src + row0 + (int64_t)t * TILE64)[v];
    }
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int64_t rem = a.n - row0;
  const int nt_valid = (int)min((int64_t)a.ntiles, (rem + TILE64 - 1) / TILE64);
  const int last_valid = (int)(rem - (int64_t)(nt_valid - 1) * TILE64);
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int nwaves = nthreads >> 6;
  auto slot_of = [&](int i) { return i * a.ntg + ((i & 1) ? (a.ntg - 1 - g) : g); };
  auto code_of = [&](int s) {
    return __builtin_amdgcn_readfirstlane(((const __attribute__((address_space(4))) int32_t*)(ja.code_off))[s]);
  };
  auto ld_flag = [&](int slot) {
    return OUT ? 0u : __hip_atomic_load(a.fail + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  uint64_t area;
  asm volatile(
      "s_getpc_b64 s[88:89]\n"
      "s_add_u32 s88, s88, sr_jit64_code@rel32@lo+4\n"
      "s_addc_u32 s89, s89, sr_jit64_code@rel32@hi+12"
      : "={s[88:89]}"(area)
      :
      : "scc");  // s_add / s_addc: a carry chain of the compiler must not span this
  const uint32_t lds_lane = (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) double*)sX) +
                            (uint32_t)lane * 16u;
  const uint32_t tilebytes = (uint32_t)(narr * TILE64 * 8);
  const uint32_t woff = W ? (uint32_t)((1 + ja.nraw) * TILE64 * 8) : 0u;
  const uint32_t lane2 = (uint32_t)lane * R64;
  const uint32_t partial = (uint32_t)last_valid;
  const uint32_t nt_u = (uint32_t)nt_valid;
  Part<double>* dst = a.partial + (size_t)rg * ((size_t)a.ntg * a.tpb) + (size_t)g * a.tpb;

  int m = wave < a.tpb ? (a.tpb - wave + nwaves - 1) / nwaves : 0;
  while (m > 0 && slot_of(wave + (m - 1) * nwaves) >= a.nlist) --m;
  m = __builtin_amdgcn_readfirstlane(m);
  uint32_t fnext = m > 0 ? ld_flag(slot_of(wave)) : 0u;
  for (int k = 0; k < m; ++k) {
    const int i = __builtin_amdgcn_readfirstlane(wave + k * nwaves);
    const int s = __builtin_amdgcn_readfirstlane(slot_of(i));
    const bool more = k + 1 < m;
    const bool skip = __builtin_amdgcn_readfirstlane((int)fnext) != 0;
    if (more) fnext = ld_flag(slot_of(wave + (k + 1) * nwaves));
    double lsum = 0.0, chk = skip ? __builtin_nan("") : 0.0;
    if (!skip) {
      const uint64_t target = area + (uint32_t)code_of(s);
      uint32_t la = lds_lane;
      uint32_t tile = 0, status;
      if constexpr (OUT) {  // the tree's output rows of this row group
        const int t = __builtin_amdgcn_readfirstlane(a.list[s]);
        uint64_t optr = reinterpret_cast<uint64_t>(a.out + (size_t)t * (size_t)a.out_stride + row0);
        asm volatile("s_swappc_b64 s[76:77], %[tgt]"
                     : "+{v[44:45]}"(lsum), "+{v[40:41]}"(chk), "+{v42}"(la), "+{s64}"(tile), "={s69}"(status),
                       "+{s[92:93]}"(optr)
                     : [tgt] "s"(target), "{v43}"(lane2), "{s65}"(nt_u), "{s66}"(partial), "{s67}"(tilebytes),
                       "{s68}"(woff)
                     : SR_JIT64_CLOBBERS, "memory");
      } else {
        asm volatile("s_swappc_b64 s[76:77], %[tgt]"
                     : "+{v[44:45]}"(lsum), "+{v[40:41]}"(chk), "+{v42}"(la), "+{s64}"(tile), "={s69}"(status)
                     : [tgt] "s"(target), "{v43}"(lane2), "{s65}"(nt_u), "{s66}"(partial), "{s67}"(tilebytes),
                       "{s68}"(woff)
                     : SR_JIT64_CLOBBERS, "memory");
      }
      (void)status;
    }
    lsum = wave_sum(lsum);
    chk = __builtin_amdgcn_ballot_w64(chk != chk) != 0 ? __builtin_nan("") : 0.0;
    if (lane == 0) dst[i] = Part<double>{lsum, chk};
    if (!OUT && !skip && chk != chk && lane == 0)
      __hip_atomic_store(a.fail + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// The Float64 tree loop written by hand, as jit_template.hip SR_JIT_LOOP_TEXT
// (the waves take their trees from an LDS counter). Registers outside the
// Float64 tree code's (gen_jit64.py SR_JIT64_CLOBBERS): v88 the lane's LDS
// tile address, v89 the counter's LDS address, s46 tpb, s47 ntg, s48 g, s49
// ntg-1-g, s50 nlist, s[52:53] failure flags, s[54:55] code offsets, s[56:57]
// the group's partials (Part<double>, 16 bytes), s[88:89] the code area;
// return s[94:95]; temps s58-s63, s[96:97], v0-v3, v90-v92. The wave sum is
// wave_sum<double>'s: v + dpp(v) per step on both halves, in Float64.
#define SR_JIT64_DPP_STEP(CTRL)                                                       \
  "s_nop 1\n"                                                                         \
  "v_mov_b32_dpp v0, v2 " CTRL " bank_mask:0xf\n"                                    \
  "v_mov_b32_dpp v1, v3 " CTRL " bank_mask:0xf\n"                                    \
  "v_add_f64 v[2:3], v[2:3], v[0:1]\n"
#define SR_JIT64_LOOP_TEXT                                                            \
  ".globl sr_jit64_loop\n.hidden sr_jit64_loop\n.p2align 6\nsr_jit64_loop:\n"         \
  "v_mov_b32_e32 v90, 1\n"                                                            \
  ".Lsr64_next:\n"                                                                    \
  "s_mov_b64 s[96:97], exec\n"                                                        \
  "s_mov_b64 exec, 1\n"                                                               \
  "ds_add_rtn_u32 v91, v89, v90\n"                                                    \
  "s_waitcnt lgkmcnt(0)\n"                                                            \
  "s_mov_b64 exec, s[96:97]\n"                                                        \
  "v_readlane_b32 s60, v91, 0\n"                                                      \
  "s_cmp_ge_u32 s60, s46\n"                                                           \
  "s_cbranch_scc1 .Lsr64_done\n"                                                      \
  "s_mul_i32 s61, s60, s47\n"                                                         \
  "s_bitcmp1_b32 s60, 0\n"                                                            \
  "s_cselect_b32 s62, s49, s48\n"                                                     \
  "s_add_u32 s61, s61, s62\n"                                                         \
  "s_cmp_ge_u32 s61, s50\n"                                                           \
  "s_cbranch_scc1 .Lsr64_done\n"                                                      \
  "s_lshl_b32 s62, s61, 2\n"                                                          \
  "v_mov_b32_e32 v91, s62\n"                                                          \
  "global_load_dword v92, v91, s[52:53] sc1\n"                                        \
  "s_load_dword s63, s[54:55], s62\n"                                                 \
  "s_waitcnt vmcnt(0) lgkmcnt(0)\n"                                                   \
  "v_readfirstlane_b32 s62, v92\n"                                                    \
  "s_cmp_lg_u32 s62, 0\n"                                                             \
  "s_cbranch_scc1 .Lsr64_skip\n"                                                      \
  "s_add_u32 s96, s88, s63\n"                                                         \
  "s_addc_u32 s97, s89, 0\n"                                                          \
  "v_mov_b32_e32 v42, v88\n"                                                          \
  "v_mov_b32_e32 v44, 0\n"                                                            \
  "v_mov_b32_e32 v45, 0\n"                                                            \
  "v_mov_b32_e32 v40, 0\n"                                                            \
  "v_mov_b32_e32 v41, 0\n"                                                            \
  "s_mov_b32 s64, 0\n"                                                                \
  "s_swappc_b64 s[76:77], s[96:97]\n"                                                 \
  "v_mov_b32_e32 v90, 1\n"                                                            \
  "v_cmp_u_f64_e32 vcc, v[40:41], v[40:41]\n"                                         \
  "v_mov_b32_e32 v2, v44\n"                                                           \
  "v_mov_b32_e32 v3, v45\n"                                                           \
  SR_JIT64_DPP_STEP("quad_perm:[1,0,3,2] row_mask:0xf")                               \
  SR_JIT64_DPP_STEP("quad_perm:[2,3,0,1] row_mask:0xf")                               \
  SR_JIT64_DPP_STEP("row_half_mirror row_mask:0xf")                                   \
  SR_JIT64_DPP_STEP("row_mirror row_mask:0xf")                                        \
  "v_mov_b32_e32 v0, 0\n"                                                             \
  "v_mov_b32_e32 v1, 0\n"                                                             \
  SR_JIT64_DPP_STEP("row_bcast:15 row_mask:0xa")                                      \
  "v_mov_b32_e32 v0, 0\n"                                                             \
  "v_mov_b32_e32 v1, 0\n"                                                             \
  SR_JIT64_DPP_STEP("row_bcast:31 row_mask:0xc")                                      \
  "s_nop 1\n"                                                                         \
  "v_readlane_b32 s62, v2, 63\n"                                                      \
  "v_readlane_b32 s63, v3, 63\n"                                                      \
  "s_cmp_lg_u64 vcc, 0\n"                                                             \
  "s_cselect_b32 s59, 0x7ff80000, 0\n"                                                \
  "s_mov_b64 s[96:97], exec\n"                                                        \
  "s_mov_b64 exec, 1\n"                                                               \
  "v_mov_b32_e32 v0, s62\n"                                                           \
  "v_mov_b32_e32 v1, s63\n"                                                           \
  "v_mov_b32_e32 v2, 0\n"                                                             \
  "v_mov_b32_e32 v3, s59\n"                                                           \
  "s_lshl_b32 s62, s60, 4\n"                                                          \
  "v_mov_b32_e32 v91, s62\n"                                                          \
  "global_store_dwordx4 v91, v[0:3], s[56:57]\n"                                      \
  "s_cmp_eq_u32 s59, 0\n"                                                             \
  "s_cbranch_scc1 .Lsr64_nf\n"                                                        \
  "s_lshl_b32 s62, s61, 2\n"                                                          \
  "v_mov_b32_e32 v91, s62\n"                                                          \
  "global_store_dword v91, v90, s[52:53] sc1\n"                                       \
  ".Lsr64_nf:\n"                                                                      \
  "s_mov_b64 exec, s[96:97]\n"                                                        \
  "s_branch .Lsr64_next\n"                                                            \
  ".Lsr64_skip:\n"                                                                    \
  "s_mov_b64 s[96:97], exec\n"                                                        \
  "s_mov_b64 exec, 1\n"                                                               \
  "v_mov_b32_e32 v0, 0\n"                                                             \
  "v_mov_b32_e32 v1, 0\n"                                                             \
  "v_mov_b32_e32 v2, 0\n"                                                             \
  "v_mov_b32_e32 v3, 0x7ff80000\n"                                                    \
  "s_lshl_b32 s62, s60, 4\n"                                                          \
  "v_mov_b32_e32 v91, s62\n"                                                          \
  "global_store_dwordx4 v91, v[0:3], s[56:57]\n"                                      \
  "s_mov_b64 exec, s[96:97]\n"                                                        \
  "s_branch .Lsr64_next\n"                                                            \
  ".Lsr64_done:\n"                                                                    \
  "s_waitcnt vmcnt(0) lgkmcnt(0)\n"                                                   \
  "s_setpc_b64 s[94:95]\n"

extern "C" __global__ void __launch_bounds__(64) sr_jit64_loop_holder() { asm volatile("s_endpgm\n" SR_JIT64_LOOP_TEXT); }

template <bool W>
__device__ __forceinline__ void jit64_eval_dl_body(const Jit64Args& ja) {
  const EvalArgs<double>& a = ja.e;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* sX = reinterpret_cast<double*>(smem);
  const int narr = 1 + ja.nraw + (W ? 1 : 0);
  const int rows = a.ntiles * TILE64;
  const int rg = blockIdx.x / a.ntg;
  const int g = blockIdx.x - rg * a.ntg;
  const int64_t row0 = (int64_t)rg * rows;
  const int nthreads = __builtin_amdgcn_readfirstlane((int)blockDim.x);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(sX + (size_t)narr * rows);  // launch64 adds 16 bytes
  {
    constexpr int V = TILE64 / 2;
    const int total = a.ntiles * narr * V;
    for (int idx = threadIdx.x; idx < total; idx += nthreads) {
      const int v = idx % V;
      const int tk = idx / V;
      const int k = tk % narr;
      const int t = tk / narr;
      const double* src = k == 0 ? a.y : (k <= ja.nraw ? a.X + (size_t)(k - 1) * a.n_pad : a.w);
      reinterpret_cast<double2*>(sX + (size_t)tk * TILE64)[v] =
          reinterpret_cast<const double2*>(src + row0 + (int64_t)t * TILE64)[v];
    }
    if (threadIdx.x == 0) *cnt = 0u;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t rem = a.n - row0;
  const int nt_valid = (int)min((int64_t)a.ntiles, (rem + TILE64 - 1) / TILE64);
  const int last_valid = (int)(rem - (int64_t)(nt_valid - 1) * TILE64);
  uint64_t area;
  asm volatile(
      "s_getpc_b64 s[88:89]\n"
      "s_add_u32 s88, s88, sr_jit64_code@rel32@lo+4\n"
      "s_addc_u32 s89, s89, sr_jit64_code@rel32@hi+12"
      : "={s[88:89]}"(area)
      :
      : "scc");
  const uint32_t lds_lane = (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) double*)sX) +
                            (uint32_t)lane * 16u;
  const uint32_t cnt_addr = (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) uint32_t*)cnt);
  const uint32_t tilebytes = (uint32_t)(narr * TILE64 * 8);
  const uint32_t woff = W ? (uint32_t)((1 + ja.nraw) * TILE64 * 8) : 0u;
  const uint32_t lane2 = (uint32_t)lane * R64;
  const uint32_t partial = (uint32_t)last_valid;
  const uint32_t nt_u = (uint32_t)nt_valid;
  const uint32_t tpb = (uint32_t)a.tpb, ntg = (uint32_t)a.ntg, gg = (uint32_t)g, g1 = (uint32_t)(a.ntg - 1 - g);
  const uint32_t nlist = (uint32_t)a.nlist;
  const uint64_t failp = reinterpret_cast<uint64_t>(a.fail), codep = reinterpret_cast<uint64_t>(ja.code_off);
  const uint64_t dstp = reinterpret_cast<uint64_t>(a.partial + (size_t)rg * ((size_t)a.ntg * a.tpb) + (size_t)g * a.tpb);
  asm volatile(
      "s_getpc_b64 s[96:97]\n"
      "s_add_u32 s96, s96, sr_jit64_loop@rel32@lo+4\n"
      "s_addc_u32 s97, s97, sr_jit64_loop@rel32@hi+12\n"
      "s_swappc_b64 s[94:95], s[96:97]"
      :
      : "{v88}"(lds_lane), "{v89}"(cnt_addr), "{v43}"(lane2), "{s65}"(nt_u), "{s66}"(partial), "{s67}"(tilebytes),
        "{s68}"(woff), "{s46}"(tpb), "{s47}"(ntg), "{s48}"(gg), "{s49}"(g1), "{s50}"(nlist), "{s[52:53]}"(failp),
        "{s[54:55]}"(codep), "{s[56:57]}"(dstp), "{s[88:89]}"(area)
      : SR_JIT64_CLOBBERS, "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s69", "s94", "s95", "s96", "s97",
        "v40", "v41", "v42", "v44", "v45", "v90", "v91", "v92", "memory");
}
// ---- Float64 gradient tree code (jit64.cpp GradGen64) ------------------------------
// One workgroup = (row group, tree group) as sr_jit64_eval; each tree's code
// runs the forward and the reverse pass of every tile, leaves Σ w·r² in LSUM
// and the marker in CHK, and itself stores Σ_rows ∂L/∂c_j of each of its
// constants (summed over the wave) to this row group's partials (gpart).
struct Jit64GradArgs {
  EvalArgs<double> e;
  const int32_t* code_off;  // [nlist] byte offset of each slot's gradient code
  const double* consts;     // [total constants + 16] the program's constants
  const int32_t* cbase;     // [nlist] first constant of the slot's tree
  double* gpart;            // [nrg][nconst] per-row-group ∂L/∂c
  int nconst;
  int nraw;                 // feature columns staged
};

template <bool W>
__device__ __forceinline__ void jit64_grad_body(const Jit64GradArgs& ja) {
  const EvalArgs<double>& a = ja.e;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* sX = reinterpret_cast<double*>(smem);
  const int narr = 1 + ja.nraw + (W ? 1 : 0);
  const int rows = a.ntiles * TILE64;
  const int rg = blockIdx.x / a.ntg;
  const int g = blockIdx.x - rg * a.ntg;
  const int64_t row0 = (int64_t)rg * rows;
  const int nthreads = __builtin_amdgcn_readfirstlane((int)blockDim.x);
  {
    constexpr int V = TILE64 / 2;
    const int total = a.ntiles * narr * V;
    for (int idx = threadIdx.x; idx < total; idx += nthreads) {
      const int v = idx % V;
      const int tk = idx / V;
      const int k = tk % narr;
      const int t = tk / narr;
      const double* src = k == 0 ? a.y : (k <= ja.nraw ? a.X + (size_t)(k - 1) * a.n_pad : a.w);
      reinterpret_cast<double2*>(sX + (size_t)tk * TILE64)[v] =
          reinterpret_cast<const double2*>(src + row0 + (int64_t)t * TILE64)[v];
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t rem = a.n - row0;
  const int nt_valid = (int)min((int64_t)a.ntiles, (rem + TILE64 - 1) / TILE64);
  const int last_valid = (int)(rem - (int64_t)(nt_valid - 1) * TILE64);
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int nwaves = nthreads >> 6;
  auto slot_of = [&](int i) { return i * a.ntg + ((i & 1) ? (a.ntg - 1 - g) : g); };
  auto sld = [&](const int32_t* p, int s) {
    return __builtin_amdgcn_readfirstlane(((const __attribute__((address_space(4))) int32_t*)(p))[s]);
  };
  auto ld_flag = [&](int slot) { return __hip_atomic_load(a.fail + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  uint64_t area;
  asm volatile(
      "s_getpc_b64 s[88:89]\n"
      "s_add_u32 s88, s88, sr_jit64_code@rel32@lo+4\n"
      "s_addc_u32 s89, s89, sr_jit64_code@rel32@hi+12"
      : "={s[88:89]}"(area)
      :
      : "scc");  // s_add / s_addc: a carry chain of the compiler must not span this
  const uint32_t lds_lane = (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) double*)sX) +
                            (uint32_t)lane * 16u;
  const uint32_t tilebytes = (uint32_t)(narr * TILE64 * 8);
  const uint32_t woff = W ? (uint32_t)((1 + ja.nraw) * TILE64 * 8) : 0u;
  const uint32_t lane2 = (uint32_t)lane * R64;
  const uint32_t partial = (uint32_t)last_valid;
  const uint32_t nt_u = (uint32_t)nt_valid;
  Part<double>* dst = a.partial + (size_t)rg * ((size_t)a.ntg * a.tpb) + (size_t)g * a.tpb;
  double* gdst = ja.gpart + (size_t)rg * (size_t)ja.nconst;

  int m = wave < a.tpb ? (a.tpb - wave + nwaves - 1) / nwaves : 0;
  while (m > 0 && slot_of(wave + (m - 1) * nwaves) >= a.nlist) --m;
  m = __builtin_amdgcn_readfirstlane(m);
  uint32_t fnext = m > 0 ? ld_flag(slot_of(wave)) : 0u;
  for (int k = 0; k < m; ++k) {
    const int i = __builtin_amdgcn_readfirstlane(wave + k * nwaves);
    const int s = __builtin_amdgcn_readfirstlane(slot_of(i));
    const bool more = k + 1 < m;
    const bool skip = __builtin_amdgcn_readfirstlane((int)fnext) != 0;
    if (more) fnext = ld_flag(slot_of(wave + (k + 1) * nwaves));
    double lsum = 0.0, chk = skip ? __builtin_nan("") : 0.0;
    if (!skip) {
      const int cb = sld(ja.cbase, s);
      const uint64_t target = area + (uint32_t)sld(ja.code_off, s);
      const uint64_t cptr = reinterpret_cast<uint64_t>(ja.consts + cb);
      const uint64_t gptr = reinterpret_cast<uint64_t>(gdst + cb);
      uint32_t la = lds_lane;
      uint32_t tile = 0, status;
      asm volatile("s_swappc_b64 s[76:77], %[tgt]"
                   : "+{v[44:45]}"(lsum), "+{v[40:41]}"(chk), "+{v42}"(la), "+{s64}"(tile), "={s69}"(status)
                   : [tgt] "s"(target), "{v43}"(lane2), "{s65}"(nt_u), "{s66}"(partial), "{s67}"(tilebytes),
                     "{s68}"(woff), "{s[78:79]}"(cptr), "{s[84:85]}"(gptr)
                   : SR_JIT64_GRAD_CLOBBERS, "memory");
      (void)status;
    }
    // a skipped or failed tree's ∂L/∂c partials are not read (finalize marks it failed)
    lsum = wave_sum(lsum);
    chk = __builtin_amdgcn_ballot_w64(chk != chk) != 0 ? __builtin_nan("") : 0.0;
    if (lane == 0) dst[i] = Part<double>{lsum, chk};
    if (!skip && chk != chk && lane == 0)
      __hip_atomic_store(a.fail + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
extern "C" __global__ void __launch_bounds__(256) sr_jit64_grad(Jit64GradArgs ja) { jit64_grad_body<false>(ja); }
extern "C" __global__ void __launch_bounds__(256) sr_jit64_grad_w(Jit64GradArgs ja) { jit64_grad_body<true>(ja); }

// The Float64 gradient tree code's loop, hand-written as SR_JIT64_LOOP_TEXT
// (the waves of a workgroup take their trees from an LDS counter: NaN-heavy
// batches end most trees early). Registers as there, except: v200 / v201 the
// lane's LDS tile / the counter's address, temps v202-v204 (above the
// gradient code's registers, gen_jit64.py SR_JIT64_GRAD_CLOBBERS); s[92:93]
// this row group's ∂L/∂c partials, s[98:99] the slots' first constants
// (cbase), s[100:101] the constants; per tree s[78:79] = constants + 8·cbase,
// s[84:85] = partials + 8·cbase (the gradient code's inputs), s91 a temp.
#define SR_JIT64_GLOOP_TEXT                                                           \
  ".globl sr_jit64_gloop\n.hidden sr_jit64_gloop\n.p2align 6\nsr_jit64_gloop:\n"     \
  "v_mov_b32_e32 v202, 1\n"                                                           \
  ".Lsr64g_next:\n"                                                                   \
  "s_mov_b64 s[96:97], exec\n"                                                        \
  "s_mov_b64 exec, 1\n"                                                               \
  "ds_add_rtn_u32 v203, v201, v202\n"                                                 \
  "s_waitcnt lgkmcnt(0)\n"                                                            \
  "s_mov_b64 exec, s[96:97]\n"                                                        \
  "v_readlane_b32 s60, v203, 0\n"                                                     \
  "s_cmp_ge_u32 s60, s46\n"                                                           \
  "s_cbranch_scc1 .Lsr64g_done\n"                                                     \
  "s_mul_i32 s61, s60, s47\n"                                                         \
  "s_bitcmp1_b32 s60, 0\n"                                                            \
  "s_cselect_b32 s62, s49, s48\n"                                                     \
  "s_add_u32 s61, s61, s62\n"                                                         \
  "s_cmp_ge_u32 s61, s50\n"                                                           \
  "s_cbranch_scc1 .Lsr64g_done\n"                                                     \
  "s_lshl_b32 s62, s61, 2\n"                                                          \
  "v_mov_b32_e32 v203, s62\n"                                                         \
  "global_load_dword v204, v203, s[52:53] sc1\n"                                      \
  "s_load_dword s63, s[54:55], s62\n"                                                 \
  "s_load_dword s91, s[98:99], s62\n"                                                 \
  "s_waitcnt vmcnt(0) lgkmcnt(0)\n"                                                   \
  "v_readfirstlane_b32 s62, v204\n"                                                   \
  "s_cmp_lg_u32 s62, 0\n"                                                             \
  "s_cbranch_scc1 .Lsr64g_skip\n"                                                     \
  "s_add_u32 s96, s88, s63\n"                                                         \
  "s_addc_u32 s97, s89, 0\n"                                                          \
  "s_lshl_b32 s62, s91, 3\n"                                                          \
  "s_add_u32 s78, s100, s62\n"                                                        \
  "s_addc_u32 s79, s101, 0\n"                                                         \
  "s_add_u32 s84, s92, s62\n"                                                         \
  "s_addc_u32 s85, s93, 0\n"                                                          \
  "v_mov_b32_e32 v42, v200\n"                                                         \
  "v_mov_b32_e32 v44, 0\n"                                                            \
  "v_mov_b32_e32 v45, 0\n"                                                            \
  "v_mov_b32_e32 v40, 0\n"                                                            \
  "v_mov_b32_e32 v41, 0\n"                                                            \
  "s_mov_b32 s64, 0\n"                                                                \
  "s_swappc_b64 s[76:77], s[96:97]\n"                                                 \
  "v_mov_b32_e32 v202, 1\n"                                                           \
  "v_cmp_u_f64_e32 vcc, v[40:41], v[40:41]\n"                                         \
  "v_mov_b32_e32 v2, v44\n"                                                           \
  "v_mov_b32_e32 v3, v45\n"                                                           \
  SR_JIT64_DPP_STEP("quad_perm:[1,0,3,2] row_mask:0xf")                               \
  SR_JIT64_DPP_STEP("quad_perm:[2,3,0,1] row_mask:0xf")                               \
  SR_JIT64_DPP_STEP("row_half_mirror row_mask:0xf")                                   \
  SR_JIT64_DPP_STEP("row_mirror row_mask:0xf")                                        \
  "v_mov_b32_e32 v0, 0\n"                                                             \
  "v_mov_b32_e32 v1, 0\n"                                                             \
  SR_JIT64_DPP_STEP("row_bcast:15 row_mask:0xa")                                      \
  "v_mov_b32_e32 v0, 0\n"                                                             \
  "v_mov_b32_e32 v1, 0\n"                                                             \
  SR_JIT64_DPP_STEP("row_bcast:31 row_mask:0xc")                                      \
  "s_nop 1\n"                                                                         \
  "v_readlane_b32 s62, v2, 63\n"                                                      \
  "v_readlane_b32 s63, v3, 63\n"                                                      \
  "s_cmp_lg_u64 vcc, 0\n"                                                             \
  "s_cselect_b32 s59, 0x7ff80000, 0\n"                                                \
  "s_mov_b64 s[96:97], exec\n"                                                        \
  "s_mov_b64 exec, 1\n"                                                               \
  "v_mov_b32_e32 v0, s62\n"                                                           \
  "v_mov_b32_e32 v1, s63\n"                                                           \
  "v_mov_b32_e32 v2, 0\n"                                                             \
  "v_mov_b32_e32 v3, s59\n"                                                           \
  "s_lshl_b32 s62, s60, 4\n"                                                          \
  "v_mov_b32_e32 v203, s62\n"                                                         \
  "global_store_dwordx4 v203, v[0:3], s[56:57]\n"                                     \
  "s_cmp_eq_u32 s59, 0\n"                                                             \
  "s_cbranch_scc1 .Lsr64g_nf\n"                                                       \
  "s_lshl_b32 s62, s61, 2\n"                                                          \
  "v_mov_b32_e32 v203, s62\n"                                                         \
  "global_store_dword v203, v202, s[52:53] sc1\n"                                     \
  ".Lsr64g_nf:\n"                                                                     \
  "s_mov_b64 exec, s[96:97]\n"                                                        \
  "s_branch .Lsr64g_next\n"                                                           \
  ".Lsr64g_skip:\n"                                                                   \
  "s_mov_b64 s[96:97], exec\n"                                                        \
  "s_mov_b64 exec, 1\n"                                                               \
  "v_mov_b32_e32 v0, 0\n"                                                             \
  "v_mov_b32_e32 v1, 0\n"                                                             \
  "v_mov_b32_e32 v2, 0\n"                                                             \
  "v_mov_b32_e32 v3, 0x7ff80000\n"                                                    \
  "s_lshl_b32 s62, s60, 4\n"                                                          \
  "v_mov_b32_e32 v203, s62\n"                                                         \
  "global_store_dwordx4 v203, v[0:3], s[56:57]\n"                                     \
  "s_mov_b64 exec, s[96:97]\n"                                                        \
  "s_branch .Lsr64g_next\n"                                                           \
  ".Lsr64g_done:\n"                                                                   \
  "s_waitcnt vmcnt(0) lgkmcnt(0)\n"                                                   \
  "s_setpc_b64 s[94:95]\n"

extern "C" __global__ void __launch_bounds__(64) sr_jit64_gloop_holder() { asm volatile("s_endpgm\n" SR_JIT64_GLOOP_TEXT); }

template <bool W>
__device__ __forceinline__ void jit64_grad_dl_body(const Jit64GradArgs& ja) {
  const EvalArgs<double>& a = ja.e;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* sX = reinterpret_cast<double*>(smem);
  const int narr = 1 + ja.nraw + (W ? 1 : 0);
  const int rows = a.ntiles * TILE64;
  const int rg = blockIdx.x / a.ntg;
  const int g = blockIdx.x - rg * a.ntg;
  const int64_t row0 = (int64_t)rg * rows;
  const int nthreads = __builtin_amdgcn_readfirstlane((int)blockDim.x);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(sX + (size_t)narr * rows);  // launch_grad_code64 adds 16 bytes
  {
    constexpr int V = TILE64 / 2;
    const int total = a.ntiles * narr * V;
    for (int idx = threadIdx.x; idx < total; idx += nthreads) {
      const int v = idx % V;
      const int tk = idx / V;
      const int k = tk % narr;
      const int t = tk / narr;
      const double* src = k == 0 ? a.y : (k <= ja.nraw ? a.X + (size_t)(k - 1) * a.n_pad : a.w);
      reinterpret_cast<double2*>(sX + (size_t)tk * TILE64)[v] =
          reinterpret_cast<const double2*>(src + row0 + (int64_t)t * TILE64)[v];
    }
    if (threadIdx.x == 0) *cnt = 0u;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t rem = a.n - row0;
  const int nt_valid = (int)min((int64_t)a.ntiles, (rem + TILE64 - 1) / TILE64);
  const int last_valid = (int)(rem - (int64_t)(nt_valid - 1) * TILE64);
  uint64_t area;
  asm volatile(
      "s_getpc_b64 s[88:89]\n"
      "s_add_u32 s88, s88, sr_jit64_code@rel32@lo+4\n"
      "s_addc_u32 s89, s89, sr_jit64_code@rel32@hi+12"
      : "={s[88:89]}"(area)
      :
      : "scc");
  const uint32_t lds_lane = (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) double*)sX) +
                            (uint32_t)lane * 16u;
  const uint32_t cnt_addr = (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) uint32_t*)cnt);
  const uint32_t tilebytes = (uint32_t)(narr * TILE64 * 8);
  const uint32_t woff = W ? (uint32_t)((1 + ja.nraw) * TILE64 * 8) : 0u;
  const uint32_t lane2 = (uint32_t)lane * R64;
  const uint32_t partial = (uint32_t)last_valid;
  const uint32_t nt_u = (uint32_t)nt_valid;
  const uint32_t tpb = (uint32_t)a.tpb, ntg = (uint32_t)a.ntg, gg = (uint32_t)g, g1 = (uint32_t)(a.ntg - 1 - g);
  const uint32_t nlist = (uint32_t)a.nlist;
  const uint64_t failp = reinterpret_cast<uint64_t>(a.fail), codep = reinterpret_cast<uint64_t>(ja.code_off);
  const uint64_t dstp = reinterpret_cast<uint64_t>(a.partial + (size_t)rg * ((size_t)a.ntg * a.tpb) + (size_t)g * a.tpb);
  const uint64_t gdstp = reinterpret_cast<uint64_t>(ja.gpart + (size_t)rg * (size_t)ja.nconst);
  const uint64_t cbp = reinterpret_cast<uint64_t>(ja.cbase), constp = reinterpret_cast<uint64_t>(ja.consts);
  asm volatile(
      "s_getpc_b64 s[96:97]\n"
      "s_add_u32 s96, s96, sr_jit64_gloop@rel32@lo+4\n"
      "s_addc_u32 s97, s97, sr_jit64_gloop@rel32@hi+12\n"
      "s_swappc_b64 s[94:95], s[96:97]"
      :
      : "{v200}"(lds_lane), "{v201}"(cnt_addr), "{v43}"(lane2), "{s65}"(nt_u), "{s66}"(partial), "{s67}"(tilebytes),
        "{s68}"(woff), "{s46}"(tpb), "{s47}"(ntg), "{s48}"(gg), "{s49}"(g1), "{s50}"(nlist), "{s[52:53]}"(failp),
        "{s[54:55]}"(codep), "{s[56:57]}"(dstp), "{s[88:89]}"(area), "{s[92:93]}"(gdstp), "{s[98:99]}"(cbp),
        "{s[100:101]}"(constp)
      : SR_JIT64_GRAD_CLOBBERS, "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s69", "s78", "s79", "s84", "s85",
        "s91", "s94", "s95", "s96", "s97", "v40", "v41", "v42", "v44", "v45", "v202", "v203", "v204", "memory");
}
extern "C" __global__ void __launch_bounds__(256) sr_jit64_grad_dl(Jit64GradArgs ja) { jit64_grad_dl_body<false>(ja); }
extern "C" __global__ void __launch_bounds__(256) sr_jit64_grad_dlw(Jit64GradArgs ja) { jit64_grad_dl_body<true>(ja); }

extern "C" __global__ void __launch_bounds__(1024) sr_jit64_eval_dl(Jit64Args ja) { jit64_eval_dl_body<false>(ja); }
extern "C" __global__ void __launch_bounds__(1024) sr_jit64_eval_dlw(Jit64Args ja) { jit64_eval_dl_body<true>(ja); }
extern "C" __global__ void __launch_bounds__(1024) sr_jit64_eval(Jit64Args ja) { jit64_eval_body<false>(ja); }
extern "C" __global__ void __launch_bounds__(1024) sr_jit64_eval_w(Jit64Args ja) { jit64_eval_body<true>(ja); }
extern "C" __global__ void __launch_bounds__(1024) sr_jit64_out(Jit64Args ja) { jit64_eval_body<false, true>(ja); }
