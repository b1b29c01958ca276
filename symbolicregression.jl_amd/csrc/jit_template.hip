// jit_template.hip — the code object that carries compiled tree code (jit.cpp).
//
// Built once (make) into a standalone gfx950 code object, embedded in
// libsrhip.so, copied and patched per program: jit.cpp writes the machine
// code of every tree into the `sr_jit_code` area and loads the image with
// hipModuleLoadData. Three kernels:
//   sr_jit_routines  never launched: holds the operator routines of
//                    gen_jit.py (FAST and PRECISE regions, same layout);
//   sr_jit_area      never launched: s_endpgm, then the code area (filled
//                    with s_endpgm, so a stray jump ends the wave);
//   sr_jit_eval      the driver: one workgroup = (row group, tree group) as
//                    in eval_kernel (eval_kernel.h), but the row group is
//                    staged tile-major ([tile][y, x_0 .. x_{F-1}, w][256]) so
//                    that tree code addresses every array of a tile with an
//                    immediate offset, and each tree is one call of its code.
// Trees without code run in the interpreter's launch (api.cpp); a tree whose
// code hands a tile back (a sin/cos argument beyond the fast reduction) is
// flagged in `bail` and re-evaluated by the interpreter after this launch.
#include <hip/hip_runtime.h>

#include "interp.h"
#include "kernels.h"
#include "gen/jit_layout_r4.h"
#include "gen/jit_routines_r4.inc"

#ifndef SR_JIT_AREA_WORDS
#define SR_JIT_AREA_WORDS "65536"
#endif

using namespace srhip;
using namespace srhip::interp;

extern "C" __global__ void __launch_bounds__(64) sr_jit_routines() { asm volatile(SR_JIT_ROUTINES_TEXT); }

extern "C" __global__ void __launch_bounds__(64) sr_jit_area() {
  asm volatile("s_endpgm\n.globl sr_jit_code\n.hidden sr_jit_code\nsr_jit_code:\n.fill " SR_JIT_AREA_WORDS ", 4, 0xbf810000\n");
}

namespace {
constexpr int R = SR_JIT_R;
constexpr int TILE = 64 * R;
}  // namespace

// Block → (row group, tree group). Default: rg = b / ntg, g = b % ntg.
// a.rotate == 2 (SRHIP_RG_XCD=1, experiment): blocks are dealt round-robin
// over the 8 XCDs (b % 8 share one), so rg = (b/8 / ntg)·8 + b % 8 and
// g = (b/8) % ntg put every tree group of a row group on the same XCD (its X
// tile is read from HBM once per XCD); the grid is padded to whole octets of
// row groups and the padding blocks return at once.
// a.rotate == 3 (SRHIP_TG_MAJOR=1, experiment): the same XCD deal, but an
// XCD's blocks run tree group by tree group, g = (b/8) / nrg8, rg =
// ((b/8) % nrg8)·8 + b % 8, so the workgroups resident on its CUs share their
// tree code in the instruction cache.
__device__ __forceinline__ bool block_of(const EvalArgs<float>& a, int& rg, int& g) {
  const int b = blockIdx.x;
  if (a.rotate == 3) {
    const int k = b >> 3;
    const int nrg8 = (a.nrg + 7) >> 3;
    g = k / nrg8;
    rg = (k - g * nrg8) * 8 + (b & 7);
    return rg < a.nrg && g < a.ntg;
  }
  if (a.rotate == 2) {
    const int k = b >> 3;
    rg = (k / a.ntg) * 8 + (b & 7);
    g = k % a.ntg;
    return rg < a.nrg;
  }
  rg = b / a.ntg;
  g = b - rg * a.ntg;
  return true;
}

struct JitArgs {
  EvalArgs<float> e;
  const int32_t* code_off;  // [nlist] byte offset of each slot's tree code in the area
  uint32_t* bail;           // [nlist] set when tree code hands a tile back
  uint32_t* counters;       // [0] counts those slots, [1] tiles redone with the PRECISE routines
  int fast;                 // 1: trees may run their FAST-routine path (guarded)
  int part_lds;             // 1: per-tree partials gathered in LDS (after the tiles) and
                            //    written out together at the end; 0: straight to global memory
  int nraw, nder;           // raw feature columns and derived columns (jit.h Columns)
  uint32_t der[48];         // derived column k: (operator << 16) | feature
  const float* dcols;       // [nder][n_pad] the derived columns (sr_jit_derive), or null: staged ones computed here
  int nbig;                 // row groups [0, nbig) hold e.ntiles tiles; the tail row groups after them
  int ts;                   // hold ts tiles each (the last round of workgroups in smaller pieces)
  int dyn;                  // hand-written prefetching loop: a tree redone PRECISE in one row group runs PRECISE in the later ones
  const float* gcols;       // [ngcol][n_pad] shared-subtree columns (jit.h Columns), or null: tree code
                            // reads column g of this row group at s[36:37] + g·s38 (literal code only)
};

// A derived column's value: the PRECISE routine of the operator (the same
// device_ops.h code as the tree code's PRECISE region and the interpreters).
__device__ __forceinline__ float derive_uop(int op, float x) {
  switch (op) {
#define SR_DERIVE_CASE(U) case U: return dev::uop<U>(x);
    SR_DERIVE_CASE(SRHIP_UOP_EXP) SR_DERIVE_CASE(SRHIP_UOP_LOG) SR_DERIVE_CASE(SRHIP_UOP_LOG2)
    SR_DERIVE_CASE(SRHIP_UOP_LOG10) SR_DERIVE_CASE(SRHIP_UOP_LOG1P) SR_DERIVE_CASE(SRHIP_UOP_SQRT)
    SR_DERIVE_CASE(SRHIP_UOP_SIN) SR_DERIVE_CASE(SRHIP_UOP_COS) SR_DERIVE_CASE(SRHIP_UOP_TAN)
    SR_DERIVE_CASE(SRHIP_UOP_SINH) SR_DERIVE_CASE(SRHIP_UOP_COSH) SR_DERIVE_CASE(SRHIP_UOP_TANH)
    SR_DERIVE_CASE(SRHIP_UOP_ATAN) SR_DERIVE_CASE(SRHIP_UOP_ASINH) SR_DERIVE_CASE(SRHIP_UOP_ACOSH)
    SR_DERIVE_CASE(SRHIP_UOP_ATANH_CLIP) SR_DERIVE_CASE(SRHIP_UOP_ERF) SR_DERIVE_CASE(SRHIP_UOP_ERFC)
    SR_DERIVE_CASE(SRHIP_UOP_GAMMA) SR_DERIVE_CASE(SRHIP_UOP_RELU) SR_DERIVE_CASE(SRHIP_UOP_ROUND)
    SR_DERIVE_CASE(SRHIP_UOP_FLOOR) SR_DERIVE_CASE(SRHIP_UOP_CEIL) SR_DERIVE_CASE(SRHIP_UOP_SIGN)
    SR_DERIVE_CASE(SRHIP_UOP_INV)
#undef SR_DERIVE_CASE
    default: return __builtin_nanf("");  // not derivable: jit.cpp never asks
  }
}

// a wave-uniform 64-bit value in an SGPR pair (inline-asm operands pinned to SGPRs)
__device__ __forceinline__ uint64_t sgpr64(uint64_t v) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32);
}

// OUT: per-row output tree code (srhip_eval_tree_array): no y column is
// staged, no failure flags are read or set (every tile of every tree is
// evaluated, as the interpreter's MODE_OUT does), and each tree's code gets
// its output rows of this row group in s[92:93] (jit.cpp S_OUT).
template <bool W, bool MEMC, bool OUT = false, bool DYN = false>
__device__ __forceinline__ void jit_eval_body(const JitArgs& ja) {
  const EvalArgs<float>& a = ja.e;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* sX = reinterpret_cast<float*>(smem);
  const int ncol = ja.nraw + ja.nder;
  const int narr = 1 + ncol + (W ? 1 : 0);
  const int rows = a.ntiles * TILE;  // LDS layout: room for a full row group
  int rg, g;
  if (!block_of(a, rg, g)) return;
  const bool tail = rg >= ja.nbig;
  const int ntl = tail ? ja.ts : a.ntiles;  // tiles of this row group
  const int64_t row0 = tail ? (int64_t)ja.nbig * rows + (int64_t)(rg - ja.nbig) * ja.ts * TILE : (int64_t)rg * rows;
  const int nthreads = __builtin_amdgcn_readfirstlane((int)blockDim.x);
  // per-tree partials: gathered in LDS after the tiles when the host made room
  // for them (few trees per group), else stored straight to global memory
  Part<float>* gdst = a.partial + (size_t)rg * ((size_t)a.ntg * a.tpb) + (size_t)g * a.tpb;
  Part<float>* sPart = reinterpret_cast<Part<float>*>(sX + (size_t)narr * rows);
  Part<float>* dst = ja.part_lds ? sPart : gdst;
  // the tree counter after the tiles (and the partials): launch() adds 16 bytes
  uint32_t* cnt = reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned char*>(sPart) +
                                              (ja.part_lds ? (size_t)a.tpb * sizeof(Part<float>) : 0));

  // 1. stage the row group tile-major: tile t, array k (0 = y, 1 .. nraw =
  //    x_{k-1}, then the derived columns u(x_f), last = w); one wave per
  //    (tile, array), so a derived column's operator is wave-uniform
  {
    constexpr int V = TILE / 4;  // float4 per array per tile
    const int total = ntl * narr * V;
    for (int idx = threadIdx.x; idx < total; idx += nthreads) {
      const int v = idx % V;
      const int tk = idx / V;
      const int k = tk % narr;
      const int t = tk / narr;
      if (OUT && k == 0) continue;  // no y
      if (k > ja.nraw && k <= ncol && ja.dcols) {
        const float* src = ja.dcols + (size_t)(k - 1 - ja.nraw) * a.n_pad;
        reinterpret_cast<float4*>(sX + (size_t)tk * TILE)[v] =
            reinterpret_cast<const float4*>(src + row0 + (int64_t)t * TILE)[v];
        continue;
      }
      if (k > ja.nraw && k <= ncol) {
        const uint32_t d = ja.der[k - 1 - ja.nraw];
        const int op = __builtin_amdgcn_readfirstlane((int)(d >> 16));
        const float4 x = reinterpret_cast<const float4*>(a.X + (size_t)(d & 0xffffu) * a.n_pad + row0 +
                                                         (int64_t)t * TILE)[v];
        reinterpret_cast<float4*>(sX + (size_t)tk * TILE)[v] =
            make_float4(derive_uop(op, x.x), derive_uop(op, x.y), derive_uop(op, x.z), derive_uop(op, x.w));
        continue;
      }
      const float* src = k == 0 ? a.y : (k <= ja.nraw ? a.X + (size_t)(k - 1) * a.n_pad : a.w);
      reinterpret_cast<float4*>(sX + (size_t)tk * TILE)[v] =
          reinterpret_cast<const float4*>(src + row0 + (int64_t)t * TILE)[v];
    }
    if (DYN && threadIdx.x == 0) *cnt = 0u;
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int64_t rem = a.n - row0;
  const int nt_valid = (int)min((int64_t)ntl, (rem + TILE - 1) / TILE);
  const int last_valid = (int)(rem - (int64_t)(nt_valid - 1) * TILE);
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int nwaves = nthreads >> 6;
  auto slot_of = [&](int i) { return a.contig ? g * a.tpb + i : i * a.ntg + ((i & 1) ? (a.ntg - 1 - g) : g); };
  auto code_of = [&](int s) {
    return __builtin_amdgcn_readfirstlane(((const __attribute__((address_space(4))) int32_t*)(ja.code_off))[s]);
  };
  // the slot's program (memory-constant tree code loads its constants from it)
  auto prog_of = [&](int s) {
    return reinterpret_cast<uint64_t>(
        a.prog + __builtin_amdgcn_readfirstlane(((const __attribute__((address_space(4))) int32_t*)(a.list_off))[s]));
  };
  auto ld_flag = [&](int slot) {
    return OUT ? 0u : __hip_atomic_load(a.fail + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };

  // address of the code area (PC-relative, resolved when the image is linked)
  uint64_t area;
  asm volatile(
      "s_getpc_b64 s[88:89]\n"
      "s_add_u32 s88, s88, sr_jit_code@rel32@lo+4\n"
      "s_addc_u32 s89, s89, sr_jit_code@rel32@hi+12"
      : "={s[88:89]}"(area)
      :
      : "scc");  // s_add / s_addc: a carry chain of the compiler must not span this
  const uint32_t lds_lane = (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) float*)sX) +
                            (uint32_t)lane * 16u;
  const uint32_t tilebytes = (uint32_t)(narr * TILE * 4);
  const uint32_t woff = W ? (uint32_t)((1 + ncol) * TILE * 4) : 0u;  // 0: unweighted
  const uint32_t lane4 = (uint32_t)lane * R;
  const uint32_t partial = (uint32_t)last_valid;
  const uint32_t nt_u = (uint32_t)nt_valid;
  const uint32_t fastok = (uint32_t)ja.fast;
  // shared-subtree columns: column 0 at this row group's first row, column stride in bytes
  const uint64_t gcb = sgpr64(ja.gcols ? reinterpret_cast<uint64_t>(ja.gcols + row0) : 0ull);
  const uint32_t gstride = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a.n_pad * 4));

  uint32_t redos = 0;  // tiles redone with the PRECISE routines (counted by tree code)
  // one tree of slot s (list position i) on this row group: its code at coff
  auto run_tree = [&](const int i, const int s, const bool skip, const int32_t coff) {
    float lsum = 0.0f, chk = skip ? __builtin_nanf("") : 0.0f;
    if (!skip) {
      const uint64_t target = area + (uint32_t)coff;
      uint32_t la = lds_lane;
      uint32_t tile = 0, status;
      if constexpr (OUT) {  // the tree's output rows of this row group
        const int t = __builtin_amdgcn_readfirstlane(a.list[s]);
        uint64_t optr = reinterpret_cast<uint64_t>(a.out + (size_t)t * (size_t)a.out_stride + row0);
        if constexpr (MEMC) {
          uint64_t pptr = prog_of(s);
          asm volatile("s_swappc_b64 s[76:77], %[tgt]"
                       : "+{v42}"(lsum), "+{v40}"(chk), "+{v41}"(la), "+{s64}"(tile), "={s69}"(status),
                         "+{s84}"(redos), "+{s[56:57]}"(pptr), "+{s[92:93]}"(optr)
                       : [tgt] "s"(target), "{v43}"(lane4), "{s65}"(nt_u), "{s66}"(partial),
                         "{s67}"(tilebytes), "{s68}"(woff), "{s79}"(fastok)
                       : SR_JIT_CLOBBERS_MEMC, "memory");
        } else {
          asm volatile("s_swappc_b64 s[76:77], %[tgt]"
                       : "+{v42}"(lsum), "+{v40}"(chk), "+{v41}"(la), "+{s64}"(tile), "={s69}"(status),
                         "+{s84}"(redos), "+{s[92:93]}"(optr)
                       : [tgt] "s"(target), "{v43}"(lane4), "{s65}"(nt_u), "{s66}"(partial),
                         "{s67}"(tilebytes), "{s68}"(woff), "{s79}"(fastok)
                       : SR_JIT_CLOBBERS, "memory");
        }
      } else if constexpr (MEMC) {  // memory-constant tree code: its program in s[56:57], constants in s24..s39
        uint64_t pptr = prog_of(s);
        asm volatile("s_swappc_b64 s[76:77], %[tgt]"
                     : "+{v42}"(lsum), "+{v40}"(chk), "+{v41}"(la), "+{s64}"(tile), "={s69}"(status),
                       "+{s84}"(redos), "+{s[56:57]}"(pptr)
                     : [tgt] "s"(target), "{v43}"(lane4), "{s65}"(nt_u), "{s66}"(partial),
                       "{s67}"(tilebytes), "{s68}"(woff), "{s79}"(fastok)
                     : SR_JIT_CLOBBERS_MEMC, "memory");
      } else {
        asm volatile("s_swappc_b64 s[76:77], %[tgt]"
                     : "+{v42}"(lsum), "+{v40}"(chk), "+{v41}"(la), "+{s64}"(tile), "={s69}"(status),
                       "+{s84}"(redos)
                     : [tgt] "s"(target), "{v43}"(lane4), "{s65}"(nt_u), "{s66}"(partial),
                       "{s67}"(tilebytes), "{s68}"(woff), "{s79}"(fastok), "{s[36:37]}"(gcb), "{s38}"(gstride)
                     : SR_JIT_CLOBBERS, "memory");
      }
      if (__builtin_amdgcn_readfirstlane((int)status) != 0) {
        // a tile the routines cannot do (sin/cos argument beyond the fast
        // reduction): the host re-evaluates this tree with the interpreter;
        // the other row groups skip it
        chk = __builtin_nanf("");
        if (lane == 0) {
          __hip_atomic_store(ja.bail + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_add(ja.counters, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    // the marker only has to say whether some row failed: a ballot, not a sum
    lsum = wave_sum(lsum);
    chk = __builtin_amdgcn_ballot_w64(chk != chk) != 0 ? __builtin_nanf("") : 0.0f;
    if (lane == 0) dst[i] = Part<float>{lsum, chk};
    if (!OUT && !skip && chk != chk && lane == 0)
      __hip_atomic_store(a.fail + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  if constexpr (DYN) {
    auto claim = [&]() -> int {
      uint32_t v = 0u;
      if (lane == 0) v = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return __builtin_amdgcn_readfirstlane((int)v);
    };
    auto valid = [&](int i) { return i < a.tpb && slot_of(i) < a.nlist; };
    int i = claim();
    int32_t cnext = valid(i) ? code_of(slot_of(i)) : 0;
    while (valid(i)) {
      const int s = __builtin_amdgcn_readfirstlane(slot_of(i));
      const int inx = claim();
      const int32_t coff = cnext;
      if (valid(inx)) cnext = code_of(slot_of(inx));
      run_tree(i, s, false, coff);
      i = inx;
    }
  } else {
    int m = wave < a.tpb ? (a.tpb - wave + nwaves - 1) / nwaves : 0;
    while (m > 0 && slot_of(wave + (m - 1) * nwaves) >= a.nlist) --m;
    m = __builtin_amdgcn_readfirstlane(m);
    uint32_t fnext = m > 0 ? ld_flag(slot_of(wave)) : 0u;
    // the next slot's code offset is loaded one tree ahead, like its flag
    int32_t cnext = m > 0 ? code_of(slot_of(wave)) : 0;
    for (int k = 0; k < m; ++k) {
      const int i = __builtin_amdgcn_readfirstlane(wave + k * nwaves);
      const int s = __builtin_amdgcn_readfirstlane(slot_of(i));
      const bool more = k + 1 < m;
      const bool skip = __builtin_amdgcn_readfirstlane((int)fnext) != 0;
      const int32_t coff = cnext;
      if (more) {
        fnext = ld_flag(slot_of(wave + (k + 1) * nwaves));
        cnext = code_of(slot_of(wave + (k + 1) * nwaves));
      }
      run_tree(i, s, skip, coff);
    }
  }
  if (lane == 0 && __builtin_amdgcn_readfirstlane((int)redos) != 0)
    __hip_atomic_fetch_add(ja.counters + 1, (uint32_t)__builtin_amdgcn_readfirstlane((int)redos),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (ja.part_lds) {  // slots no wave ran keep whatever: finalize ignores them
    __syncthreads();
    for (int i = threadIdx.x; i < a.tpb; i += nthreads) gdst[i] = sPart[i];
  }
}

// The derived columns of a call, once per row: out[k][r] = u_k(x_{f_k}[r]) for
// r < n_pad (padding rows replicate the last row, as X does).
struct DeriveArgs {
  const float* X;
  int64_t n_pad;
  int nder;
  uint32_t der[48];
  float* out;
};
extern "C" __global__ void __launch_bounds__(256) sr_jit_derive(DeriveArgs da) {
  const int k = blockIdx.y;
  const uint32_t d = da.der[k];
  const int op = (int)(d >> 16);
  const float* x = da.X + (size_t)(d & 0xffffu) * da.n_pad;
  float* o = da.out + (size_t)k * da.n_pad;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < da.n_pad / 4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    reinterpret_cast<float4*>(o)[i] = make_float4(derive_uop(op, v.x), derive_uop(op, v.y), derive_uop(op, v.z),
                                                  derive_uop(op, v.w));
  }
}

extern "C" __global__ void __launch_bounds__(1024) sr_jit_eval(JitArgs ja) { jit_eval_body<false, false>(ja); }
extern "C" __global__ void __launch_bounds__(1024) sr_jit_eval_w(JitArgs ja) { jit_eval_body<true, false>(ja); }
extern "C" __global__ void __launch_bounds__(1024) sr_jit_eval_m(JitArgs ja) { jit_eval_body<false, true>(ja); }
extern "C" __global__ void __launch_bounds__(1024) sr_jit_eval_mw(JitArgs ja) { jit_eval_body<true, true>(ja); }
extern "C" __global__ void __launch_bounds__(1024) sr_jit_out(JitArgs ja) { jit_eval_body<false, false, true>(ja); }
extern "C" __global__ void __launch_bounds__(1024) sr_jit_out_m(JitArgs ja) { jit_eval_body<false, true, true>(ja); }
extern "C" __global__ void __launch_bounds__(1024) sr_jit_out_d(JitArgs ja) { jit_eval_body<false, false, true, true>(ja); }
extern "C" __global__ void __launch_bounds__(1024) sr_jit_out_md(JitArgs ja) { jit_eval_body<false, true, true, true>(ja); }

// ---- the tree loop as hand-written code (sr_jit_eval_dl, SRHIP_JIT_DYNLOOP) -------
// The waves of a workgroup take the group's trees from an LDS counter (one
// ds_add_rtn per tree), so a wave that drew cheap trees takes more and the
// workgroup ends with its waves together. The loop around the tree calls is
// written here, not compiled: the compiler only sets up its fixed registers
// once and never allocates around a tree call (compiled variants of such
// loops broke the driver). Registers (none of them written by
// tree code, gen_jit.py SR_JIT_CLOBBERS):
//   v30 the lane's LDS tile address, v31 the counter's LDS address, v43 lane*R
//   s40 tpb, s41 ntg, s42 g, s43 ntg-1-g, s44 nlist (slots of this part)
//   s[46:47] failure flags, s[48:49] code offsets, s[50:51] this group's
//   global partials, s52 partials in LDS (1) or global (0), s53 their LDS
//   address, s[54:55] bail flags, s[92:93] counters, s[88:89] the code area,
//   memory-constant code (sr_jit_loop_m): s[98:99] the programs, s[100:101]
//   list_off, each tree's program address into s[56:57] (SR_JIT_LOOP_PROG),
//   s65-s68 / s79 / s84 as for the compiled loop; return address s[94:95];
//   temps s58-s63, s96-s97, v0-v2, v89-v91.
// Per tree i (slot s = i*ntg + (i odd ? ntg-1-g : g)): a set failure flag
// skips it (partial {0, NaN}); else its code runs; a bail (s69 != 0) sets the
// slot's bail flag and counts it; the loss is summed over the wave in the
// order of interp.h wave_sum; lane 0 stores the partial {Σ, NaN or 0} and, if
// some row failed, the slot's failure flag (vector stores only).
#define SR_JIT_LOOP_TEXT(NAME, PROG)                                                              \
  ".globl " #NAME "\n.hidden " #NAME "\n.p2align 6\n" #NAME ":\n"               \
  "v_mov_b32_e32 v89, 1\n"                                                            \
  ".L" #NAME "_next:\n"                                                                     \
  "s_mov_b64 s[58:59], exec\n"                                                        \
  "s_mov_b64 exec, 1\n"                                                               \
  "ds_add_rtn_u32 v90, v31, v89\n"                                                    \
  "s_waitcnt lgkmcnt(0)\n"                                                            \
  "s_mov_b64 exec, s[58:59]\n"                                                        \
  "v_readlane_b32 s60, v90, 0\n"                                                      \
  "s_cmp_ge_u32 s60, s40\n"                                                           \
  "s_cbranch_scc1 .L" #NAME "_done\n"                                                       \
  "s_mul_i32 s61, s60, s41\n"                                                         \
  "s_bitcmp1_b32 s60, 0\n"                                                            \
  "s_cselect_b32 s62, s43, s42\n"                                                     \
  "s_add_u32 s61, s61, s62\n"                                                         \
  "s_cmp_ge_u32 s61, s44\n"                                                           \
  "s_cbranch_scc1 .L" #NAME "_done\n"                                                       \
  "s_lshl_b32 s62, s61, 2\n"                                                          \
  "v_mov_b32_e32 v90, s62\n"                                                          \
  "global_load_dword v91, v90, s[46:47] sc1\n"                                        \
  "s_load_dword s63, s[48:49], s62\n"                                                 \
  "s_waitcnt vmcnt(0) lgkmcnt(0)\n"                                                   \
  "v_readfirstlane_b32 s62, v91\n"                                                    \
  "s_cmp_lg_u32 s62, 0\n"                                                             \
  "s_cbranch_scc1 .L" #NAME "_skip\n"                                                       \
  "s_add_u32 s96, s88, s63\n"                                                         \
  "s_addc_u32 s97, s89, 0\n"                                                          \
  PROG                                                                                \
  "v_mov_b32_e32 v41, v30\n"                                                          \
  "v_mov_b32_e32 v42, 0\n"                                                            \
  "v_mov_b32_e32 v40, 0\n"                                                            \
  "s_mov_b32 s64, 0\n"                                                                \
  "s_swappc_b64 s[76:77], s[96:97]\n"                                                 \
  "v_mov_b32_e32 v89, 1\n"                                                            \
  "s_cmp_eq_u32 s69, 0\n"                                                             \
  "s_cbranch_scc1 .L" #NAME "_sum\n"                                                        \
  "v_mov_b32_e32 v40, 0x7fc00000\n"                                                   \
  "s_mov_b64 s[58:59], exec\n"                                                        \
  "s_mov_b64 exec, 1\n"                                                               \
  "s_lshl_b32 s62, s61, 2\n"                                                          \
  "v_mov_b32_e32 v90, s62\n"                                                          \
  "global_store_dword v90, v89, s[54:55] sc1\n"                                       \
  "v_mov_b32_e32 v90, 0\n"                                                            \
  "global_atomic_add v90, v89, s[92:93]\n"                                            \
  "s_mov_b64 exec, s[58:59]\n"                                                        \
  ".L" #NAME "_sum:\n"                                                                      \
  "v_cmp_u_f32_e32 vcc, v40, v40\n"                                                   \
  "s_nop 1\n"                                                                         \
  "v_add_f32_dpp v1, v42, v42 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
  "s_nop 1\n"                                                                         \
  "v_add_f32_dpp v1, v1, v1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
  "s_nop 1\n"                                                                         \
  "v_add_f32_dpp v1, v1, v1 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
  "s_nop 1\n"                                                                         \
  "v_add_f32_dpp v1, v1, v1 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n"     \
  "v_mov_b32_e32 v2, 0\n"                                                             \
  "s_nop 1\n"                                                                         \
  "v_mov_b32_dpp v2, v1 row_bcast:15 row_mask:0xa bank_mask:0xf\n"                    \
  "v_add_f32_e32 v1, v1, v2\n"                                                        \
  "v_mov_b32_e32 v2, 0\n"                                                             \
  "s_nop 1\n"                                                                         \
  "v_mov_b32_dpp v2, v1 row_bcast:31 row_mask:0xc bank_mask:0xf\n"                    \
  "v_add_f32_e32 v1, v1, v2\n"                                                        \
  "s_nop 1\n"                                                                         \
  "v_readlane_b32 s62, v1, 63\n"                                                      \
  "s_cmp_lg_u64 vcc, 0\n"                                                             \
  "s_cselect_b32 s63, 0x7fc00000, 0\n"                                                \
  "s_mov_b64 s[58:59], exec\n"                                                        \
  "s_mov_b64 exec, 1\n"                                                               \
  "v_mov_b32_e32 v0, s62\n"                                                           \
  "s_lshl_b32 s62, s60, 2\n"                                                          \
  "s_cmp_eq_u32 s52, 0\n"                                                             \
  "s_cbranch_scc1 .L" #NAME "_g1\n"                                                         \
  "v_mov_b32_e32 v2, s53\n"                                                           \
  "v_add_u32_e32 v2, s62, v2\n"                                                       \
  "ds_write_b32 v2, v0\n"                                                         \
  "s_branch .L" #NAME "_st1\n"                                                              \
  ".L" #NAME "_g1:\n"                                                                       \
  "v_mov_b32_e32 v2, s62\n"                                                           \
  "global_store_dword v2, v0, s[50:51]\n"                                       \
  ".L" #NAME "_st1:\n"                                                                      \
  "s_cmp_eq_u32 s63, 0\n"                                                             \
  "s_cbranch_scc1 .L" #NAME "_nf\n"                                                         \
  "s_lshl_b32 s62, s61, 2\n"                                                          \
  "v_mov_b32_e32 v2, s62\n"                                                           \
  "global_store_dword v2, v89, s[46:47] sc1\n"                                        \
  ".L" #NAME "_nf:\n"                                                                       \
  "s_mov_b64 exec, s[58:59]\n"                                                        \
  "s_branch .L" #NAME "_next\n"                                                             \
  ".L" #NAME "_skip:\n"                                                                     \
  "s_mov_b64 s[58:59], exec\n"                                                        \
  "s_mov_b64 exec, 1\n"                                                               \
  "v_mov_b32_e32 v0, 0\n"                                                             \
  "s_lshl_b32 s62, s60, 2\n"                                                          \
  "s_cmp_eq_u32 s52, 0\n"                                                             \
  "s_cbranch_scc1 .L" #NAME "_g2\n"                                                         \
  "v_mov_b32_e32 v2, s53\n"                                                           \
  "v_add_u32_e32 v2, s62, v2\n"                                                       \
  "ds_write_b32 v2, v0\n"                                                         \
  "s_branch .L" #NAME "_st2\n"                                                              \
  ".L" #NAME "_g2:\n"                                                                       \
  "v_mov_b32_e32 v2, s62\n"                                                           \
  "global_store_dword v2, v0, s[50:51]\n"                                       \
  ".L" #NAME "_st2:\n"                                                                      \
  "s_mov_b64 exec, s[58:59]\n"                                                        \
  "s_branch .L" #NAME "_next\n"                                                             \
  ".L" #NAME "_done:\n"                                                                     \
  "s_waitcnt vmcnt(0) lgkmcnt(0)\n"                                                   \
  "s_setpc_b64 s[94:95]\n"
// The same loop with the next tree claimed and its failure flag / code offset
// loaded before the current tree runs (their latency under its work):
// next i s58, slot s59, flag v92, code offset s23; exec saved in s[96:97].
#define SR_JIT_LOOP_PF_TEXT(NAME)                                                      \
  ".globl " #NAME "\n.hidden " #NAME "\n.p2align 6\n" #NAME ":\n"               \
  "v_mov_b32_e32 v89, 1\n"                                                       \
  "s_mov_b64 s[96:97], exec\n"                                                   \
  "s_mov_b64 exec, 1\n"                                                          \
  "ds_add_rtn_u32 v90, v31, v89\n"                                               \
  "s_waitcnt lgkmcnt(0)\n"                                                       \
  "s_mov_b64 exec, s[96:97]\n"                                                   \
  "v_readlane_b32 s58, v90, 0\n"                                                 \
  "s_cmp_ge_u32 s58, s40\n"                                                      \
  "s_cbranch_scc1 .L" #NAME "_inv0\n"                                        \
  "s_mul_i32 s59, s58, s41\n"                                                    \
  "s_bitcmp1_b32 s58, 0\n"                                                       \
  "s_cselect_b32 s62, s43, s42\n"                                                \
  "s_add_u32 s59, s59, s62\n"                                                    \
  "s_cmp_ge_u32 s59, s44\n"                                                      \
  "s_cbranch_scc1 .L" #NAME "_inv0\n"                                        \
  "s_lshl_b32 s62, s59, 2\n"                                                     \
  "v_mov_b32_e32 v90, s62\n"                                                     \
  "global_load_dword v92, v90, s[46:47] sc1\n"                                   \
  "s_load_dword s23, s[48:49], s62\n"                                            \
  "s_branch .L" #NAME "_ok0\n"                                        \
  ".L" #NAME "_inv0:\n"                                        \
  "s_mov_b32 s58, -1\n"                                                          \
  ".L" #NAME "_ok0:\n"                                        \
  ".L" #NAME "_next:\n"                                        \
  "s_cmp_ge_u32 s58, s40\n"                                                      \
  "s_cbranch_scc1 .L" #NAME "_done\n"                                        \
  "s_waitcnt vmcnt(0) lgkmcnt(0)\n"                                              \
  "v_readfirstlane_b32 s62, v92\n"                                               \
  "s_mov_b32 s60, s58\n"                                                         \
  "s_mov_b32 s61, s59\n"                                                         \
  "s_mov_b32 s63, s23\n"                                                         \
  "s_mov_b32 s91, s62\n"                                                         \
  "s_mov_b64 s[96:97], exec\n"                                                   \
  "s_mov_b64 exec, 1\n"                                                          \
  "ds_add_rtn_u32 v90, v31, v89\n"                                               \
  "s_waitcnt lgkmcnt(0)\n"                                                       \
  "s_mov_b64 exec, s[96:97]\n"                                                   \
  "v_readlane_b32 s58, v90, 0\n"                                                 \
  "s_cmp_ge_u32 s58, s40\n"                                                      \
  "s_cbranch_scc1 .L" #NAME "_inv1\n"                                        \
  "s_mul_i32 s59, s58, s41\n"                                                    \
  "s_bitcmp1_b32 s58, 0\n"                                                       \
  "s_cselect_b32 s62, s43, s42\n"                                                \
  "s_add_u32 s59, s59, s62\n"                                                    \
  "s_cmp_ge_u32 s59, s44\n"                                                      \
  "s_cbranch_scc1 .L" #NAME "_inv1\n"                                        \
  "s_lshl_b32 s62, s59, 2\n"                                                     \
  "v_mov_b32_e32 v90, s62\n"                                                     \
  "global_load_dword v92, v90, s[46:47] sc1\n"                                   \
  "s_load_dword s23, s[48:49], s62\n"                                            \
  "s_branch .L" #NAME "_ok1\n"                                        \
  ".L" #NAME "_inv1:\n"                                        \
  "s_mov_b32 s58, -1\n"                                                          \
  ".L" #NAME "_ok1:\n"                                        \
  "s_bitcmp1_b32 s91, 0\n"                                                       \
  "s_cbranch_scc1 .L" #NAME "_skip\n"                                        \
  "s_and_b32 s79, s45, 1\n"                                                          \
  "s_bitcmp1_b32 s91, 1\n"                                                           \
  "s_cselect_b32 s79, 0, s79\n"                                                      \
  "s_mov_b32 s91, s84\n"                                                             \
  "s_add_u32 s96, s88, s63\n"                                                         \
  "s_addc_u32 s97, s89, 0\n"                                                          \
  "v_mov_b32_e32 v41, v30\n"                                                          \
  "v_mov_b32_e32 v42, 0\n"                                                            \
  "v_mov_b32_e32 v40, 0\n"                                                            \
  "s_mov_b32 s64, 0\n"                                                                \
  "s_swappc_b64 s[76:77], s[96:97]\n"                                                 \
  "v_mov_b32_e32 v89, 1\n"                                                            \
  "s_cmp_eq_u32 s84, s91\n"                                                          \
  "s_cbranch_scc1 .L" #NAME "_nore\n"                                       \
  "s_bitcmp1_b32 s45, 1\n"                                                           \
  "s_cbranch_scc0 .L" #NAME "_nore\n"                                       \
  "s_mov_b64 s[96:97], exec\n"                                                       \
  "s_mov_b64 exec, 1\n"                                                              \
  "s_lshl_b32 s62, s61, 2\n"                                                         \
  "v_mov_b32_e32 v90, s62\n"                                                         \
  "v_mov_b32_e32 v91, 2\n"                                                           \
  "global_atomic_or v90, v91, s[46:47]\n"                                           \
  "s_mov_b64 exec, s[96:97]\n"                                                       \
  ".L" #NAME "_nore:\n"                                                   \
  "s_cmp_eq_u32 s69, 0\n"                                                             \
  "s_cbranch_scc1 .L" #NAME "_sum\n"                                                        \
  "v_mov_b32_e32 v40, 0x7fc00000\n"                                                   \
  "s_mov_b64 s[96:97], exec\n"                                                        \
  "s_mov_b64 exec, 1\n"                                                               \
  "s_lshl_b32 s62, s61, 2\n"                                                          \
  "v_mov_b32_e32 v90, s62\n"                                                          \
  "global_store_dword v90, v89, s[54:55] sc1\n"                                       \
  "v_mov_b32_e32 v90, 0\n"                                                            \
  "global_atomic_add v90, v89, s[92:93]\n"                                            \
  "s_mov_b64 exec, s[96:97]\n"                                                        \
  ".L" #NAME "_sum:\n"                                                                      \
  "v_cmp_u_f32_e32 vcc, v40, v40\n"                                                   \
  "s_nop 1\n"                                                                         \
  "v_add_f32_dpp v1, v42, v42 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
  "s_nop 1\n"                                                                         \
  "v_add_f32_dpp v1, v1, v1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
  "s_nop 1\n"                                                                         \
  "v_add_f32_dpp v1, v1, v1 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
  "s_nop 1\n"                                                                         \
  "v_add_f32_dpp v1, v1, v1 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n"     \
  "v_mov_b32_e32 v2, 0\n"                                                             \
  "s_nop 1\n"                                                                         \
  "v_mov_b32_dpp v2, v1 row_bcast:15 row_mask:0xa bank_mask:0xf\n"                    \
  "v_add_f32_e32 v1, v1, v2\n"                                                        \
  "v_mov_b32_e32 v2, 0\n"                                                             \
  "s_nop 1\n"                                                                         \
  "v_mov_b32_dpp v2, v1 row_bcast:31 row_mask:0xc bank_mask:0xf\n"                    \
  "v_add_f32_e32 v1, v1, v2\n"                                                        \
  "s_nop 1\n"                                                                         \
  "v_readlane_b32 s62, v1, 63\n"                                                      \
  "s_cmp_lg_u64 vcc, 0\n"                                                             \
  "s_cselect_b32 s63, 0x7fc00000, 0\n"                                                \
  "s_mov_b64 s[96:97], exec\n"                                                        \
  "s_mov_b64 exec, 1\n"                                                               \
  "v_mov_b32_e32 v0, s62\n"                                                           \
  "s_lshl_b32 s62, s60, 2\n"                                                          \
  "s_cmp_eq_u32 s52, 0\n"                                                             \
  "s_cbranch_scc1 .L" #NAME "_g1\n"                                                         \
  "v_mov_b32_e32 v2, s53\n"                                                           \
  "v_add_u32_e32 v2, s62, v2\n"                                                       \
  "ds_write_b32 v2, v0\n"                                                         \
  "s_branch .L" #NAME "_st1\n"                                                              \
  ".L" #NAME "_g1:\n"                                                                       \
  "v_mov_b32_e32 v2, s62\n"                                                           \
  "global_store_dword v2, v0, s[50:51]\n"                                       \
  ".L" #NAME "_st1:\n"                                                                      \
  "s_cmp_eq_u32 s63, 0\n"                                                             \
  "s_cbranch_scc1 .L" #NAME "_nf\n"                                                         \
  "s_lshl_b32 s62, s61, 2\n"                                                          \
  "v_mov_b32_e32 v2, s62\n"                                                           \
  "global_store_dword v2, v89, s[46:47] sc1\n"                                        \
  ".L" #NAME "_nf:\n"                                                                       \
  "s_mov_b64 exec, s[96:97]\n"                                                        \
  "s_branch .L" #NAME "_next\n"                                                             \
  ".L" #NAME "_skip:\n"                                                                     \
  "s_mov_b64 s[96:97], exec\n"                                                        \
  "s_mov_b64 exec, 1\n"                                                               \
  "v_mov_b32_e32 v0, 0\n"                                                             \
  "s_lshl_b32 s62, s60, 2\n"                                                          \
  "s_cmp_eq_u32 s52, 0\n"                                                             \
  "s_cbranch_scc1 .L" #NAME "_g2\n"                                                         \
  "v_mov_b32_e32 v2, s53\n"                                                           \
  "v_add_u32_e32 v2, s62, v2\n"                                                       \
  "ds_write_b32 v2, v0\n"                                                         \
  "s_branch .L" #NAME "_st2\n"                                                              \
  ".L" #NAME "_g2:\n"                                                                       \
  "v_mov_b32_e32 v2, s62\n"                                                           \
  "global_store_dword v2, v0, s[50:51]\n"                                       \
  ".L" #NAME "_st2:\n"                                                                      \
  "s_mov_b64 exec, s[96:97]\n"                                                        \
  "s_branch .L" #NAME "_next\n"                                                             \
  ".L" #NAME "_done:\n"                                                                     \
  "s_waitcnt vmcnt(0) lgkmcnt(0)\n"                                                   \
  "s_setpc_b64 s[94:95]\n"


// the slot's program (memory-constant tree code loads its constants from it):
// s[56:57] = program base s[98:99] + 8 * list_off[slot] (list_off at s[100:101])
#define SR_JIT_LOOP_PROG                                                              \
  "s_lshl_b32 s62, s61, 2\n"                                                          \
  "s_load_dword s91, s[100:101], s62\n"                                               \
  "s_waitcnt lgkmcnt(0)\n"                                                            \
  "s_lshl_b32 s91, s91, 3\n"                                                          \
  "s_add_u32 s56, s98, s91\n"                                                         \
  "s_addc_u32 s57, s99, 0\n"
extern "C" __global__ void __launch_bounds__(64) sr_jit_loop_holder() {
  asm volatile("s_endpgm\n" SR_JIT_LOOP_TEXT(sr_jit_loop, "") SR_JIT_LOOP_TEXT(sr_jit_loop_m, SR_JIT_LOOP_PROG)
                   SR_JIT_LOOP_PF_TEXT(sr_jit_loop_p));
}

template <bool W, bool MEMC, bool PF = false>
__device__ __forceinline__ void jit_eval_dl_body(const JitArgs& ja) {
  const EvalArgs<float>& a = ja.e;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* sX = reinterpret_cast<float*>(smem);
  const int ncol = ja.nraw + ja.nder;
  const int narr = 1 + ncol + (W ? 1 : 0);
  const int rows = a.ntiles * TILE;
  int rg, g;
  if (!block_of(a, rg, g)) return;
  const bool tail = rg >= ja.nbig;
  const int ntl = tail ? ja.ts : a.ntiles;
  const int64_t row0 = tail ? (int64_t)ja.nbig * rows + (int64_t)(rg - ja.nbig) * ja.ts * TILE : (int64_t)rg * rows;
  const int nthreads = __builtin_amdgcn_readfirstlane((int)blockDim.x);
  // 4-byte partials (Σ only): a failed tree is known from its slot's failure
  // flag, which every loop sets when a row fails (finalize_kernel part4)
  float* gdst = reinterpret_cast<float*>(a.partial) + (size_t)rg * ((size_t)a.ntg * a.tpb) + (size_t)g * a.tpb;
  Part<float>* sPart = reinterpret_cast<Part<float>*>(sX + (size_t)narr * rows);
  // the tree counter after the tiles (and the partials): launch() adds 16 bytes
  uint32_t* cnt = reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned char*>(sPart) +
                                              (ja.part_lds ? (size_t)a.tpb * sizeof(Part<float>) : 0));
  {
    constexpr int V = TILE / 4;
    const int total = ntl * narr * V;
    for (int idx = threadIdx.x; idx < total; idx += nthreads) {
      const int v = idx % V;
      const int tk = idx / V;
      const int k = tk % narr;
      const int t = tk / narr;
      if (k > ja.nraw && k <= ncol && ja.dcols) {
        const float* src = ja.dcols + (size_t)(k - 1 - ja.nraw) * a.n_pad;
        reinterpret_cast<float4*>(sX + (size_t)tk * TILE)[v] =
            reinterpret_cast<const float4*>(src + row0 + (int64_t)t * TILE)[v];
        continue;
      }
      if (k > ja.nraw && k <= ncol) {
        const uint32_t d = ja.der[k - 1 - ja.nraw];
        const int op = __builtin_amdgcn_readfirstlane((int)(d >> 16));
        const float4 x = reinterpret_cast<const float4*>(a.X + (size_t)(d & 0xffffu) * a.n_pad + row0 +
                                                         (int64_t)t * TILE)[v];
        reinterpret_cast<float4*>(sX + (size_t)tk * TILE)[v] =
            make_float4(derive_uop(op, x.x), derive_uop(op, x.y), derive_uop(op, x.z), derive_uop(op, x.w));
        continue;
      }
      const float* src = k == 0 ? a.y : (k <= ja.nraw ? a.X + (size_t)(k - 1) * a.n_pad : a.w);
      reinterpret_cast<float4*>(sX + (size_t)tk * TILE)[v] =
          reinterpret_cast<const float4*>(src + row0 + (int64_t)t * TILE)[v];
    }
    if (threadIdx.x == 0) *cnt = 0u;
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int64_t rem = a.n - row0;
  const int nt_valid = (int)min((int64_t)ntl, (rem + TILE - 1) / TILE);
  const int last_valid = (int)(rem - (int64_t)(nt_valid - 1) * TILE);
  uint64_t area;
  asm volatile(
      "s_getpc_b64 s[88:89]\n"
      "s_add_u32 s88, s88, sr_jit_code@rel32@lo+4\n"
      "s_addc_u32 s89, s89, sr_jit_code@rel32@hi+12"
      : "={s[88:89]}"(area)
      :
      : "scc");  // s_add / s_addc: a carry chain of the compiler must not span this
  const uint32_t lds_lane = (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) float*)sX) +
                            (uint32_t)lane * 16u;
  const uint32_t cnt_addr = (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) uint32_t*)cnt);
  const uint32_t spart = (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) Part<float>*)sPart);
  const uint32_t tilebytes = (uint32_t)(narr * TILE * 4);
  const uint32_t woff = W ? (uint32_t)((1 + ncol) * TILE * 4) : 0u;
  const uint32_t lane4 = (uint32_t)lane * R;
  const uint32_t partial = (uint32_t)last_valid;
  const uint32_t nt_u = (uint32_t)nt_valid;
  const uint32_t fastok = (uint32_t)ja.fast;
  const uint32_t tpb = (uint32_t)a.tpb, ntg = (uint32_t)a.ntg, gg = (uint32_t)g, g1 = (uint32_t)(a.ntg - 1 - g);
  const uint32_t nlist = (uint32_t)a.nlist, plds = (uint32_t)ja.part_lds;
  const uint64_t failp = reinterpret_cast<uint64_t>(a.fail), codep = reinterpret_cast<uint64_t>(ja.code_off);
  const uint64_t dstp = reinterpret_cast<uint64_t>(gdst), bailp = reinterpret_cast<uint64_t>(ja.bail);
  const uint64_t cntp = reinterpret_cast<uint64_t>(ja.counters);
  const uint64_t gcb = sgpr64(ja.gcols ? reinterpret_cast<uint64_t>(ja.gcols + row0) : 0ull);
  const uint32_t gstride = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a.n_pad * 4));
  uint32_t redos = 0;
  if constexpr (MEMC) {
    const uint64_t progp = reinterpret_cast<uint64_t>(a.prog), lop = reinterpret_cast<uint64_t>(a.list_off);
    asm volatile(
        "s_getpc_b64 s[96:97]\n"
        "s_add_u32 s96, s96, sr_jit_loop_m@rel32@lo+4\n"
        "s_addc_u32 s97, s97, sr_jit_loop_m@rel32@hi+12\n"
        "s_swappc_b64 s[94:95], s[96:97]"
        : "+{s84}"(redos)
        : "{v30}"(lds_lane), "{v31}"(cnt_addr), "{v43}"(lane4), "{s65}"(nt_u), "{s66}"(partial), "{s67}"(tilebytes),
          "{s68}"(woff), "{s79}"(fastok), "{s40}"(tpb), "{s41}"(ntg), "{s42}"(gg), "{s43}"(g1), "{s44}"(nlist),
          "{s[46:47]}"(failp), "{s[48:49]}"(codep), "{s[50:51]}"(dstp), "{s52}"(plds), "{s53}"(spart),
          "{s[54:55]}"(bailp), "{s[92:93]}"(cntp), "{s[88:89]}"(area), "{s[98:99]}"(progp), "{s[100:101]}"(lop)
        : SR_JIT_CLOBBERS_MEMC, "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s69", "s91", "s94",
          "s95", "s96", "s97", "v40", "v41", "v42", "v89", "v90", "v91", "memory");
  } else if constexpr (PF) {
    const uint32_t fastflags = fastok | (ja.dyn ? 2u : 0u);  // JitArgs::dyn: sticky PRECISE per tree
    asm volatile(
        "s_getpc_b64 s[96:97]\n"
        "s_add_u32 s96, s96, sr_jit_loop_p@rel32@lo+4\n"
        "s_addc_u32 s97, s97, sr_jit_loop_p@rel32@hi+12\n"
        "s_swappc_b64 s[94:95], s[96:97]"
        : "+{s84}"(redos)
        : "{v30}"(lds_lane), "{v31}"(cnt_addr), "{v43}"(lane4), "{s65}"(nt_u), "{s66}"(partial), "{s67}"(tilebytes),
          "{s68}"(woff), "{s45}"(fastflags), "{s40}"(tpb), "{s41}"(ntg), "{s42}"(gg), "{s43}"(g1), "{s44}"(nlist),
          "{s[46:47]}"(failp), "{s[48:49]}"(codep), "{s[50:51]}"(dstp), "{s52}"(plds), "{s53}"(spart),
          "{s[54:55]}"(bailp), "{s[92:93]}"(cntp), "{s[88:89]}"(area), "{s[36:37]}"(gcb), "{s38}"(gstride)
        : SR_JIT_CLOBBERS, "s23", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s69", "s79", "s91", "s94", "s95",
          "s96", "s97", "v40", "v41", "v42", "v89", "v90", "v91", "v92", "memory");
  } else {
    asm volatile(
        "s_getpc_b64 s[96:97]\n"
        "s_add_u32 s96, s96, sr_jit_loop@rel32@lo+4\n"
        "s_addc_u32 s97, s97, sr_jit_loop@rel32@hi+12\n"
        "s_swappc_b64 s[94:95], s[96:97]"
        : "+{s84}"(redos)
        : "{v30}"(lds_lane), "{v31}"(cnt_addr), "{v43}"(lane4), "{s65}"(nt_u), "{s66}"(partial), "{s67}"(tilebytes),
          "{s68}"(woff), "{s79}"(fastok), "{s40}"(tpb), "{s41}"(ntg), "{s42}"(gg), "{s43}"(g1), "{s44}"(nlist),
          "{s[46:47]}"(failp), "{s[48:49]}"(codep), "{s[50:51]}"(dstp), "{s52}"(plds), "{s53}"(spart),
          "{s[54:55]}"(bailp), "{s[92:93]}"(cntp), "{s[88:89]}"(area), "{s[36:37]}"(gcb), "{s38}"(gstride)
        : SR_JIT_CLOBBERS, "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s69", "s91", "s94", "s95", "s96", "s97",
          "v40", "v41", "v42", "v89", "v90", "v91", "memory");
  }
  if (lane == 0 && __builtin_amdgcn_readfirstlane((int)redos) != 0)
    __hip_atomic_fetch_add(ja.counters + 1, (uint32_t)__builtin_amdgcn_readfirstlane((int)redos),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (ja.part_lds) {  // slots no wave ran keep whatever: finalize ignores them
    __syncthreads();
    const float* sPart4 = reinterpret_cast<const float*>(sPart);
    for (int i = threadIdx.x; i < a.tpb; i += nthreads) gdst[i] = sPart4[i];
  }
}
extern "C" __global__ void __launch_bounds__(1024) sr_jit_eval_dl(JitArgs ja) { jit_eval_dl_body<false, false>(ja); }
extern "C" __global__ void __launch_bounds__(1024) sr_jit_eval_dlw(JitArgs ja) { jit_eval_dl_body<true, false>(ja); }
extern "C" __global__ void __launch_bounds__(1024) sr_jit_eval_dlp(JitArgs ja) { jit_eval_dl_body<false, false, true>(ja); }
extern "C" __global__ void __launch_bounds__(1024) sr_jit_eval_dlpw(JitArgs ja) { jit_eval_dl_body<true, false, true>(ja); }
extern "C" __global__ void __launch_bounds__(1024) sr_jit_eval_dlm(JitArgs ja) { jit_eval_dl_body<false, true>(ja); }
extern "C" __global__ void __launch_bounds__(1024) sr_jit_eval_dlmw(JitArgs ja) { jit_eval_dl_body<true, true>(ja); }

// ---- gradient tree code (jit_grad.cpp) ---------------------------------------------
// One workgroup = (row group, tree group) as above; each tree's code runs the
// forward pass and the reverse (adjoint) pass of every tile, leaves Σ w·ℓ in
// LSUM and the marker in CHK, and itself stores Σ w·ℓ'·∂ŷ/∂c_j of each of its
// constants (summed over the wave) to this row group's partials. LDS holds
// the row tiles only, so two or more tiles of a wide dataset fit.
struct JitGradArgs {
  EvalArgs<float> e;        // rows, tiles, list / fail / partial as for sr_jit_eval
  const int32_t* code_off;  // [nlist] byte offset of each slot's gradient code
  const float* consts;      // [total constants + 16] the program's constants
  const int32_t* cbase;     // [nlist] first constant of the slot's tree
  const int32_t* ncon;      // [nlist] its constant count (<= SR_JIT_G_NGACC)
  float* gpart;             // [nrg][nconst] per-row-group Σ w·ℓ'·∂ŷ/∂c
  int nconst;
  int dyn;                  // (reserved, as JitArgs::dyn)
  const float* gcols;       // [ngcol][n_pad] shared-subtree columns (jit_grad.cpp GradGen::S_GCOL), or null
};

template <bool W>
__device__ __forceinline__ void jit_grad_body(const JitGradArgs& ja) {
  const EvalArgs<float>& a = ja.e;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* sX = reinterpret_cast<float*>(smem);
  const int narr = 1 + a.nfeat + (W ? 1 : 0);
  int rg, g;
  if (!block_of(a, rg, g)) return;
  const int rows = a.ntiles * TILE;
  const int64_t row0 = (int64_t)rg * rows;
  {
    constexpr int V = TILE / 4;
    const int total = a.ntiles * narr * V;
    for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
      const int v = idx % V;
      const int tk = idx / V;
      const int k = tk % narr;
      const int t = tk / narr;
      const float* src = k == 0 ? a.y : (k <= a.nfeat ? a.X + (size_t)(k - 1) * a.n_pad : a.w);
      reinterpret_cast<float4*>(sX + (size_t)tk * TILE)[v] =
          reinterpret_cast<const float4*>(src + row0 + (int64_t)t * TILE)[v];
    }
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int64_t rem = a.n - row0;
  const int nt_valid = (int)min((int64_t)a.ntiles, (rem + TILE - 1) / TILE);
  const int last_valid = (int)(rem - (int64_t)(nt_valid - 1) * TILE);
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int nwaves = (int)(blockDim.x >> 6);
  auto slot_of = [&](int i) { return a.contig ? g * a.tpb + i : i * a.ntg + ((i & 1) ? (a.ntg - 1 - g) : g); };
  auto sld = [&](const int32_t* p, int s) {
    return __builtin_amdgcn_readfirstlane(((const __attribute__((address_space(4))) int32_t*)(p))[s]);
  };
  auto ld_flag = [&](int slot) { return __hip_atomic_load(a.fail + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  uint64_t area;
  asm volatile(
      "s_getpc_b64 s[88:89]\n"
      "s_add_u32 s88, s88, sr_jit_code@rel32@lo+4\n"
      "s_addc_u32 s89, s89, sr_jit_code@rel32@hi+12"
      : "={s[88:89]}"(area)
      :
      : "scc");  // s_add / s_addc: a carry chain of the compiler must not span this
  const uint32_t lds_lane = (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) float*)sX) +
                            (uint32_t)lane * 16u;
  const uint32_t tilebytes = (uint32_t)(narr * TILE * 4);
  const uint32_t woff = W ? (uint32_t)((1 + a.nfeat) * TILE * 4) : 0u;
  const uint32_t lane4 = (uint32_t)lane * R;
  const uint32_t partial = (uint32_t)last_valid;
  const uint32_t nt_u = (uint32_t)nt_valid;

  int m = wave < a.tpb ? (a.tpb - wave + nwaves - 1) / nwaves : 0;
  while (m > 0 && slot_of(wave + (m - 1) * nwaves) >= a.nlist) --m;
  m = __builtin_amdgcn_readfirstlane(m);
  uint32_t fnext = m > 0 ? ld_flag(slot_of(wave)) : 0u;
  float* gdst = ja.gpart + (size_t)rg * (size_t)ja.nconst;
  Part<float>* dst = a.partial + (size_t)rg * ((size_t)a.ntg * a.tpb) + (size_t)g * a.tpb;
  const uint64_t gcb = sgpr64(ja.gcols ? reinterpret_cast<uint64_t>(ja.gcols + row0) : 0ull);
  const uint32_t gstride = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a.n_pad * 4));
  for (int k = 0; k < m; ++k) {
    const int i = __builtin_amdgcn_readfirstlane(wave + k * nwaves);
    const int s = __builtin_amdgcn_readfirstlane(slot_of(i));
    const bool more = k + 1 < m;
    const bool skip = __builtin_amdgcn_readfirstlane((int)fnext) != 0;
    if (more) fnext = ld_flag(slot_of(wave + (k + 1) * nwaves));
    float lsum = 0.0f, chk = skip ? __builtin_nanf("") : 0.0f;
    if (!skip) {
      const int cb = sld(ja.cbase, s);
      const uint64_t target = area + (uint32_t)sld(ja.code_off, s);
      const uint64_t cptr = reinterpret_cast<uint64_t>(ja.consts + cb);
      const uint64_t gptr = reinterpret_cast<uint64_t>(gdst + cb);
      uint32_t la = lds_lane;
      uint32_t tile = 0, status;
      asm volatile("s_swappc_b64 s[76:77], %[tgt]"
                   : "+{v42}"(lsum), "+{v40}"(chk), "+{v41}"(la), "+{s64}"(tile), "={s69}"(status)
                   : [tgt] "s"(target), "{v43}"(lane4), "{s65}"(nt_u), "{s66}"(partial), "{s67}"(tilebytes),
                     "{s68}"(woff), "{s[78:79]}"(cptr), "{s[84:85]}"(gptr), "{s[98:99]}"(gcb), "{s100}"(gstride)
                   : SR_JIT_GRAD_CLOBBERS, "memory");
      (void)status;
    }
    // a skipped tree writes no ∂L/∂c partials: finalize marks it failed
    lsum = wave_sum(lsum);
    chk = __builtin_amdgcn_ballot_w64(chk != chk) != 0 ? __builtin_nanf("") : 0.0f;
    if (lane == 0) dst[i] = Part<float>{lsum, chk};
    if (!skip && chk != chk && lane == 0)
      __hip_atomic_store(a.fail + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

extern "C" __global__ void __launch_bounds__(256) sr_jit_grad(JitGradArgs ja) { jit_grad_body<false>(ja); }
extern "C" __global__ void __launch_bounds__(256) sr_jit_grad_w(JitGradArgs ja) { jit_grad_body<true>(ja); }

// The gradient tree code's loop, hand-written as SR_JIT_LOOP_TEXT (the waves
// of a workgroup take their trees from an LDS counter). Registers as there,
// except: s[50:51] the group's partials (global), s[52:53] the slots' first
// constants (cbase), s[54:55] the constants, s[56:57] this row group's ∂L/∂c
// partials; per tree s[78:79] = constants + cbase, s[84:85] = partials +
// cbase (the gradient code's inputs); temps s58-s63, s91, s96-s97, v0-v2,
// v153-v155 (above the gradient code's registers, gen_jit.py
// SR_JIT_GRAD_CLOBBERS). No bails and no redo count in gradient code.
#define SR_JIT_GLOOP_TEXT                                                             \
  ".globl sr_jit_gloop\n.hidden sr_jit_gloop\n.p2align 6\nsr_jit_gloop:\n"            \
  "v_mov_b32_e32 v153, 1\n"                                                           \
  ".Lsrg_next:\n"                                                                     \
  "s_mov_b64 s[58:59], exec\n"                                                        \
  "s_mov_b64 exec, 1\n"                                                               \
  "ds_add_rtn_u32 v154, v31, v153\n"                                                  \
  "s_waitcnt lgkmcnt(0)\n"                                                            \
  "s_mov_b64 exec, s[58:59]\n"                                                        \
  "v_readlane_b32 s60, v154, 0\n"                                                     \
  "s_cmp_ge_u32 s60, s40\n"                                                           \
  "s_cbranch_scc1 .Lsrg_done\n"                                                       \
  "s_mul_i32 s61, s60, s41\n"                                                         \
  "s_bitcmp1_b32 s60, 0\n"                                                            \
  "s_cselect_b32 s62, s43, s42\n"                                                     \
  "s_add_u32 s61, s61, s62\n"                                                         \
  "s_cmp_ge_u32 s61, s44\n"                                                           \
  "s_cbranch_scc1 .Lsrg_done\n"                                                       \
  "s_lshl_b32 s62, s61, 2\n"                                                          \
  "v_mov_b32_e32 v154, s62\n"                                                         \
  "global_load_dword v155, v154, s[46:47] sc1\n"                                      \
  "s_load_dword s63, s[48:49], s62\n"                                                 \
  "s_load_dword s91, s[52:53], s62\n"                                                 \
  "s_waitcnt vmcnt(0) lgkmcnt(0)\n"                                                   \
  "v_readfirstlane_b32 s62, v155\n"                                                   \
  "s_cmp_lg_u32 s62, 0\n"                                                             \
  "s_cbranch_scc1 .Lsrg_skip\n"                                                       \
  "s_add_u32 s96, s88, s63\n"                                                         \
  "s_addc_u32 s97, s89, 0\n"                                                          \
  "s_lshl_b32 s62, s91, 2\n"                                                          \
  "s_add_u32 s78, s54, s62\n"                                                         \
  "s_addc_u32 s79, s55, 0\n"                                                          \
  "s_add_u32 s84, s56, s62\n"                                                         \
  "s_addc_u32 s85, s57, 0\n"                                                          \
  "v_mov_b32_e32 v41, v30\n"                                                          \
  "v_mov_b32_e32 v42, 0\n"                                                            \
  "v_mov_b32_e32 v40, 0\n"                                                            \
  "s_mov_b32 s64, 0\n"                                                                \
  "s_swappc_b64 s[76:77], s[96:97]\n"                                                 \
  "v_mov_b32_e32 v153, 1\n"                                                           \
  "v_cmp_u_f32_e32 vcc, v40, v40\n"                                                   \
  "s_nop 1\n"                                                                         \
  "v_add_f32_dpp v1, v42, v42 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
  "s_nop 1\n"                                                                         \
  "v_add_f32_dpp v1, v1, v1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
  "s_nop 1\n"                                                                         \
  "v_add_f32_dpp v1, v1, v1 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
  "s_nop 1\n"                                                                         \
  "v_add_f32_dpp v1, v1, v1 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n"     \
  "v_mov_b32_e32 v2, 0\n"                                                             \
  "s_nop 1\n"                                                                         \
  "v_mov_b32_dpp v2, v1 row_bcast:15 row_mask:0xa bank_mask:0xf\n"                    \
  "v_add_f32_e32 v1, v1, v2\n"                                                        \
  "v_mov_b32_e32 v2, 0\n"                                                             \
  "s_nop 1\n"                                                                         \
  "v_mov_b32_dpp v2, v1 row_bcast:31 row_mask:0xc bank_mask:0xf\n"                    \
  "v_add_f32_e32 v1, v1, v2\n"                                                        \
  "s_nop 1\n"                                                                         \
  "v_readlane_b32 s62, v1, 63\n"                                                      \
  "s_cmp_lg_u64 vcc, 0\n"                                                             \
  "s_cselect_b32 s63, 0x7fc00000, 0\n"                                                \
  "s_mov_b64 s[58:59], exec\n"                                                        \
  "s_mov_b64 exec, 1\n"                                                               \
  "v_mov_b32_e32 v0, s62\n"                                                           \
  "v_mov_b32_e32 v1, s63\n"                                                           \
  "s_lshl_b32 s62, s60, 3\n"                                                          \
  "v_mov_b32_e32 v2, s62\n"                                                           \
  "global_store_dwordx2 v2, v[0:1], s[50:51]\n"                                       \
  "s_cmp_eq_u32 s63, 0\n"                                                             \
  "s_cbranch_scc1 .Lsrg_nf\n"                                                         \
  "s_lshl_b32 s62, s61, 2\n"                                                          \
  "v_mov_b32_e32 v2, s62\n"                                                           \
  "global_store_dword v2, v153, s[46:47] sc1\n"                                       \
  ".Lsrg_nf:\n"                                                                       \
  "s_mov_b64 exec, s[58:59]\n"                                                        \
  "s_branch .Lsrg_next\n"                                                             \
  ".Lsrg_skip:\n"                                                                     \
  "s_mov_b64 s[58:59], exec\n"                                                        \
  "s_mov_b64 exec, 1\n"                                                               \
  "v_mov_b32_e32 v0, 0\n"                                                             \
  "v_mov_b32_e32 v1, 0x7fc00000\n"                                                    \
  "s_lshl_b32 s62, s60, 3\n"                                                          \
  "v_mov_b32_e32 v2, s62\n"                                                           \
  "global_store_dwordx2 v2, v[0:1], s[50:51]\n"                                       \
  "s_mov_b64 exec, s[58:59]\n"                                                        \
  "s_branch .Lsrg_next\n"                                                             \
  ".Lsrg_done:\n"                                                                     \
  "s_waitcnt vmcnt(0) lgkmcnt(0)\n"                                                   \
  "s_setpc_b64 s[94:95]\n"

extern "C" __global__ void __launch_bounds__(64) sr_jit_gloop_holder() { asm volatile("s_endpgm\n" SR_JIT_GLOOP_TEXT); }

template <bool W>
__device__ __forceinline__ void jit_grad_dl_body(const JitGradArgs& ja) {
  const EvalArgs<float>& a = ja.e;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* sX = reinterpret_cast<float*>(smem);
  const int narr = 1 + a.nfeat + (W ? 1 : 0);
  int rg, g;
  if (!block_of(a, rg, g)) return;
  const int rows = a.ntiles * TILE;
  const int64_t row0 = (int64_t)rg * rows;
  uint32_t* cnt = reinterpret_cast<uint32_t*>(sX + (size_t)narr * rows);  // launch_grad adds 16 bytes
  {
    constexpr int V = TILE / 4;
    const int total = a.ntiles * narr * V;
    for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
      const int v = idx % V;
      const int tk = idx / V;
      const int k = tk % narr;
      const int t = tk / narr;
      const float* src = k == 0 ? a.y : (k <= a.nfeat ? a.X + (size_t)(k - 1) * a.n_pad : a.w);
      reinterpret_cast<float4*>(sX + (size_t)tk * TILE)[v] =
          reinterpret_cast<const float4*>(src + row0 + (int64_t)t * TILE)[v];
    }
    if (threadIdx.x == 0) *cnt = 0u;
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int64_t rem = a.n - row0;
  const int nt_valid = (int)min((int64_t)a.ntiles, (rem + TILE - 1) / TILE);
  const int last_valid = (int)(rem - (int64_t)(nt_valid - 1) * TILE);
  uint64_t area;
  asm volatile(
      "s_getpc_b64 s[88:89]\n"
      "s_add_u32 s88, s88, sr_jit_code@rel32@lo+4\n"
      "s_addc_u32 s89, s89, sr_jit_code@rel32@hi+12"
      : "={s[88:89]}"(area)
      :
      : "scc");  // s_add / s_addc: a carry chain of the compiler must not span this
  const uint32_t lds_lane = (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) float*)sX) +
                            (uint32_t)lane * 16u;
  const uint32_t cnt_addr = (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) uint32_t*)cnt);
  const uint32_t tilebytes = (uint32_t)(narr * TILE * 4);
  const uint32_t woff = W ? (uint32_t)((1 + a.nfeat) * TILE * 4) : 0u;
  const uint32_t lane4 = (uint32_t)lane * R;
  const uint32_t partial = (uint32_t)last_valid;
  const uint32_t nt_u = (uint32_t)nt_valid;
  const uint32_t tpb = (uint32_t)a.tpb, ntg = (uint32_t)a.ntg, gg = (uint32_t)g, g1 = (uint32_t)(a.ntg - 1 - g);
  const uint32_t nlist = (uint32_t)a.nlist;
  const uint64_t failp = reinterpret_cast<uint64_t>(a.fail), codep = reinterpret_cast<uint64_t>(ja.code_off);
  const uint64_t dstp = reinterpret_cast<uint64_t>(a.partial + (size_t)rg * ((size_t)a.ntg * a.tpb) + (size_t)g * a.tpb);
  const uint64_t cbp = reinterpret_cast<uint64_t>(ja.cbase), constp = reinterpret_cast<uint64_t>(ja.consts);
  const uint64_t gdstp = reinterpret_cast<uint64_t>(ja.gpart + (size_t)rg * (size_t)ja.nconst);
  const uint64_t gcb = sgpr64(ja.gcols ? reinterpret_cast<uint64_t>(ja.gcols + row0) : 0ull);
  const uint32_t gstride = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a.n_pad * 4));
  asm volatile(
      "s_getpc_b64 s[96:97]\n"
      "s_add_u32 s96, s96, sr_jit_gloop@rel32@lo+4\n"
      "s_addc_u32 s97, s97, sr_jit_gloop@rel32@hi+12\n"
      "s_swappc_b64 s[94:95], s[96:97]"
      :
      : "{v30}"(lds_lane), "{v31}"(cnt_addr), "{v43}"(lane4), "{s65}"(nt_u), "{s66}"(partial), "{s67}"(tilebytes),
        "{s68}"(woff), "{s40}"(tpb), "{s41}"(ntg), "{s42}"(gg), "{s43}"(g1), "{s44}"(nlist), "{s[46:47]}"(failp),
        "{s[48:49]}"(codep), "{s[50:51]}"(dstp), "{s[52:53]}"(cbp), "{s[54:55]}"(constp), "{s[56:57]}"(gdstp),
        "{s[88:89]}"(area), "{s[98:99]}"(gcb), "{s100}"(gstride)
      : SR_JIT_GRAD_CLOBBERS, "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s69", "s78", "s79", "s84", "s85",
        "s91", "s94", "s95", "s96", "s97", "v40", "v41", "v42", "v153", "v154", "v155", "memory");
}
extern "C" __global__ void __launch_bounds__(256) sr_jit_grad_dl(JitGradArgs ja) { jit_grad_dl_body<false>(ja); }
extern "C" __global__ void __launch_bounds__(256) sr_jit_grad_dlw(JitGradArgs ja) { jit_grad_dl_body<true>(ja); }
