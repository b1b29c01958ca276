// eval_kernel.h — CDNA4 (gfx950) kernels of the batched tree evaluator.
//
// eval_kernel: one workgroup = (row group, tree group).
//   1. The workgroup stages its row group (ntiles × 64·R rows) of every
//      feature, y and w into LDS once (16-byte vector loads, coalesced).
//   2. The waves take the group's trees round-robin (trees are sorted by
//      cost, longest first) and run each program over every tile: the program is wave-uniform (scalar
//      loads, uniform branches), each instruction processes R rows per lane
//      held in VGPRs; leaf features come straight from LDS with ds_read_b128.
//   3. Per tree the wave reduces Σ w·ℓ and the non-finite marker over its
//      lanes into an LDS slot; the workgroup writes all its slots with one
//      coalesced store. finalize_kernel sums the row groups in fp64.
// There is no MFMA: this is a VALU-bound interpreter, not a contraction.
//
// This header holds the kernel templates; eval_f32.hip / eval_f64.hip
// instantiate the variants of one element type each (parallel compiles).
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "interp.h"
#include "kernels.h"

// Experimental switches (make EXTRA=-D...): SR_VP selects the driver of the
// shallow variant (0: scalar-load fetch, 1/2: VGPR-resident program).
#ifndef SR_VP
#define SR_VP 0
#endif
// SR_TI: the threaded interpreter (gen_asm_interp.py) for f32 trees of the
// BASIC operator set in the shallow kernel; 0 keeps the C++ dispatch only.
#ifndef SR_TI
#define SR_TI 1
#endif
#ifndef SR_R32
#define SR_R32 8  // rows per lane of the shallow f32 kernel
#endif
#if SR_TI && defined(__HIP_DEVICE_COMPILE__)
#if SR_R32 == 16
#include "gen/asm_interp_f32_r16.inc"
#else
#include "gen/asm_interp_f32_r8.inc"
#endif
#endif

namespace srhip {
namespace {

using namespace interp;

// Σ over this lane's rows of the tile of w·ℓ(ŷ, y); masked rows (past n) add 0.
template <int LK, bool W, bool MASK, typename T, int R>
__device__ __forceinline__ T tile_loss(const T (&acc)[R], const T (&yv)[R], const T (&wv)[R],
                                       double lp, int lane, int valid) {
  T s0 = T(0), s1 = T(0);
#pragma unroll
  for (int e = 0; e < R; ++e) {
    T l = dev::elem_loss<T>(LK, lp, acc[e], yv[e]);
    if constexpr (W) l = wv[e] * l;
    if constexpr (MASK) {
      const int row = row_of<T, R>(e, lane);
      l = row < valid ? l : T(0);
    }
    if (e & 1) s1 += l; else s0 += l;
  }
  return s0 + s1;
}

// Kernel mode of a MODE_LOSS launch whose loss is L2 (the default loss):
// the tile epilogue is compiled for it instead of switching on a.loss.
constexpr int kModeLossL2 = 2;

template <typename T>
__device__ __forceinline__ T qnan_v() { return __builtin_nan(""); }
template <>
__device__ __forceinline__ float qnan_v<float>() { return __builtin_nanf(""); }

// One tile of one program through the threaded interpreter block
// (gen_asm_interp.py): `recs` = the program's instruction records
// (ti_records_kernel), `lane_addr` = LDS byte address of this lane's rows of
// feature 0 in the tile. Returns false if the block bailed out (an opcode or
// argument it does not handle); acc/chk are then garbage and the caller
// re-runs the tile with the C++ interpreter.
template <int R>
__device__ __forceinline__ bool run_program_ti(const uint4* recs, uint32_t lane_addr, float (&acc)[R],
                                               float& chk) {
#if SR_TI && defined(__HIP_DEVICE_COMPILE__)
  static_assert(R == SR_TI_R, "threaded block generated for another R");
  uint32_t bail;
  const uint64_t rp = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)recs) |
                      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)((uintptr_t)recs >> 32)) << 32);
  const uint32_t lane = lane_addr;
  asm volatile(SR_TI_TEXT : SR_TI_OUTPUTS(acc, chk, bail) : SR_TI_INPUTS(rp, lane) : SR_TI_CLOBBERS);
  return bail == 0;
#else
  (void)recs; (void)lane_addr; (void)acc; (void)chk;
  return false;
#endif
}

template <bool W, bool MASK, typename T, int R>
__device__ __forceinline__ T tile_loss_any(int lk, const T (&acc)[R], const T (&yv)[R],
                                           const T (&wv)[R], double lp, int lane, int valid) {
  switch (lk) {
    case SRHIP_LOSS_L2: return tile_loss<SRHIP_LOSS_L2, W, MASK>(acc, yv, wv, lp, lane, valid);
    case SRHIP_LOSS_L1: return tile_loss<SRHIP_LOSS_L1, W, MASK>(acc, yv, wv, lp, lane, valid);
    case SRHIP_LOSS_LP: return tile_loss<SRHIP_LOSS_LP, W, MASK>(acc, yv, wv, lp, lane, valid);
    case SRHIP_LOSS_HUBER: return tile_loss<SRHIP_LOSS_HUBER, W, MASK>(acc, yv, wv, lp, lane, valid);
    case SRHIP_LOSS_LOGCOSH: return tile_loss<SRHIP_LOSS_LOGCOSH, W, MASK>(acc, yv, wv, lp, lane, valid);
    case SRHIP_LOSS_L1EPSINS: return tile_loss<SRHIP_LOSS_L1EPSINS, W, MASK>(acc, yv, wv, lp, lane, valid);
    case SRHIP_LOSS_L2EPSINS: return tile_loss<SRHIP_LOSS_L2EPSINS, W, MASK>(acc, yv, wv, lp, lane, valid);
    case SRHIP_LOSS_QUANTILE: return tile_loss<SRHIP_LOSS_QUANTILE, W, MASK>(acc, yv, wv, lp, lane, valid);
    case SRHIP_LOSS_PERIODIC: return tile_loss<SRHIP_LOSS_PERIODIC, W, MASK>(acc, yv, wv, lp, lane, valid);
    case SRHIP_LOSS_LPINT: return tile_loss<SRHIP_LOSS_LPINT, W, MASK>(acc, yv, wv, lp, lane, valid);
    default: return tile_loss<SRHIP_LOSS_LOGITDIST, W, MASK>(acc, yv, wv, lp, lane, valid);
  }
}

// Occupancy floor of the shallow f32 variant: 5 waves per SIMD (<= 96 VGPRs;
// the LDS row tile allows 6 workgroups per CU). Without it the compiler
// settles at 97-104 VGPRs and 4 waves.
// (R = 16 pins 130 VGPRs of threaded-interpreter state: 3 waves.)
template <typename T, int R, int D>
constexpr int kWavesPerEU = (sizeof(T) == 4 && D == kShallowSlots) ? (R > 8 ? 3 : 5) : 1;
// One tree of a workgroup's group on its row tiles: the loss (or the per-row
// outputs) of tree slot s into sPart[i], its failure flag set when a row fails
// (the body of the interpreter's tree loop, static or dynamic deal).
template <typename T, int R, int D, int SET, int MODE, bool W, bool VP, bool TI>
__device__ __forceinline__ void eval_tree_in_group(const EvalArgs<T>& a, int i, int s, bool skip, const VProg<T>& vp,
                                                   const Ins<T>* prog, const T* sX, const T* sY, const T* sW,
                                                   Part<T>* sPart, int rows, int lane, int64_t row0, int nt_valid,
                                                   int last_valid, double lp) {
  constexpr int TILE = 64 * R;
  constexpr bool EE = MODE != MODE_OUT;
  CIns<T>* p = const_prog(prog);
  T lsum = T(0), chk = skip ? qnan_v<T>() : T(0);
  for (int tl = 0; tl < (skip ? 0 : nt_valid); ++tl) {
    const T* sXt = sX + tl * TILE;
    T acc[R];
    bool done = false;
    if constexpr (TI) {
      if (a.ti_rec) {
        const T chk0 = chk;
        const uint32_t lds = (uint32_t)reinterpret_cast<uintptr_t>(
            (const __attribute__((address_space(3))) T*)(sXt)) + (uint32_t)lane * 16u;
        done = run_program_ti<R>(a.ti_rec + (size_t)s * 64, lds, acc, chk);
        if (!done) chk = chk0;
      }
    }
    if (done) {
    } else if constexpr (VP && SR_VP == 2) run_program_v2<T, R, D, SET>(vp, sXt, rows, lane, acc, chk);
    else if constexpr (VP) run_program_v<T, R, D, SET>(vp, sXt, rows, lane, acc, chk);
    else run_program<T, R, D, SET>(p, sXt, rows, lane, acc, chk);
#pragma unroll
    for (int r = 0; r < R; ++r) chk = mark(acc[r], chk);  // root value
    if constexpr (MODE == MODE_OUT) {
      const int t = __builtin_amdgcn_readfirstlane(a.list[s]);
      store_rows<T, R>(a.out + (size_t)t * a.out_stride + row0 + tl * TILE, lane, acc);
    } else {
      T yv[R], wv[R];
      lds_rows<T, R>(sY + tl * TILE, lane, yv);
      if constexpr (W) lds_rows<T, R>(sW + tl * TILE, lane, wv);
      if constexpr (MODE == kModeLossL2) {  // L2 known at compile time: no loss switch
        if (tl < nt_valid - 1 || last_valid == TILE)
          lsum += tile_loss<SRHIP_LOSS_L2, W, false>(acc, yv, wv, lp, lane, TILE);
        else
          lsum += tile_loss<SRHIP_LOSS_L2, W, true>(acc, yv, wv, lp, lane, last_valid);
      } else if (tl < nt_valid - 1 || last_valid == TILE) {
        lsum += tile_loss_any<W, false, T, R>(a.loss, acc, yv, wv, lp, lane, TILE);
      } else {
        lsum += tile_loss_any<W, true, T, R>(a.loss, acc, yv, wv, lp, lane, last_valid);
      }
      if (__builtin_amdgcn_ballot_w64(chk != chk) != 0) break;  // failed: the rest is moot
    }
  }
  lsum = wave_sum(lsum);
  chk = wave_sum(chk);
  if (lane == 0) sPart[i] = Part<T>{lsum, chk};
  if constexpr (EE) {
    if (!skip && chk != chk && lane == 0)
      __hip_atomic_store(a.fail + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <typename T, int R, int D, int SET, int MODE, bool W>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kWavesPerEU<T, R, D>)))
eval_kernel(EvalArgs<T> a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int TILE = 64 * R;
  using V = typename V16<T>::type;
  constexpr int N = V16<T>::N;
  const int rows = a.ntiles * TILE;
  const int narr = a.nfeat + (MODE != MODE_OUT ? (W ? 2 : 1) : 0);
  T* sX = reinterpret_cast<T*>(smem);
  T* sY = sX + (size_t)a.nfeat * rows;
  T* sW = sY + rows;
  Part<T>* sPart = reinterpret_cast<Part<T>*>(sX + (size_t)narr * rows);

  const int rg = blockIdx.x / a.ntg;
  const int g = blockIdx.x - rg * a.ntg;
  const int64_t row0 = (int64_t)rg * rows;
  // per-tree row sets: the group's one tree (slot g) reads its own segment
  const int64_t seg0 = a.seg ? a.seg * (int64_t)a.list[g < a.nlist ? g : 0] : 0;

  // 1. stage the row group in LDS
  {
    const int vper = rows / N;
    const int total = narr * vper;
    for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
      const int arr = idx / vper;
      const int v = idx - arr * vper;
      const T* src = arr < a.nfeat ? a.X + (size_t)arr * a.n_pad : (arr == a.nfeat ? a.y : a.w);
      reinterpret_cast<V*>(sX + (size_t)arr * rows)[v] = reinterpret_cast<const V*>(src + seg0 + row0)[v];
    }
    for (int i = threadIdx.x; i < a.tpb; i += blockDim.x) sPart[i] = Part<T>{T(0), T(0)};
    if (threadIdx.x == 0) *reinterpret_cast<uint32_t*>(sPart + a.tpb) = 0u;  // tree counter (a.rotate & 4)
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int64_t rem = a.n - row0;
  const int nt_valid = (int)min((int64_t)a.ntiles, (rem + TILE - 1) / TILE);
  const int last_valid = (int)(rem - (int64_t)(nt_valid - 1) * TILE);
  const double lp = a.lparam;

  // 2. trees of this group, taken dynamically by the waves
  // Waves take the group's (cost-sorted) trees round-robin: a static,
  // wave-uniform schedule (no atomics, no divergent loop exit).
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int nwaves = (int)(blockDim.x >> 6);
  // The shallow variant keeps each tree's program in VGPRs (run_program_v);
  // the next tree's program is loaded while the current one runs.
  constexpr bool VP = SR_VP != 0 && D == kShallowSlots;
  constexpr bool TI = SR_TI != 0 && std::is_same<T, float>::value && R == SR_R32 && D == kShallowSlots;
  auto slot_of = [&](int i) { return i * a.ntg + ((i & 1) ? (a.ntg - 1 - g) : g); };
  // list_off is read through the constant address space: scalar loads (the
  // early-exit flag stores would otherwise make the compiler use vector loads)
  auto prog_of = [&](int s) {
    return a.prog + __builtin_amdgcn_readfirstlane(
                        ((const __attribute__((address_space(4))) int32_t*)(a.list_off))[s]);
  };
  VProg<T> vnext;
  // TI: the program in VGPRs (lane j = instruction j; shallow programs have at
  // most kVProgMax instructions and the code buffer is padded by 64), loaded
  // one tree ahead so its memory latency overlaps the current tree
  // Early exit (MODE_LOSS): DynamicExpressions stops a tree at its first
  // non-finite value. A wave that sees one marks the list slot in a.fail; the
  // row groups that reach the slot later skip it (their partial is the failure
  // marker). Flags are read one tree ahead; a stale 0 only costs the work.
  constexpr bool EE = MODE != MODE_OUT;
  auto ld_flag = [&](int slot) {
    return __hip_atomic_load(a.fail + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  uint32_t fnext = 0;

  // Each wave runs the trees i = wave + k·nwaves, k < m. With a.rotate the
  // sequence starts at k = rot (row group rg at fraction rg/nrg of it): row
  // groups then reach a tree at different times, so a failure found by one
  // row group is skipped by the others that get there later (a tree that
  // overflows on a few rows is otherwise evaluated by every row group at
  // once). Each wave keeps its own set of trees: load balance is unchanged.
  if (a.rotate & 4) {
    // Dynamic dealing (round 4): the waves take the group's trees from an LDS
    // counter, one tree claimed ahead (its flag and program loaded while the
    // current one runs); claim c runs tree (c + rot) mod tpb, rot = the row
    // group's share of tpb (a.rotate & 1), so row groups still reach a tree
    // at different times.
    uint32_t* cnt = reinterpret_cast<uint32_t*>(sPart + a.tpb);
    const int drot = (EE && (a.rotate & 1)) ? __builtin_amdgcn_readfirstlane((int)(((int64_t)rg * a.tpb) / a.nrg)) : 0;
    auto claim = [&]() {
      int c = a.tpb;
      for (;;) {
        uint32_t v = 0;
        if (lane == 0) v = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        c = __builtin_amdgcn_readfirstlane((int)v);
        if (c >= a.tpb) return a.tpb;
        const int i = c + drot < a.tpb ? c + drot : c + drot - a.tpb;
        if (slot_of(i) < a.nlist) return i;
      }
    };
    int inext = claim();
    if (inext < a.tpb) {
      if constexpr (EE) fnext = ld_flag(slot_of(inext));
      if constexpr (VP) vnext.load(prog_of(slot_of(inext)), lane);
    }
    while (inext < a.tpb) {
      const int i = __builtin_amdgcn_readfirstlane(inext);
      const int s = __builtin_amdgcn_readfirstlane(slot_of(i));
      inext = claim();
      const bool more = inext < a.tpb;
      const int s2 = __builtin_amdgcn_readfirstlane(more ? slot_of(inext) : s);
      VProg<T> vp;
      if constexpr (VP) {
        vp = vnext;
        if (more) vnext.load(prog_of(s2), lane);
      }
      const bool skip = EE && __builtin_amdgcn_readfirstlane((int)fnext) != 0;
      if constexpr (EE) {
        if (more) fnext = ld_flag(s2);
      }
      eval_tree_in_group<T, R, D, SET, MODE, W, VP, TI>(a, i, s, skip, vp, prog_of(s), sX, sY, sW, sPart, rows, lane,
                                                        row0, nt_valid, last_valid, lp);
    }
  } else {
  int m = wave < a.tpb ? (a.tpb - wave + nwaves - 1) / nwaves : 0;
  while (m > 0 && slot_of(wave + (m - 1) * nwaves) >= a.nlist) --m;
  m = __builtin_amdgcn_readfirstlane(m);
  const int rot = (EE && a.rotate && m > 1)
                      ? __builtin_amdgcn_readfirstlane((int)(((int64_t)rg * m) / a.nrg))
                      : 0;
  auto idx_of = [&](int k) {
    const int kk = k + rot < m ? k + rot : k + rot - m;
    return wave + kk * nwaves;
  };
  if (m > 0) {
    if constexpr (EE) fnext = ld_flag(slot_of(idx_of(0)));
    if constexpr (VP) vnext.load(prog_of(slot_of(idx_of(0))), lane);
  }
  for (int k = 0; k < m; ++k) {
    // all wave-uniform: keep the schedule in SGPRs
    const int i = __builtin_amdgcn_readfirstlane(idx_of(k));
    const int s = __builtin_amdgcn_readfirstlane(slot_of(i));
    const bool more = k + 1 < m;
    const int s2 = __builtin_amdgcn_readfirstlane(more ? slot_of(idx_of(k + 1)) : s);
    VProg<T> vp;
    if constexpr (VP) {
      vp = vnext;
      if (more) vnext.load(prog_of(s2), lane);
    }
    const bool skip = EE && __builtin_amdgcn_readfirstlane((int)fnext) != 0;
    if constexpr (EE) {
      if (more) fnext = ld_flag(s2);
    }
    eval_tree_in_group<T, R, D, SET, MODE, W, VP, TI>(a, i, s, skip, vp, prog_of(s), sX, sY, sW, sPart, rows, lane,
                                                      row0, nt_valid, last_valid, lp);
  }
  }  // static deal
  __syncthreads();
  // 3. one coalesced store of the group's partials
  Part<T>* dst = a.partial + (size_t)rg * ((size_t)a.ntg * a.tpb) + (size_t)g * a.tpb;
  for (int i = threadIdx.x; i < a.tpb; i += blockDim.x) dst[i] = sPart[i];
}

template <typename T, int R, int D, int SET, int MODE, bool W>
hipError_t launch_one(const EvalPlan& plan, const EvalArgs<T>& a, hipStream_t stream) {
  // raise the dynamic-LDS ceiling once per kernel instantiation: a function-
  // local static is initialised exactly once even with concurrent callers
  static const hipError_t attr_err = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&eval_kernel<T, R, D, SET, MODE, W>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr_err != hipSuccess) return attr_err;
  const unsigned grid = (unsigned)a.nrg * (unsigned)a.ntg;
  hipLaunchKernelGGL((eval_kernel<T, R, D, SET, MODE, W>), dim3(grid), dim3(plan.threads),
                     plan.lds_bytes, stream, a);  // (plan_geometry: + 16 bytes after the partials, the tree counter)
  return hipGetLastError();
}

template <typename T, int R, int D, int SET>
hipError_t launch_rd(const EvalPlan& plan, const EvalArgs<T>& a, int mode, hipStream_t stream) {
  if (mode == MODE_OUT) return launch_one<T, R, D, SET, MODE_OUT, false>(plan, a, stream);
  if (a.loss == SRHIP_LOSS_L2) {
    if (a.w) return launch_one<T, R, D, SET, kModeLossL2, true>(plan, a, stream);
    return launch_one<T, R, D, SET, kModeLossL2, false>(plan, a, stream);
  }
  if (a.w) return launch_one<T, R, D, SET, MODE_LOSS, true>(plan, a, stream);
  return launch_one<T, R, D, SET, MODE_LOSS, false>(plan, a, stream);
}

}  // namespace
}  // namespace srhip
