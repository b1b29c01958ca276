// kernels.hip — CDNA4 (gfx950) kernels of the batched tree evaluator.
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
#include <hip/hip_runtime.h>

#include "interp.h"
#include "kernels.h"

namespace srhip {
namespace {

using namespace interp;

// Σ over this lane's rows of the tile of w·ℓ(ŷ, y); masked rows (past n) add 0.
template <int LK, bool W, bool MASK, typename T, int R>
__device__ __forceinline__ T tile_loss(const T (&acc)[R], const T (&yv)[R], const T (&wv)[R],
                                       T lp, int lane, int valid) {
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

template <bool W, bool MASK, typename T, int R>
__device__ __forceinline__ T tile_loss_any(int lk, const T (&acc)[R], const T (&yv)[R],
                                           const T (&wv)[R], T lp, int lane, int valid) {
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
    default: return tile_loss<SRHIP_LOSS_LOGITDIST, W, MASK>(acc, yv, wv, lp, lane, valid);
  }
}

template <typename T, int R, int D, int MODE, bool W>
__global__ void __launch_bounds__(256) eval_kernel(EvalArgs<T> a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int TILE = 64 * R;
  using V = typename V16<T>::type;
  constexpr int N = V16<T>::N;
  const int rows = a.ntiles * TILE;
  const int narr = a.nfeat + (MODE == MODE_LOSS ? (W ? 2 : 1) : 0);
  T* sX = reinterpret_cast<T*>(smem);
  T* sY = sX + (size_t)a.nfeat * rows;
  T* sW = sY + rows;
  Part<T>* sPart = reinterpret_cast<Part<T>*>(sX + (size_t)narr * rows);

  const int rg = blockIdx.x / a.ntg;
  const int g = blockIdx.x - rg * a.ntg;
  const int64_t row0 = (int64_t)rg * rows;

  // 1. stage the row group in LDS
  {
    const int vper = rows / N;
    const int total = narr * vper;
    for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
      const int arr = idx / vper;
      const int v = idx - arr * vper;
      const T* src = arr < a.nfeat ? a.X + (size_t)arr * a.n_pad : (arr == a.nfeat ? a.y : a.w);
      reinterpret_cast<V*>(sX + (size_t)arr * rows)[v] = reinterpret_cast<const V*>(src + row0)[v];
    }
    for (int i = threadIdx.x; i < a.tpb; i += blockDim.x) sPart[i] = Part<T>{T(0), T(0)};
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int64_t rem = a.n - row0;
  const int nt_valid = (int)min((int64_t)a.ntiles, (rem + TILE - 1) / TILE);
  const int last_valid = (int)(rem - (int64_t)(nt_valid - 1) * TILE);
  const T lp = a.lparam;

  // 2. trees of this group, taken dynamically by the waves
  // Waves take the group's (cost-sorted) trees round-robin: a static,
  // wave-uniform schedule (no atomics, no divergent loop exit).
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int nwaves = (int)(blockDim.x >> 6);
  for (int i = wave; i < a.tpb; i += nwaves) {
    const int s = i * a.ntg + ((i & 1) ? (a.ntg - 1 - g) : g);
    if (s >= a.nlist) continue;
    const int t = __builtin_amdgcn_readfirstlane(a.list[s]);
    const Ins<T>* p = a.prog + __builtin_amdgcn_readfirstlane(a.tree_off[t]);
    T lsum = T(0), chk = T(0);
    for (int tl = 0; tl < nt_valid; ++tl) {
      const T* sXt = sX + tl * TILE;
      T acc[R];
      run_program<T, R, D>(p, sXt, rows, lane, acc, chk);
#pragma unroll
      for (int r = 0; r < R; ++r) chk = mark(acc[r], chk);  // root value
      if constexpr (MODE == MODE_OUT) {
        store_rows<T, R>(a.out + (size_t)t * a.out_stride + row0 + tl * TILE, lane, acc);
      } else {
        T yv[R], wv[R];
        lds_rows<T, R>(sY + tl * TILE, lane, yv);
        if constexpr (W) lds_rows<T, R>(sW + tl * TILE, lane, wv);
        if (tl < nt_valid - 1 || last_valid == TILE)
          lsum += tile_loss_any<W, false, T, R>(a.loss, acc, yv, wv, lp, lane, TILE);
        else
          lsum += tile_loss_any<W, true, T, R>(a.loss, acc, yv, wv, lp, lane, last_valid);
      }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      lsum += __shfl_xor(lsum, off);
      chk += __shfl_xor(chk, off);
    }
    if (lane == 0) sPart[i] = Part<T>{lsum, chk};
  }
  __syncthreads();
  // 3. one coalesced store of the group's partials
  Part<T>* dst = a.partial + (size_t)rg * ((size_t)a.ntg * a.tpb) + (size_t)g * a.tpb;
  for (int i = threadIdx.x; i < a.tpb; i += blockDim.x) dst[i] = sPart[i];
}

template <typename T>
__global__ void __launch_bounds__(256) finalize_kernel(EvalArgs<T> a, double* __restrict__ out_sum,
                                                       uint8_t* __restrict__ out_ok) {
  __shared__ double ss[4][64];
  __shared__ double sc[4][64];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int npos = a.ntg * a.tpb;
  const int pos = blockIdx.x * 64 + lane;
  double s = 0.0, c = 0.0;
  if (pos < npos) {
    for (int rg = w; rg < a.nrg; rg += 4) {
      const Part<T> q = a.partial[(size_t)rg * npos + pos];
      s += (double)q.sum;
      c += (double)q.chk;
    }
  }
  ss[w][lane] = s;
  sc[w][lane] = c;
  __syncthreads();
  if (w == 0 && pos < npos) {
    s = (ss[0][lane] + ss[1][lane]) + (ss[2][lane] + ss[3][lane]);
    c = (sc[0][lane] + sc[1][lane]) + (sc[2][lane] + sc[3][lane]);
    const int g = pos / a.tpb;
    const int i = pos - g * a.tpb;
    const int sidx = i * a.ntg + ((i & 1) ? (a.ntg - 1 - g) : g);
    if (sidx < a.nlist) {
      const int t = a.list[sidx];
      const bool ok = !__builtin_isnan(c);
      out_sum[t] = ok ? s : __builtin_nan("");
      out_ok[t] = ok ? 1 : 0;
    }
  }
}

template <typename T>
__global__ void pack_x_kernel(const T* __restrict__ src, int layout, int64_t src_stride,
                              int64_t rows, int nfeat, int64_t n_pad, T* __restrict__ dst,
                              int* __restrict__ bad) {
  const int64_t total = n_pad * nfeat;
  int found = 0;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t f = idx / n_pad;
    const int64_t i = idx - f * n_pad;
    const int64_t si = i < rows ? i : rows - 1;
    const T v = layout == SRHIP_X_JULIA ? src[si * nfeat + f] : src[f * src_stride + si];
    dst[idx] = v;
    if (i < rows && !__builtin_isfinite(v)) found = 1;
  }
  if (found) atomicOr(bad, 1);
}

template <typename T>
__global__ void pack_vec_kernel(const T* __restrict__ src, int64_t rows, int64_t n_pad,
                                T* __restrict__ dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_pad;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i < rows ? i : rows - 1];
}

template <typename T>
__global__ void gather_rows_kernel(const T* __restrict__ X, const T* __restrict__ y,
                                   const T* __restrict__ w, int nfeat, int64_t src_pad,
                                   const int64_t* __restrict__ idx, int64_t nidx,
                                   int64_t dst_pad, T* __restrict__ Xd, T* __restrict__ yd,
                                   T* __restrict__ wd) {
  const int64_t total = dst_pad * (nfeat + 2);
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < total;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t f = k / dst_pad;
    const int64_t j = k - f * dst_pad;
    const int64_t r = idx[j < nidx ? j : nidx - 1];
    if (f < nfeat) Xd[f * dst_pad + j] = X[f * src_pad + r];
    else if (f == nfeat) yd[j] = y[r];
    else if (w) wd[j] = w[r];
  }
}

template <typename T, int R, int D, int MODE, bool W>
hipError_t launch_one(const EvalPlan& plan, const EvalArgs<T>& a, hipStream_t stream) {
  static bool attr_set = false;  // raise the dynamic-LDS ceiling once per kernel
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&eval_kernel<T, R, D, MODE, W>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const unsigned grid = (unsigned)a.nrg * (unsigned)a.ntg;
  hipLaunchKernelGGL((eval_kernel<T, R, D, MODE, W>), dim3(grid), dim3(plan.threads),
                     plan.lds_bytes, stream, a);
  return hipGetLastError();
}

template <typename T, int R, int D>
hipError_t launch_rd(const EvalPlan& plan, const EvalArgs<T>& a, int mode, hipStream_t stream) {
  if (mode == MODE_OUT) return launch_one<T, R, D, MODE_OUT, false>(plan, a, stream);
  if (a.w) return launch_one<T, R, D, MODE_LOSS, true>(plan, a, stream);
  return launch_one<T, R, D, MODE_LOSS, false>(plan, a, stream);
}

}  // namespace

// Kernel variants: (rows per lane R, stack slots D).
//   f32: (8, 4) for ordinary trees, (4, 16) for deep ones
//   f64: (4, 4) and (2, 16)
static inline int variant_R(int dtype, bool deep) {
  return dtype == SRHIP_F32 ? (deep ? 4 : 8) : (deep ? 2 : 4);
}

bool plan_geometry(size_t esz, int R, int D, int narr, size_t part_bytes, int64_t n, int nlist,
                   EvalPlan* p) {
  p->R = R;
  p->D = D;
  p->tile = 64 * R;
  p->threads = 256;
  const size_t per_tile = (size_t)narr * p->tile * esz;
  const size_t budget = 40 * 1024;
  int nt = 1;
  while ((int64_t)nt * 2 * p->tile <= 8192 && per_tile * nt * 2 <= budget &&
         (int64_t)nt * p->tile < n)
    nt *= 2;
  p->ntiles = nt;
  p->rows_wg = nt * p->tile;
  p->nrg = (int)((n + p->rows_wg - 1) / p->rows_wg);
  if (p->nrg < 1) p->nrg = 1;
  const int target_wg = 8192;
  int ntg = (target_wg + p->nrg - 1) / p->nrg;
  const int max_groups = (nlist + 3) / 4;  // at least ~4 trees (one per wave) per group
  if (ntg > max_groups) ntg = max_groups;
  if (ntg < 1) ntg = 1;
  p->tpb = (nlist + ntg - 1) / ntg;
  p->ntg = (nlist + p->tpb - 1) / p->tpb;
  p->lds_bytes = per_tile * nt + (size_t)p->tpb * part_bytes + 16;
  return p->lds_bytes <= 160 * 1024;
}

bool plan_eval(int dtype, bool deep, int mode, bool weighted, int nfeat, int64_t n,
               int nlist, EvalPlan* p) {
  const size_t esz = dtype == SRHIP_F32 ? 4 : 8;
  const int narr = nfeat + (mode == MODE_LOSS ? (weighted ? 2 : 1) : 0);
  return plan_geometry(esz, variant_R(dtype, deep), deep ? kMaxSlots : 4, narr, 2 * esz, n, nlist, p);
}

template <typename T>
hipError_t launch_eval(const EvalPlan& plan, const EvalArgs<T>& a, int mode, hipStream_t stream) {
  if constexpr (sizeof(T) == 4) {
    if (plan.D == 4) return launch_rd<T, 8, 4>(plan, a, mode, stream);
    return launch_rd<T, 4, kMaxSlots>(plan, a, mode, stream);
  } else {
    if (plan.D == 4) return launch_rd<T, 4, 4>(plan, a, mode, stream);
    return launch_rd<T, 2, kMaxSlots>(plan, a, mode, stream);
  }
}

template <typename T>
hipError_t launch_finalize(const EvalArgs<T>& a, double* out_sum, uint8_t* out_ok,
                           hipStream_t stream) {
  const int npos = a.ntg * a.tpb;
  const unsigned grid = (unsigned)((npos + 63) / 64);
  hipLaunchKernelGGL((finalize_kernel<T>), dim3(grid), dim3(256), 0, stream, a, out_sum, out_ok);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_pack_x(const T* src, int layout, int64_t src_stride, int64_t rows, int nfeat,
                         int64_t n_pad, T* dst, int* bad, hipStream_t stream) {
  const int64_t total = n_pad * nfeat;
  unsigned grid = (unsigned)std::min<int64_t>((total + 255) / 256, 4096);
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL((pack_x_kernel<T>), dim3(grid), dim3(256), 0, stream, src, layout,
                     src_stride, rows, nfeat, n_pad, dst, bad);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_pack_vec(const T* src, int64_t rows, int64_t n_pad, T* dst, hipStream_t stream) {
  unsigned grid = (unsigned)std::min<int64_t>((n_pad + 255) / 256, 4096);
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL((pack_vec_kernel<T>), dim3(grid), dim3(256), 0, stream, src, rows, n_pad, dst);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_gather_rows(const T* X, const T* y, const T* w, int nfeat, int64_t src_pad,
                              const int64_t* idx, int64_t nidx, int64_t dst_pad, T* Xd, T* yd,
                              T* wd, hipStream_t stream) {
  const int64_t total = dst_pad * (nfeat + 2);
  unsigned grid = (unsigned)std::min<int64_t>((total + 255) / 256, 4096);
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL((gather_rows_kernel<T>), dim3(grid), dim3(256), 0, stream, X, y, w, nfeat,
                     src_pad, idx, nidx, dst_pad, Xd, yd, wd);
  return hipGetLastError();
}

#define SR_INST(T)                                                                             \
  template hipError_t launch_eval<T>(const EvalPlan&, const EvalArgs<T>&, int, hipStream_t);  \
  template hipError_t launch_finalize<T>(const EvalArgs<T>&, double*, uint8_t*, hipStream_t); \
  template hipError_t launch_pack_x<T>(const T*, int, int64_t, int64_t, int, int64_t, T*,     \
                                       int*, hipStream_t);                                    \
  template hipError_t launch_pack_vec<T>(const T*, int64_t, int64_t, T*, hipStream_t);         \
  template hipError_t launch_gather_rows<T>(const T*, const T*, const T*, int, int64_t,        \
                                            const int64_t*, int64_t, int64_t, T*, T*, T*,      \
                                            hipStream_t);
SR_INST(float)
SR_INST(double)

}  // namespace srhip
