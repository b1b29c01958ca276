// grad_kernels.hip — constant-gradient kernels (forward mode, fused with the
// loss): the batched replacement for ConstantOptimization.jl's gradients
// (src/ConstantOptimization.jl:12-65 evaluates the loss by finite
// differences; eval_grad_tree_array(...; variable=false),
// src/InterfaceDynamicExpressions.jl:105-107, gives ∂ŷ/∂c per row).
//
// Same workgroup structure as eval_kernel (row group staged in LDS, waves take
// work items round-robin); a work item is (tree, tangent group of kGradG
// constants). GRAD_LOSS returns Σ w·ℓ and Σ w·ℓ'(r)·∂ŷ/∂c_k per constant;
// GRAD_OUT writes ŷ and ∂ŷ/∂c_k per row.
#include <hip/hip_runtime.h>

#include "grad_interp.h"
#include "kernels.h"

namespace srhip {
namespace {

using namespace interp;

template <typename T, int R, int D, int MODE, bool W, int G, int SET>
__global__ void __launch_bounds__(256) grad_kernel(GradArgs<T> a) {
  constexpr int S = 2 + G;
  constexpr int TILE = 64 * R;
  using V = typename V16<T>::type;
  constexpr int N = V16<T>::N;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int rows = a.ntiles * TILE;
  const int narr = a.nfeat + (MODE == GRAD_LOSS ? (W ? 2 : 1) : 0);
  T* sX = reinterpret_cast<T*>(smem);
  T* sY = sX + (size_t)a.nfeat * rows;
  T* sW = sY + rows;
  T* sPart = sX + (size_t)narr * rows;

  const int rg = blockIdx.x / a.ntg;
  const int g = blockIdx.x - rg * a.ntg;
  const int64_t row0 = (int64_t)rg * rows;
  {
    const int vper = rows / N;
    const int total = narr * vper;
    for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
      const int arr = idx / vper;
      const int v = idx - arr * vper;
      const T* src = arr < a.nfeat ? a.X + (size_t)arr * a.n_pad : (arr == a.nfeat ? a.y : a.w);
      reinterpret_cast<V*>(sX + (size_t)arr * rows)[v] = reinterpret_cast<const V*>(src + row0)[v];
    }
    for (int i = threadIdx.x; i < a.tpb * S; i += blockDim.x) sPart[i] = T(0);
    if (threadIdx.x == 0) *reinterpret_cast<uint32_t*>(sPart + a.tpb * S) = 0u;  // item counter (a.dyn)
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int64_t rem = a.n - row0;
  const int nt_valid = (int)min((int64_t)a.ntiles, (rem + TILE - 1) / TILE);
  const int last_valid = (int)(rem - (int64_t)(nt_valid - 1) * TILE);
  const double lp = a.lparam;

  // Waves take the group's (cost-sorted) items round-robin, or (a.dyn, the
  // default) from an LDS counter, so a wave that drew cheap items takes more.
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int nwaves = (int)(blockDim.x >> 6);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(sPart + a.tpb * S);
  auto claim = [&]() {
    uint32_t v = 0;
    if (lane == 0) v = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return __builtin_amdgcn_readfirstlane((int)v);
  };
  for (int i = a.dyn ? claim() : wave; i < a.tpb; i = a.dyn ? claim() : i + nwaves) {
    const int s = i * a.ntg + ((i & 1) ? (a.ntg - 1 - g) : g);
    if (s >= a.nitems) continue;
    const int item = __builtin_amdgcn_readfirstlane(a.items[s]);
    const int t = item & 0xffffff;
    const int g0 = (item >> 24) * kGradG;  // groups are kGradG constants; G of them carried
    CIns<T>* p = const_prog(a.prog + __builtin_amdgcn_readfirstlane(a.tree_off[t]));
    const int cbase = __builtin_amdgcn_readfirstlane(a.const_off[t]);
    const int nc = __builtin_amdgcn_readfirstlane(a.const_off[t + 1]) - cbase;
    T acc[S];
#pragma unroll
    for (int k = 0; k < S; ++k) acc[k] = T(0);  // [0] Σ w·ℓ, [1] marker, [2+j] Σ w·ℓ'·∂ŷ/∂c
    for (int tl = 0; tl < nt_valid; ++tl) {
      const T* sXt = sX + tl * TILE;
      Dual<T, R, G> d;
      run_program_grad<T, R, D, G, SET>(p, sXt, rows, lane, g0, d, acc[1]);
#pragma unroll
      for (int r = 0; r < R; ++r) acc[1] = mark(d.v[r], acc[1]);
      if constexpr (MODE == GRAD_OUT) {
        const int64_t off = row0 + tl * TILE;
        if (g0 == 0) store_rows<T, R>(a.out_value + (size_t)t * a.out_stride + off, lane, d.v);
#pragma unroll
        for (int j = 0; j < G; ++j)
          if (g0 + j < nc)
            store_rows<T, R>(a.out_grad + (size_t)(cbase + g0 + j) * a.out_stride + off, lane, d.d[j]);
      } else {
        T yv[R], wv[R];
        lds_rows<T, R>(sY + tl * TILE, lane, yv);
        if constexpr (W) lds_rows<T, R>(sW + tl * TILE, lane, wv);
        const int valid = (tl < nt_valid - 1) ? TILE : last_valid;
#pragma unroll
        for (int e = 0; e < R; ++e) {
          T l = dev::elem_loss<T>(a.loss, lp, d.v[e], yv[e]);
          T dl = dev::elem_dloss<T>(a.loss, lp, d.v[e], yv[e]);
          if constexpr (W) { l = wv[e] * l; dl = wv[e] * dl; }
          const bool in = row_of<T, R>(e, lane) < valid;
          acc[0] += in ? l : T(0);
#pragma unroll
          for (int j = 0; j < G; ++j) acc[2 + j] += in ? dl * d.d[j][e] : T(0);
        }
      }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
      for (int k = 0; k < S; ++k) acc[k] += __shfl_xor(acc[k], off);
    if (lane == 0)
#pragma unroll
      for (int k = 0; k < S; ++k) sPart[i * S + k] = acc[k];
  }
  __syncthreads();
  T* dst = a.partial + ((size_t)rg * ((size_t)a.ntg * a.tpb) + (size_t)g * a.tpb) * S;
  for (int i = threadIdx.x; i < a.tpb * S; i += blockDim.x) dst[i] = sPart[i];
}

template <typename T, int G>
__global__ void __launch_bounds__(256) grad_finalize_kernel(GradArgs<T> a, double* __restrict__ out_sum,
                                                            uint8_t* __restrict__ out_ok,
                                                            double* __restrict__ out_dloss) {
  constexpr int S = 2 + G;
  __shared__ double sh[4][S][64];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int npos = a.ntg * a.tpb;
  const int pos = blockIdx.x * 64 + lane;
  double acc[S];
  for (int k = 0; k < S; ++k) acc[k] = 0.0;
  if (pos < npos) {
    for (int rg = w; rg < a.nrg; rg += 4) {
      const T* q = a.partial + ((size_t)rg * npos + pos) * S;
      for (int k = 0; k < S; ++k) acc[k] += (double)q[k];
    }
  }
  for (int k = 0; k < S; ++k) sh[w][k][lane] = acc[k];
  __syncthreads();
  if (w == 0 && pos < npos) {
    for (int k = 0; k < S; ++k) acc[k] = (sh[0][k][lane] + sh[1][k][lane]) + (sh[2][k][lane] + sh[3][k][lane]);
    const int g = pos / a.tpb;
    const int i = pos - g * a.tpb;
    const int sidx = i * a.ntg + ((i & 1) ? (a.ntg - 1 - g) : g);
    if (sidx < a.nitems) {
      const int item = a.items[sidx];
      const int t = item & 0xffffff;
      const int g0 = (item >> 24) * kGradG;
      const bool ok = !__builtin_isnan(acc[1]);
      if (g0 == 0) {
        out_sum[t] = ok ? acc[0] : __builtin_nan("");
        out_ok[t] = ok ? 1 : 0;
      }
      const int cb = a.const_off[t];
      const int nc = a.const_off[t + 1] - cb;
      for (int j = 0; j < G; ++j)
        if (g0 + j < nc) out_dloss[cb + g0 + j] = ok ? acc[2 + j] : __builtin_nan("");
    }
  }
}

template <typename T, int R, int D, int MODE, bool W, int G, int SET>
hipError_t launch_grad_one(const EvalPlan& plan, const GradArgs<T>& a, hipStream_t stream) {
  // raise the dynamic-LDS ceiling once per kernel instantiation: a function-
  // local static is initialised exactly once even with concurrent callers
  static const hipError_t attr_err = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&grad_kernel<T, R, D, MODE, W, G, SET>), hipFuncAttributeMaxDynamicSharedMemorySize,
      160 * 1024);
  if (attr_err != hipSuccess) return attr_err;
  const unsigned grid = (unsigned)a.nrg * (unsigned)a.ntg;
  hipLaunchKernelGGL((grad_kernel<T, R, D, MODE, W, G, SET>), dim3(grid), dim3(plan.threads), plan.lds_bytes,
                     stream, a);
  return hipGetLastError();
}

template <typename T, int R, int D, int G, int SET>
hipError_t launch_grad_rd(const EvalPlan& plan, const GradArgs<T>& a, int mode, hipStream_t stream) {
  if (mode == GRAD_OUT) return launch_grad_one<T, R, D, GRAD_OUT, false, G, SET>(plan, a, stream);
  if (a.w) return launch_grad_one<T, R, D, GRAD_LOSS, true, G, SET>(plan, a, stream);
  return launch_grad_one<T, R, D, GRAD_LOSS, false, G, SET>(plan, a, stream);
}

// gradient variants: rows per lane R (fewer tangents leave room for more
// rows) and stack slots D
inline int grad_R(int dtype, bool deep, int G) {
  if (dtype != SRHIP_F32 || deep) return 1;
  return G <= 2 ? 4 : 2;
}

template <typename T, int G>
hipError_t launch_grad_g(const EvalPlan& plan, const GradArgs<T>& a, int mode, hipStream_t stream) {
  constexpr int RS = sizeof(T) == 4 ? (G <= 2 ? 4 : 2) : 1;  // grad_R, shallow
  if (plan.D == 4) {
    if (a.opset == OPSET_BASIC) return launch_grad_rd<T, RS, 4, G, OPSET_BASIC>(plan, a, mode, stream);
    return launch_grad_rd<T, RS, 4, G, OPSET_FULL>(plan, a, mode, stream);
  }
  return launch_grad_rd<T, 1, kMaxSlots, G, OPSET_FULL>(plan, a, mode, stream);
}

}  // namespace

bool plan_grad(int dtype, bool deep, int G, int mode, bool weighted, int nfeat, int64_t n, int nitems,
               EvalPlan* p) {
  const size_t esz = dtype == SRHIP_F32 ? 4 : 8;
  const int narr = nfeat + (mode == GRAD_LOSS ? (weighted ? 2 : 1) : 0);
  return plan_geometry(esz, grad_R(dtype, deep, G), deep ? kMaxSlots : 4, narr, (2 + G) * esz, n, nitems, p);
}

template <typename T>
hipError_t launch_grad(const EvalPlan& plan, const GradArgs<T>& a, int mode, hipStream_t stream) {
  if (plan.D != 4) return launch_grad_g<T, kGradG>(plan, a, mode, stream);  // deep programs: one variant
  if (a.G == 1) return launch_grad_g<T, 1>(plan, a, mode, stream);
  if (a.G == 2) return launch_grad_g<T, 2>(plan, a, mode, stream);
  return launch_grad_g<T, kGradG>(plan, a, mode, stream);
}

template <typename T>
hipError_t launch_grad_finalize(const GradArgs<T>& a, double* out_sum, uint8_t* out_ok, double* out_dloss,
                                hipStream_t stream) {
  const int npos = a.ntg * a.tpb;
  const unsigned grid = (unsigned)((npos + 63) / 64);
  if (a.G == 1)
    hipLaunchKernelGGL((grad_finalize_kernel<T, 1>), dim3(grid), dim3(256), 0, stream, a, out_sum, out_ok, out_dloss);
  else if (a.G == 2)
    hipLaunchKernelGGL((grad_finalize_kernel<T, 2>), dim3(grid), dim3(256), 0, stream, a, out_sum, out_ok, out_dloss);
  else
    hipLaunchKernelGGL((grad_finalize_kernel<T, kGradG>), dim3(grid), dim3(256), 0, stream, a, out_sum, out_ok,
                       out_dloss);
  return hipGetLastError();
}

template hipError_t launch_grad<float>(const EvalPlan&, const GradArgs<float>&, int, hipStream_t);
template hipError_t launch_grad<double>(const EvalPlan&, const GradArgs<double>&, int, hipStream_t);
template hipError_t launch_grad_finalize<float>(const GradArgs<float>&, double*, uint8_t*, double*, hipStream_t);
template hipError_t launch_grad_finalize<double>(const GradArgs<double>&, double*, uint8_t*, double*,
                                                 hipStream_t);

}  // namespace srhip
