// kernels.hip — host-side planning and the small support kernels of the
// batched tree evaluator: fp64 finalize of the per-row-group partials,
// dataset packing and row gathers. The evaluation kernel itself is in
// eval_kernel.h (instantiated by eval_f32.hip / eval_f64.hip).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "kernels.h"

#include <algorithm>

namespace srhip {
namespace {

// One workgroup per 16 slots; lane l of wave w sums slot l % 16 over the row
// groups rg ≡ 4w + l / 16 (mod 64) — a fixed order: the sums do not depend
// on timing — and the workgroup adds the 64 parts of each slot in a fixed tree.
// (16 slots per workgroup spread a batch's sums over 4x the CUs of one slot
// per lane: the loop per lane is a quarter as long.) It also leaves the
// launch's flags clean for the next call (no clearing launch per call): each
// slot's failure flag, and (cnt != nullptr) the tree code's counters, copied
// to cnt_host first.
constexpr int kFinWaves = 16;
constexpr int kFinPos = 16;                      // slots per workgroup
constexpr int kFinSub = 64 / kFinPos;            // row-group lanes per slot and wave
constexpr int kFinStride = kFinWaves * kFinSub;  // row groups per round of the workgroup
template <typename T>
__global__ void __launch_bounds__(64 * kFinWaves) finalize_kernel(EvalArgs<T> a, double* __restrict__ out_sum,
                                                                  uint8_t* __restrict__ out_ok,
                                                                  uint32_t* __restrict__ cnt,
                                                                  uint32_t* __restrict__ cnt_host) {
  if (cnt && blockIdx.x == 0 && threadIdx.x == 0) {
    cnt_host[0] = cnt[0];
    cnt_host[1] = cnt[1];
    cnt[0] = 0u;
    cnt[1] = 0u;
  }
  __shared__ double ss[kFinWaves * kFinSub][kFinPos];
  __shared__ double sc[kFinWaves * kFinSub][kFinPos];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int p = lane % kFinPos, r = lane / kFinPos;
  const int npos = a.ntg * a.tpb;
  const int pos = blockIdx.x * kFinPos + p;
  double s = 0.0, c = 0.0;
  if (pos < npos) {
    if (a.part4) {  // Σ only (float: the Float32 tree code's loops)
      const float* p4 = reinterpret_cast<const float*>(a.partial);
#pragma unroll 4
      for (int rg = w * kFinSub + r; rg < a.nrg; rg += kFinStride) s += (double)p4[(size_t)rg * npos + pos];
    } else {
#pragma unroll 4
      for (int rg = w * kFinSub + r; rg < a.nrg; rg += kFinStride) {
        const Part<T> q = a.partial[(size_t)rg * npos + pos];
        s += (double)q.sum;
        c += (double)q.chk;
      }
    }
  }
  const int row = w * kFinSub + r;  // = threadIdx.x / kFinPos
  ss[row][p] = s;
  sc[row][p] = c;
  __syncthreads();
  for (int k = kFinWaves * kFinSub / 2; k >= 1; k /= 2) {  // a fixed tree over the 64 parts
    if (row < k) {
      ss[row][p] += ss[row + k][p];
      sc[row][p] += sc[row + k][p];
    }
    __syncthreads();
  }
  if (row == 0 && pos < npos) {
    s = ss[0][p];
    c = sc[0][p];
    const int g = pos / a.tpb;
    const int i = pos - g * a.tpb;
    const int sidx = a.contig ? g * a.tpb + i : i * a.ntg + ((i & 1) ? (a.ntg - 1 - g) : g);
    if (sidx < a.nlist) {
      const int t = a.list[sidx];
      // part4: failed = bit 0 of the flag word (bit 1 marks a tree sticky PRECISE, JitArgs::dyn)
      const bool ok = a.part4 ? (a.fail[sidx] & 1u) == 0u : !__builtin_isnan(c);
      out_sum[t] = ok ? s : __builtin_nan("");
      out_ok[t] = ok ? 1 : 0;
      if (a.fail) a.fail[sidx] = 0u;
    }
  }
}

// zero two word ranges in one launch (the per-slot failure flags and the tree
// code's bail flags and counters, before every evaluation)
__global__ void __launch_bounds__(256) zero_words_kernel(uint32_t* __restrict__ a, int64_t na,
                                                        uint32_t* __restrict__ b, int64_t nb) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < na + nb;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (i < na) a[i] = 0u;
    else b[i - na] = 0u;
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
                                   const int64_t* __restrict__ idx, int64_t nidx, int64_t seg,
                                   int64_t dst_pad, T* __restrict__ Xd, T* __restrict__ yd,
                                   T* __restrict__ wd) {
  // seg > 0: dst_pad / seg samples back to back, sample t = idx[t·nidx ..
  // t·nidx + nidx) in rows [t·seg, t·seg + nidx), padded with its last row
  const int64_t total = dst_pad * (nfeat + 2);
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < total;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t f = k / dst_pad;
    const int64_t j = k - f * dst_pad;
    const int64_t t = seg ? j / seg : 0;
    const int64_t jj = j - t * seg;
    const int64_t r = idx[t * nidx + (jj < nidx ? jj : nidx - 1)];
    if (f < nfeat) Xd[f * dst_pad + j] = X[f * src_pad + r];
    else if (f == nfeat) yd[j] = y[r];
    else if (w) wd[j] = w[r];
  }
}

// Columns of shared subtrees (jit.h Columns) whose subtree failed somewhere
// (ok[g] == 0: a node non-finite on some row) become NaN on every row, so
// every tree reading the column fails, as DynamicExpressions fails a tree
// whose node is non-finite on any row.
__global__ void __launch_bounds__(256) poison_columns_kernel(const uint8_t* __restrict__ ok, float* __restrict__ cols,
                                                            int64_t n_pad) {
  const int g = blockIdx.y;
  if (ok[g]) return;
  float* o = cols + (size_t)g * n_pad;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad; i += (int64_t)gridDim.x * blockDim.x)
    o[i] = __builtin_nanf("");
}

}  // namespace

hipError_t launch_poison_columns(const uint8_t* ok, int ncol, float* cols, int64_t n_pad, hipStream_t stream) {
  if (ncol <= 0 || n_pad <= 0) return hipSuccess;
  const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n_pad + 255) / 256, 512));
  hipLaunchKernelGGL(poison_columns_kernel, dim3(gx, (unsigned)ncol), dim3(256), 0, stream, ok, cols, n_pad);
  return hipGetLastError();
}

// Kernel variants: (rows per lane R, stack slots D).
//   f32: (8, kShallowSlots) for ordinary trees, (4, kMaxSlots) for deep ones
//   f64: (4, kShallowSlots) and (2, kMaxSlots)
#ifndef SR_R32
#define SR_R32 8
#endif
static inline int variant_R(int dtype, bool deep) {
  return dtype == SRHIP_F32 ? (deep ? 4 : SR_R32) : (deep ? 2 : 4);
}

// Records of the threaded interpreter (gen_asm_interp.py): record 0 of a slot
// = {h(0), xo(0)}, record i+1 = {h(i+1), xo(i+1), imm(i), 0} where h(j) is the
// byte offset (from the block's base) of instruction j's handler in the parity
// j&1 and xo(j) = feature(j) * rs_bytes the LDS byte offset of its X operand;
// an (X[f], X[g]) immediate becomes g's byte offset.
#ifndef SR_R32
#define SR_R32 8
#endif
#if SR_R32 == 16
#include "gen/asm_interp_f32_r16_hoff.h"
#else
#include "gen/asm_interp_f32_r8_hoff.h"
#endif
__constant__ uint32_t c_ti_hoff[512] = SR_TI_HOFF_INIT;
__global__ void __launch_bounds__(64) ti_records_kernel(const Ins<float>* __restrict__ prog,
                                                        const int32_t* __restrict__ list_off, int nlist,
                                                        uint32_t rs_bytes, uint4* __restrict__ rec) {
  const int s = blockIdx.x, j = threadIdx.x;
  if (s >= nlist || j >= kVProgMax) return;
  const Ins<float>* p = prog + list_off[s];  // programs are followed by 64 OP_END of padding
  const uint32_t c0 = p[j].code, c1 = p[j + 1].code;
  const uint32_t op0 = c0 & 0xffu, op1 = c1 & 0xffu;
  uint32_t imm = __float_as_uint(p[j].imm);
  if (op0 >= (uint32_t)bin_opcode(V_XX, 0) && op0 < (uint32_t)bin_opcode(V_XX + 1, 0)) imm *= rs_bytes;
  rec[(size_t)s * 64 + j + 1] = make_uint4(c_ti_hoff[256u * (uint32_t)((j + 1) & 1) + op1], (c1 >> 16) * rs_bytes, imm, 0u);
  if (j == 0) rec[(size_t)s * 64] = make_uint4(c_ti_hoff[op0], (c0 >> 16) * rs_bytes, 0u, 0u);
}

hipError_t launch_ti_records(const Ins<float>* prog, const int32_t* list_off, int nlist,
                             uint32_t rs_bytes, uint4* rec, hipStream_t stream) {
  if (nlist <= 0) return hipSuccess;
  hipLaunchKernelGGL(ti_records_kernel, dim3((unsigned)nlist), dim3(64), 0, stream, prog, list_off, nlist,
                     rs_bytes, rec);
  return hipGetLastError();
}

bool plan_geometry(size_t esz, int R, int D, int narr, size_t part_bytes, int64_t n, int nlist,
                   EvalPlan* p, size_t tile_budget, size_t two_tile_cap, int target_wg_in, int min_per_group) {
  p->R = R;
  p->D = D;
  p->opset = OPSET_FULL;
  p->tile = 64 * R;
  p->threads = 256;
  const size_t per_tile = (size_t)narr * p->tile * esz;
  const size_t budget = tile_budget;
#ifndef SR_NTMAX
#define SR_NTMAX 16
#endif
  int nt = 1;
  while (nt * 2 <= SR_NTMAX && (int64_t)nt * 2 * p->tile <= 8192 && per_tile * nt * 2 <= budget &&
         (int64_t)nt * p->tile < n)
    nt *= 2;
  // SRHIP_TREE_NT (experiments): tiles per workgroup of tree code, any count
  if (two_tile_cap) {
    static const int force = [] { const char* e = std::getenv("SRHIP_TREE_NT"); return e ? std::atoi(e) : 0; }();
    if (force > 0 && per_tile * force <= 150 * 1024) nt = force;
  }
  // at least two tiles when two fit in two_tile_cap: a tree call covers twice
  // the rows (wide datasets, whose single tile already fills the budget)
  if (nt == 1 && two_tile_cap && per_tile * 2 <= two_tile_cap && (int64_t)p->tile < n) nt = 2;
  p->ntiles = nt;
  p->rows_wg = nt * p->tile;
  p->nrg = (int)((n + p->rows_wg - 1) / p->rows_wg);
  if (p->nrg < 1) p->nrg = 1;
  // SRHIP_TARGET_WG (experiments) overrides the caller's target
  static const int target_env = [] {
    const char* e = std::getenv("SRHIP_TARGET_WG");
    return e ? std::max(1, std::atoi(e)) : 0;
  }();
  const int target_wg = target_env ? target_env : target_wg_in;
  // SRHIP_MIN_PER_GROUP (experiments) overrides the caller's minimum trees per group
  static const int mpg_env = [] {
    const char* e = std::getenv("SRHIP_MIN_PER_GROUP");
    return e ? std::max(1, std::atoi(e)) : 0;
  }();
  if (mpg_env) min_per_group = mpg_env;
  int ntg = (target_wg + p->nrg - 1) / p->nrg;
  // at least min_per_group trees per group, unless that leaves fewer than 2048
  // workgroups (few rows); never fewer than ~4 trees (one per wave)
  const int max4 = std::max(1, (nlist + 3) / 4);
  const int floor_groups = (2048 + p->nrg - 1) / p->nrg;
  const int max_groups = std::min(max4, std::max((nlist + min_per_group - 1) / min_per_group, floor_groups));
  if (ntg > max_groups) ntg = max_groups;
  // XCD affinity: workgroups are dealt round-robin to the 8 XCDs, and block b
  // runs tree group b % ntg, so with ntg a divisor or multiple of 8 every XCD
  // runs a fixed subset of the tree groups and its L2 keeps only their code /
  // programs. SRHIP_XCD_NTG=1 turns it on; measured neutral on config #2
  // (3.40 vs 3.41 ms, profiles/r02i_evalknobs.txt), so off by default.
  static const bool xcd = [] {
    const char* e = std::getenv("SRHIP_XCD_NTG");
    return e && e[0] == '1';
  }();
  if (xcd && ntg > 1) {
    if (ntg <= 8) {
      int q = 1;
      while (q < ntg) q *= 2;
      ntg = q;
    } else {
      ntg = (ntg + 4) / 8 * 8;
    }
    if (ntg > max_groups) ntg = std::max(1, max_groups);
  }
  // the group's partial slots live in LDS next to the row tile: with many
  // trees and few tree groups (huge row counts) they bound the group size
  const size_t lds_cap = 160 * 1024 - 16;
  if (per_tile * nt + part_bytes > lds_cap) return false;
  const int max_tpb = (int)std::min<size_t>((lds_cap - per_tile * nt) / part_bytes, 1 << 20);
  const int min_groups = (nlist + max_tpb - 1) / max_tpb;
  if (ntg < min_groups) ntg = min_groups;
  if (ntg < 1) ntg = 1;
  p->tpb = (nlist + ntg - 1) / ntg;
  p->ntg = (nlist + p->tpb - 1) / p->tpb;
  p->lds_bytes = per_tile * nt + (size_t)p->tpb * part_bytes + 16;
  return p->lds_bytes <= 160 * 1024;
}

bool plan_eval(int dtype, bool deep, int opset, int mode, bool weighted, int nfeat, int64_t n,
               int nlist, EvalPlan* p) {
  const size_t esz = dtype == SRHIP_F32 ? 4 : 8;
  const int narr = nfeat + (mode == MODE_LOSS ? (weighted ? 2 : 1) : 0);
  const int R = variant_R(dtype, deep);
  const bool ok = plan_geometry(esz, R, deep ? kMaxSlots : kShallowSlots, narr,
                                2 * esz, n, nlist, p);
  p->opset = deep ? OPSET_FULL : opset;  // the deep variant is built for the full set only
  return ok;
}

template <typename T>
hipError_t launch_finalize(const EvalArgs<T>& a, double* out_sum, uint8_t* out_ok,
                           hipStream_t stream, uint32_t* cnt, uint32_t* cnt_host) {
  const int npos = a.ntg * a.tpb;
  const unsigned grid = (unsigned)((npos + kFinPos - 1) / kFinPos);
  hipLaunchKernelGGL((finalize_kernel<T>), dim3(grid), dim3(64 * kFinWaves), 0, stream, a, out_sum, out_ok, cnt,
                     cnt_host);
  return hipGetLastError();
}

namespace {
// Row-shard partials in device memory (srhip_eval_loss_packed): per tree
// [Σ w·ℓ (0 when failed), failed (1/0)], then Σ w — the layout the host side
// packs for the all-reduce (srhip/distributed.py pack_partials). verdict:
// 1 = fails statically, 2 = fails iff there are rows, 0 = the kernels decide.
__global__ void pack_partials_kernel(const double* __restrict__ sum, const uint8_t* __restrict__ ok,
                                     const uint8_t* __restrict__ verdict, int nt, int64_t rows, double wsum,
                                     double* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < nt) {
    const uint8_t v = verdict[t];
    bool good;
    double s = 0.0;
    if (v == 1) good = false;
    else if (v == 2) good = rows == 0;
    else if (rows == 0) good = true;
    else { good = ok[t] != 0; s = good ? sum[t] : 0.0; }
    out[2 * (size_t)t] = s;
    out[2 * (size_t)t + 1] = good ? 0.0 : 1.0;
  }
  if (t == 0) out[2 * (size_t)nt] = wsum;
}
}  // namespace

hipError_t launch_pack_partials(const double* sum, const uint8_t* ok, const uint8_t* verdict, int nt, int64_t rows,
                                double wsum, double* out, hipStream_t stream) {
  const unsigned grid = (unsigned)std::max(1, (nt + 255) / 256);
  hipLaunchKernelGGL(pack_partials_kernel, dim3(grid), dim3(256), 0, stream, sum, ok, verdict, nt, rows, wsum, out);
  return hipGetLastError();
}

hipError_t launch_zero_words(uint32_t* a, int64_t na, uint32_t* b, int64_t nb, hipStream_t stream) {
  if (na + nb <= 0) return hipSuccess;
  const unsigned grid = (unsigned)std::min<int64_t>(1024, (na + nb + 255) / 256);
  hipLaunchKernelGGL(zero_words_kernel, dim3(grid), dim3(256), 0, stream, a, na, b, nb);
  return hipGetLastError();
}

namespace {
// one wave per 64 constants, the four waves of a workgroup split the row groups
template <typename P>
__global__ void __launch_bounds__(256) gconst_finalize_kernel(const P* __restrict__ gpart, int nrg, int nconst,
                                                              const int32_t* __restrict__ cidx, int ncidx,
                                                              double* __restrict__ out) {
  __shared__ double sh[4][64];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int idx = blockIdx.x * 64 + lane;
  const int k = idx < ncidx ? cidx[idx] : -1;
  double acc = 0.0;
  if (k >= 0)
    for (int rg = w; rg < nrg; rg += 4) acc += (double)gpart[(size_t)rg * nconst + k];
  sh[w][lane] = acc;
  __syncthreads();
  if (w == 0 && k >= 0) out[k] = (sh[0][lane] + sh[1][lane]) + (sh[2][lane] + sh[3][lane]);
}
}  // namespace

hipError_t launch_gconst_finalize(const float* gpart, int nrg, int nconst, const int32_t* cidx, int ncidx,
                                  double* out, hipStream_t stream) {
  if (ncidx <= 0) return hipSuccess;
  hipLaunchKernelGGL(gconst_finalize_kernel<float>, dim3((unsigned)((ncidx + 63) / 64)), dim3(256), 0, stream, gpart,
                     nrg, nconst, cidx, ncidx, out);
  return hipGetLastError();
}
hipError_t launch_gconst_finalize(const double* gpart, int nrg, int nconst, const int32_t* cidx, int ncidx,
                                  double* out, hipStream_t stream) {
  if (ncidx <= 0) return hipSuccess;
  hipLaunchKernelGGL(gconst_finalize_kernel<double>, dim3((unsigned)((ncidx + 63) / 64)), dim3(256), 0, stream, gpart,
                     nrg, nconst, cidx, ncidx, out);
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
                              const int64_t* idx, int64_t nidx, int64_t seg, int64_t dst_pad, T* Xd,
                              T* yd, T* wd, hipStream_t stream) {
  const int64_t total = dst_pad * (nfeat + 2);
  unsigned grid = (unsigned)std::min<int64_t>((total + 255) / 256, 4096);
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL((gather_rows_kernel<T>), dim3(grid), dim3(256), 0, stream, X, y, w, nfeat,
                     src_pad, idx, nidx, seg, dst_pad, Xd, yd, wd);
  return hipGetLastError();
}

#define SR_INST(T)                                                                             \
  template hipError_t launch_finalize<T>(const EvalArgs<T>&, double*, uint8_t*, hipStream_t, uint32_t*, uint32_t*); \
  template hipError_t launch_pack_x<T>(const T*, int, int64_t, int64_t, int, int64_t, T*,     \
                                       int*, hipStream_t);                                    \
  template hipError_t launch_pack_vec<T>(const T*, int64_t, int64_t, T*, hipStream_t);         \
  template hipError_t launch_gather_rows<T>(const T*, const T*, const T*, int, int64_t,        \
                                            const int64_t*, int64_t, int64_t, int64_t, T*, T*, \
                                            T*, hipStream_t);
SR_INST(float)
SR_INST(double)

}  // namespace srhip
