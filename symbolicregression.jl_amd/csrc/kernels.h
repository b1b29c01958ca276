// kernels.h — launch interface of the HIP kernels (kernels.hip) for the
// host runtime (api.cpp). No torch, no HIP types beyond the stream.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "srhip_internal.h"

namespace srhip {

enum EvalMode : int { MODE_LOSS = 0, MODE_OUT = 1 };

// Per-(tree, row-group) partial result: Σ w·ℓ over the group's rows and the
// non-finite marker (0, or NaN when some checked value was non-finite).
template <typename T>
struct alignas(2 * sizeof(T)) Part {
  T sum;
  T chk;
};

template <typename T>
struct EvalArgs {
  const Ins<T>* prog;      // all programs
  const int32_t* tree_off; // [ntrees] program start per tree
  const int32_t* list;     // tree ids handled by this launch, cost-descending
  const int32_t* list_off; // [nlist] program start of list[s] (= tree_off[list[s]])
  uint32_t* fail;          // [nlist] MODE_LOSS: set once slot s is known to fail (early exit)
  const uint4* ti_rec;     // [nlist][64] threaded-interpreter records (nullptr: C++ dispatch)
  int nlist;
  const T* X;              // [nfeat][n_pad] feature-major, rows padded
  const T* y;              // [n_pad]
  const T* w;              // [n_pad] or nullptr
  int64_t n;               // valid rows
  int64_t n_pad;
  int nfeat;
  int ntiles;              // row tiles per workgroup
  int ntg;                 // tree groups
  int tpb;                 // trees per group
  int nrg;                 // row groups
  int loss;
  int rotate;              // MODE_LOSS: start each wave's tree sequence at row-group-dependent offsets
  int contig;              // tree group g holds list slots [g*tpb, (g+1)*tpb) (tree code: a group's
                           // code is one contiguous range); 0: slots dealt in snake order
  double lparam;           // the loss parameter (LossFunctions' Float64 field, not rounded to T)
  Part<T>* partial;        // [nrg][ntg*tpb]
  T* out;                  // MODE_OUT: [ntrees][out_stride]
  int64_t out_stride;
  // per-tree row sets (srhip_eval_loss_rowsets; interpreter, one tree per
  // group): tree t reads rows [t·seg, t·seg + n) of X / y / w; 0 = shared rows
  int64_t seg = 0;
  // finalize only: the launch wrote 4-byte partials (Σ; float at partial + rg·npos + pos) and a
  // failed tree is the one whose slot failure flag is set (the hand-written loss tree loops)
  int part4 = 0;
};

// Geometry of one evaluation launch, chosen by plan_eval().
struct EvalPlan {
  int R;          // rows per lane per instruction
  int D;          // stack slots of the kernel variant (kShallowSlots or kMaxSlots)
  int opset;      // OpSet the kernel variant is compiled for
  int tile;       // rows per tile = 64 * R
  int ntiles;
  int rows_wg;    // rows per workgroup
  int nrg, ntg, tpb;
  size_t lds_bytes;
  int threads;    // workgroup size
  // tree code only: row groups [0, nbig) of ntiles tiles, then row groups of
  // ts tiles (the last round of workgroups in smaller pieces); nbig < 0: all full
  int nbig = -1, ts = 0;
};

// Choose the geometry for `nlist` trees over `n` rows; returns false when the
// row tile of this feature count does not fit in LDS.
// Threaded-interpreter instruction records of every list slot (f32 shallow
// programs; eval_kernel.h / gen_asm_interp.py): [nlist][64] uint4.
bool ti_compiled();  // eval kernels built with the threaded interpreter (SR_TI)
hipError_t launch_ti_records(const Ins<float>* prog, const int32_t* list_off, int nlist,
                             uint32_t rs_bytes, uint4* rec, hipStream_t stream);

bool plan_eval(int dtype, bool deep, int opset, int mode, bool weighted, int nfeat,
               int64_t n, int nlist, EvalPlan* plan);
// Same, for explicit R / D / LDS arrays / partial bytes per tree slot.
// target_wg: workgroups the tree groups aim at; min_per_group: trees a group
// keeps at least (the loss tree code: 16384 / 64, measured on config #2)
bool plan_geometry(size_t esz, int R, int D, int narr, size_t part_bytes, int64_t n,
                   int nlist, EvalPlan* plan, size_t tile_budget = 40 * 1024, size_t two_tile_cap = 0,
                   int target_wg = 8192, int min_per_group = 4);

// ---- constant gradients (grad_kernels.hip) -----------------------------------
constexpr int kGradG = 4;  // tangents per pass (constants per "tangent group")
enum GradMode : int { GRAD_LOSS = 0, GRAD_OUT = 1 };

template <typename T>
struct GradArgs {
  const Ins<T>* prog;       // programs compiled for gradients (no folding)
  const int32_t* tree_off;
  const int32_t* items;     // work items: tree | (tangent group << 24)
  int nitems;
  const int32_t* const_off; // [ntrees+1]
  const T* X;
  const T* y;
  const T* w;
  int64_t n, n_pad;
  int nfeat;
  int ntiles, ntg, tpb, nrg;
  int loss;
  double lparam;
  int G;                    // tangents carried by this launch (1, 2 or kGradG)
  int opset;                // OPSET_BASIC: the programs use only the basic operators
  T* partial;               // [nrg][ntg*tpb][2 + G]
  T* out_value;             // GRAD_OUT: [ntrees][out_stride]
  T* out_grad;              // GRAD_OUT: [total consts][out_stride]
  int64_t out_stride;
  int dyn = 0;              // waves take their items from an LDS counter (SRHIP_INTERP_DYN)
};

bool plan_grad(int dtype, bool deep, int G, int mode, bool weighted, int nfeat, int64_t n,
               int nitems, EvalPlan* plan);
template <typename T>
hipError_t launch_grad(const EvalPlan& plan, const GradArgs<T>& a, int mode, hipStream_t stream);
template <typename T>
hipError_t launch_grad_finalize(const GradArgs<T>& a, double* out_sum, uint8_t* out_ok,
                                double* out_dloss, hipStream_t stream);

// Σ over row groups of the gradient tree code's per-constant partials:
// out[cidx[k]] = Σ_rg gpart[rg][cidx[k]] in fp64 (jit_grad.cpp).
// zero a[0..na) and b[0..nb) (uint32 words) in one launch
hipError_t launch_zero_words(uint32_t* a, int64_t na, uint32_t* b, int64_t nb, hipStream_t stream);
// [Σ w·ℓ, failed] per tree + Σ w into device memory (srhip_eval_loss_packed)
hipError_t launch_pack_partials(const double* sum, const uint8_t* ok, const uint8_t* verdict, int nt, int64_t rows,
                                double wsum, double* out, hipStream_t stream);
hipError_t launch_gconst_finalize(const float* gpart, int nrg, int nconst, const int32_t* cidx, int ncidx,
                                  double* out, hipStream_t stream);
// the same over Float64 partials (jit64.cpp's gradient tree code)
hipError_t launch_gconst_finalize(const double* gpart, int nrg, int nconst, const int32_t* cidx, int ncidx,
                                  double* out, hipStream_t stream);

template <typename T>
hipError_t launch_eval(const EvalPlan& plan, const EvalArgs<T>& a, int mode,
                       hipStream_t stream);

// Σ over row groups of the partials → per-tree fp64 sum and ok flag; clears
// the failure flags it read (a.fail) and, given cnt, copies the two tree-code
// counters to cnt_host and clears them.
template <typename T>
hipError_t launch_finalize(const EvalArgs<T>& a, double* out_sum,
                           uint8_t* out_ok, hipStream_t stream, uint32_t* cnt = nullptr,
                           uint32_t* cnt_host = nullptr);

// Dataset packing: src rows [0, rows) in Julia (nfeat, n) column-major layout
// (layout 0) or feature-major with row stride src_stride (layout 1) →
// dst [nfeat][n_pad], padding rows replicate the last row. Sets *bad if a
// non-finite value is seen.
template <typename T>
hipError_t launch_pack_x(const T* src, int layout, int64_t src_stride,
                         int64_t rows, int nfeat, int64_t n_pad, T* dst,
                         int* bad, hipStream_t stream);
template <typename T>
hipError_t launch_pack_vec(const T* src, int64_t rows, int64_t n_pad, T* dst,
                           hipStream_t stream);
// Shared-subtree columns (jit.h Columns): every row of column g of cols
// ([ncol][n_pad]) set to NaN when ok[g] == 0 (device memory).
hipError_t launch_poison_columns(const uint8_t* ok, int ncol, float* cols, int64_t n_pad, hipStream_t stream);
// Row gather for score_func_batch: dst[f][k] = src[f][idx[k]] (+ y, w);
// seg > 0: one sample of nidx rows per segment of seg rows (per-tree samples,
// srhip_eval_loss_rowsets), idx = [dst_pad / seg][nidx].
template <typename T>
hipError_t launch_gather_rows(const T* X, const T* y, const T* w, int nfeat,
                              int64_t src_pad, const int64_t* idx, int64_t nidx, int64_t seg,
                              int64_t dst_pad, T* Xd, T* yd, T* wd,
                              hipStream_t stream);

}  // namespace srhip
