// jit64_template.hip — the code object that carries Float64 tree code (jit64.cpp).
//
// The Float64 counterpart of jit_template.hip: built once (make) into a
// standalone gfx950 code object, embedded in libsrhip.so, copied and patched
// per program. Three kernels:
//   sr_jit64_routines  never launched: the Float64 operator routines of
//                      gen_jit64.py (one region: Float64 has no FAST path);
//   sr_jit64_area      never launched: s_endpgm, then the code area;
//   sr_jit64_eval(_w)  the driver: one workgroup = (row group, tree group) as
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

template <bool W>
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
      asm volatile("s_swappc_b64 s[76:77], %[tgt]"
                   : "+{v[44:45]}"(lsum), "+{v[40:41]}"(chk), "+{v42}"(la), "+{s64}"(tile), "={s69}"(status)
                   : [tgt] "s"(target), "{v43}"(lane2), "{s65}"(nt_u), "{s66}"(partial), "{s67}"(tilebytes),
                     "{s68}"(woff)
                   : SR_JIT64_CLOBBERS, "memory");
      (void)status;
    }
    lsum = wave_sum(lsum);
    chk = __builtin_amdgcn_ballot_w64(chk != chk) != 0 ? __builtin_nan("") : 0.0;
    if (lane == 0) dst[i] = Part<double>{lsum, chk};
    if (!skip && chk != chk && lane == 0)
      __hip_atomic_store(a.fail + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

extern "C" __global__ void __launch_bounds__(1024) sr_jit64_eval(Jit64Args ja) { jit64_eval_body<false>(ja); }
extern "C" __global__ void __launch_bounds__(1024) sr_jit64_eval_w(Jit64Args ja) { jit64_eval_body<true>(ja); }
