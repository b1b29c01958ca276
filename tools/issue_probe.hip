// issue_probe.hip — measures how gfx950 issues mixed VALU / SALU / branch
// streams, to price the interpreter's dispatch (tools/, not part of the
// library). Each wave runs ITER iterations of a body of NV independent
// v_add_f32, NS independent s_add_u32 and NB uniform compare+branch pairs.
// Grid: 256 CUs x occ workgroups of 256 threads (one wave per SIMD each).
// Prints cycles per iteration per SIMD (throughput view) for each config.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int NV, int NS, int NB, int TAKEN>
__global__ void __launch_bounds__(256) probe(float* out, int iters) {
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = threadIdx.x * 0.001f + i;
  unsigned s0 = 1, s1 = 2, s2 = 3, s3 = 4;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < NV; ++k) asm volatile("v_add_f32 %0, 1.0, %0" : "+v"(v[k & 7]));
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      if ((k & 3) == 0) asm volatile("s_add_u32 %0, %0, 3" : "+s"(s0) :: "scc");
      if ((k & 3) == 1) asm volatile("s_add_u32 %0, %0, 5" : "+s"(s1) :: "scc");
      if ((k & 3) == 2) asm volatile("s_add_u32 %0, %0, 7" : "+s"(s2) :: "scc");
      if ((k & 3) == 3) asm volatile("s_add_u32 %0, %0, 9" : "+s"(s3) :: "scc");
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      if (TAKEN) asm volatile("s_cmp_lt_u32 %0, 0xffffffff\n\ts_cbranch_scc1 1f\n\ts_nop 0\n1:" :: "s"(s0) : "scc");
      else asm volatile("s_cmp_gt_u32 %0, 0xffffffff\n\ts_cbranch_scc1 1f\n\ts_nop 0\n1:" :: "s"(s0) : "scc");
    }
  }
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc += v[i];
  if (acc == 12345.f) out[threadIdx.x] = acc + (float)(s0 + s1 + s2 + s3);
}

template <int NV, int NS, int NB, int TAKEN>
void run(const char* name, float* d, int occ) {
  const int iters = 4000;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  dim3 grid(256 * occ), block(256);
  hipLaunchKernelGGL((probe<NV, NS, NB, TAKEN>), grid, block, 0, 0, d, 16);
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL((probe<NV, NS, NB, TAKEN>), grid, block, 0, 0, d, iters);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  // cycles per iteration per SIMD at 2.4 GHz, all occ waves of the SIMD together
  const double cyc = ms * 1e-3 * 2.4e9 / iters;
  printf("%-28s occ=%d  %8.1f cyc/iter/SIMD  (%6.2f per wave-iter)\n", name, occ, cyc, cyc / occ);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
}

int main() {
  float* d;
  CHECK(hipMalloc(&d, 4096));
  for (int occ : {1, 2, 4, 8}) {
    run<32, 0, 0, 0>("valu32", d, occ);
    run<0, 32, 0, 0>("salu32", d, occ);
    run<0, 0, 16, 1>("br16 taken", d, occ);
    run<0, 0, 16, 0>("br16 not-taken", d, occ);
    run<32, 32, 0, 0>("valu32+salu32", d, occ);
    run<32, 0, 16, 1>("valu32+br16t", d, occ);
    run<32, 16, 8, 1>("valu32+salu16+br8t", d, occ);
  }
  CHECK(hipFree(d));
  return 0;
}
