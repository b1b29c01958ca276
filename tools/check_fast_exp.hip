// check_fast_exp.hip — exhaustive validation of the engine's f32 exp
// (device_ops.h fast_exp_f32) on the GPU: every float, compared with the
// correctly rounded value (f64 exp rounded once to f32) and with OCML expf.
// Prints the max ulp distance over finite inputs (tools/, not the library).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include "../symbolicregression.jl_amd/csrc/device_ops.h"

__device__ __forceinline__ long long ordered(float f) {
  const int i = __float_as_int(f);
  return i < 0 ? -(long long)(i & 0x7fffffff) : (long long)i;
}

__global__ void check(uint32_t base, unsigned long long* worst, unsigned long long* worst_ocml,
                      unsigned long long* bad_special) {
  const uint32_t bits = base + blockIdx.x * blockDim.x + threadIdx.x;
  const float x = __int_as_float((int)bits);
  if (!__builtin_isfinite(x)) return;
  const float ref = (float)exp((double)x);
  const float f = srhip::dev::fast_exp_f32(x);
  const float o = expf(x);
  long long d = ordered(f) - ordered(ref);
  d = d < 0 ? -d : d;
  long long d2 = ordered(o) - ordered(ref);
  d2 = d2 < 0 ? -d2 : d2;
  if (__builtin_isinf(ref) != __builtin_isinf(f) || __builtin_isnan(f)) atomicAdd(bad_special, 1ull);
  else atomicMax(worst, (unsigned long long)((d << 32) | bits));
  atomicMax(worst_ocml, (unsigned long long)((d2 << 32) | bits));
}

int main() {
  unsigned long long *w, *wo, *bs;
  (void)hipMalloc(&w, 8); (void)hipMalloc(&wo, 8); (void)hipMalloc(&bs, 8);
  (void)hipMemset(w, 0, 8); (void)hipMemset(wo, 0, 8); (void)hipMemset(bs, 0, 8);
  const uint32_t chunk = 1u << 26;
  for (uint64_t b = 0; b < (1ull << 32); b += chunk)
    hipLaunchKernelGGL(check, dim3(chunk / 256), dim3(256), 0, 0, (uint32_t)b, w, wo, bs);
  unsigned long long hw, ho, hb;
  (void)hipMemcpy(&hw, w, 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(&ho, wo, 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(&hb, bs, 8, hipMemcpyDeviceToHost);
  uint32_t xb = (uint32_t)hw, xo = (uint32_t)ho;
  float x, y;
  memcpy(&x, &xb, 4); memcpy(&y, &xo, 4);
  printf("fast_exp_f32: max ulp %llu (at x=%a), inf/nan mismatches %llu\n", hw >> 32, x, hb);
  printf("ocml expf   : max ulp %llu (at x=%a)\n", ho >> 32, y);
  return (hw >> 32) <= 2 && hb == 0 ? 0 : 1;
}
