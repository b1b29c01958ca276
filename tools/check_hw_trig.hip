// check_hw_trig.hip — accuracy of a sin/cos built on the hardware v_sin_f32 /
// v_cos_f32 (input in revolutions) after the engine's Cody-Waite reduction,
// over every float with |x| <= 105615, against the correctly rounded value.
// Exploration tool (tools/), not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__device__ __forceinline__ long long ordered(float f) {
  const int i = __float_as_int(f);
  return i < 0 ? -(long long)(i & 0x7fffffff) : (long long)i;
}
__device__ __forceinline__ float hw_sincos(float x, int want_cos) {
  const float q = __builtin_rintf(x * 0.636619772f);
  float r = __builtin_fmaf(q, -1.57079601e+00f, x);
  r = __builtin_fmaf(q, -3.13916473e-07f, r);
  r = __builtin_fmaf(q, -5.39030253e-15f, r);
  const int i = (int)q + want_cos;
  const float t = r * 0.159154943f;  // revolutions
  const float ps = __builtin_amdgcn_sinf(t);
  const float pc = __builtin_amdgcn_cosf(t);
  const float v = (i & 1) ? pc : ps;
  return (i & 2) ? -v : v;
}
__global__ void check(uint32_t base, int want_cos, unsigned long long* worst, unsigned long long* hist) {
  const uint32_t bits = base + blockIdx.x * blockDim.x + threadIdx.x;
  const float x = __int_as_float((int)bits);
  if (!(__builtin_fabsf(x) <= 105615.0f)) return;
  const float ref = want_cos ? (float)cos((double)x) : (float)sin((double)x);
  const float f = hw_sincos(x, want_cos);
  long long d = ordered(f) - ordered(ref);
  d = d < 0 ? -d : d;
  atomicMax(worst, (unsigned long long)((d << 32) | bits));
  atomicAdd(&hist[d > 7 ? 7 : d], 1ull);
}
int main() {
  unsigned long long *w, *h;
  (void)hipMalloc(&w, 8); (void)hipMalloc(&h, 64);
  for (int c = 0; c < 2; ++c) {
    (void)hipMemset(w, 0, 8); (void)hipMemset(h, 0, 64);
    const uint32_t chunk = 1u << 26;
    for (uint64_t b = 0; b < (1ull << 32); b += chunk)
      hipLaunchKernelGGL(check, dim3(chunk / 256), dim3(256), 0, 0, (uint32_t)b, c, w, h);
    unsigned long long hw, hh[8];
    (void)hipMemcpy(&hw, w, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hh, h, 64, hipMemcpyDeviceToHost);
    uint32_t xb = (uint32_t)hw; float x; memcpy(&x, &xb, 4);
    printf("%s: max ulp %llu at x=%a; ulp histogram 0..7+:", c ? "cos" : "sin", hw >> 32, x);
    for (int k = 0; k < 8; ++k) printf(" %llu", hh[k]);
    printf("\n");
  }
  return 0;
}
