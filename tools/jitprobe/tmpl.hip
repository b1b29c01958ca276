#include <hip/hip_runtime.h>
extern "C" __global__ void __launch_bounds__(64) sr_area() {
  asm volatile("s_endpgm\n.fill " SIZE_WORDS ", 4, 0xbf810000\n");
}
extern "C" __global__ void __launch_bounds__(256) sr_tmpl(float* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1.0f;
}
