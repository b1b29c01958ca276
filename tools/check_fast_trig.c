/* CPU validation of the engine's fast f32 sin/cos (same operations, same
 * constants as device_ops.h fast_sincos): max ulp error vs the correctly
 * rounded value (double-evaluated, rounded once) over all floats in
 * [-105615, 105615] (exhaustive with stride), which is the fast path's domain. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>

static float fast_sincos(float x, int want_cos) {
  float q = rintf(x * 0.636619772f);
  float r = fmaf(q, -1.57079601e+00f, x);
  r = fmaf(q, -3.13916473e-07f, r);
  r = fmaf(q, -5.39030253e-15f, r);
  int i = (int)q + (want_cos ? 1 : 0);
  float s = r * r;
  float pc = fmaf(fmaf(fmaf(2.44331571e-5f, s, -1.38873163e-3f), s, 4.16666457e-2f), s, -5.00000000e-1f);
  pc = fmaf(pc, s, 1.0f);
  float ps = fmaf(fmaf(-1.95152959e-4f, s, 8.33216087e-3f), s, -1.66666546e-1f);
  ps = fmaf(ps * s, r, r);
  float t = (i & 1) ? pc : ps;
  return (i & 2) ? -t : t;
}

static int64_t ulp_dist(float a, float b) {
  int32_t ia, ib;
  memcpy(&ia, &a, 4); memcpy(&ib, &b, 4);
  int64_t oa = ia < 0 ? -(int64_t)(ia & 0x7fffffff) : ia;
  int64_t ob = ib < 0 ? -(int64_t)(ib & 0x7fffffff) : ib;
  return oa > ob ? oa - ob : ob - oa;
}

int main(int argc, char** argv) {
  int stride = argc > 1 ? atoi(argv[1]) : 1;
  int64_t worst[2] = {0, 0};
  float wx[2] = {0, 0};
  double sumu[2] = {0, 0};
  long n = 0;
  /* all non-negative floats up to 105615 (and their negatives by symmetry check) */
  for (uint32_t b = 0; b < 0x47CE4780u; b += stride) {
    float x;
    memcpy(&x, &b, 4);
    for (int sgn = 0; sgn < 2; ++sgn) {
      float xx = sgn ? -x : x;
      for (int k = 0; k < 2; ++k) {
        float got = fast_sincos(xx, k);
        float ref = (float)(k ? cos((double)xx) : sin((double)xx));
        int64_t d = ulp_dist(got, ref);
        sumu[k] += d;
        if (d > worst[k]) { worst[k] = d; wx[k] = xx; }
      }
    }
    n += 2;
  }
  printf("samples %ld  sin: max %lld ulp at %.9g (mean %.3f)  cos: max %lld ulp at %.9g (mean %.3f)\n", n,
         (long long)worst[0], wx[0], sumu[0] / n, (long long)worst[1], wx[1], sumu[1] / n);
  return 0;
}
