/* CPU validation of the engine's fast f32 sin/cos (same operations, same
 * constants as device_ops.h fast_sincos): max ulp error vs the correctly
 * rounded value (double-evaluated, rounded once) over all floats in
 * [-105615, 105615] (exhaustive with stride), which is the fast path's domain. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>

/* Reduction by pi to r in [-pi/2, pi/2] and one odd polynomial:
 *   sin x = (-1)^n sin(x - n pi),            n = rint(x / pi)
 *   cos x = (-1)^(n+1) sin(x - (n + 1/2) pi), n = rint(x / pi - 1/2)
 * r = x - m pi/2 (m = 2n or 2n+1) by the 3-part Cody-Waite split of pi/2;
 * sin r = r + r^3 P(r^2), P minimax of degree 3 (tools/fit_sin.py). */
static float fast_sincos(float x, int want_cos) {
  const float n = want_cos ? rintf(fmaf(x, 0.318309873f, -0.5f)) : rintf(x * 0.318309873f);
  const float m = want_cos ? fmaf(n, 2.0f, 1.0f) : n + n;
  float r = fmaf(m, -1.57079601e+00f, x);
  r = fmaf(m, -3.13916473e-07f, r);
  r = fmaf(m, -5.39030253e-15f, r);
  const float s = r * r;
  float p = fmaf(fmaf(fmaf(2.606342605e-06f, s, -1.980987436e-04f), s, 8.333070204e-03f), s,
                 -1.666665971e-01f);
  p = p * s;
  float v = want_cos ? fmaf(p, -r, -r) : fmaf(p, r, r);
  uint32_t vb, sg = ((uint32_t)(int32_t)n) << 31;
  memcpy(&vb, &v, 4);
  vb ^= sg;
  memcpy(&v, &vb, 4);
  return v;
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
