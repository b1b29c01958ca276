// Float32 PRECISE exp / sin / cos of device_ops.h (Float64 evaluation, one
// rounding) restated on the host with fma(), old (Taylor) and new (minimax)
// polynomials, against the oracle's definition (float)f((double)x) with the
// host libm: counts of floats whose result differs, over every float of the
// fast paths' domains (sin / cos |x| <= 105615, exp [-104, 89]).
//   gcc -O2 -fopenmp -ffp-contract=off tools/check_precise.c -lm -o /tmp/check_precise && /tmp/check_precise
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static float as_f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t as_u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

static float sincos_old(float x, int want_cos) {
  const float n = want_cos ? rintf(fmaf(x, 0.318309873f, -0.5f)) : rintf(x * 0.318309873f);
  const float m = want_cos ? fmaf(n, 2.0f, 1.0f) : n + n;
  const double md = (double)m;
  double r = fma(md, -1.57079632673412561417e+00, (double)x);
  r = fma(md, -6.07710050650619224932e-11, r);
  const double s2 = r * r;
  double p = -2.81145725434552076320e-15;
  p = fma(p, s2, 7.64716373181981647590e-13);
  p = fma(p, s2, -1.60590438368216145994e-10);
  p = fma(p, s2, 2.50521083854417187751e-08);
  p = fma(p, s2, -2.75573192239858906526e-06);
  p = fma(p, s2, 1.98412698412698412698e-04);
  p = fma(p, s2, -8.33333333333333333333e-03);
  p = fma(p, s2, 1.66666666666666666667e-01);
  const double v = fma(-p * s2, r, r);
  const float f = (float)(want_cos ? -v : v);
  return as_f(as_u(f) ^ ((uint32_t)(int)n << 31));
}

static float sincos_new(float x, int want_cos) {
  const float n = want_cos ? rintf(fmaf(x, 0.318309873f, -0.5f)) : rintf(x * 0.318309873f);
  const float m = want_cos ? fmaf(n, 2.0f, 1.0f) : n + n;
  const double md = (double)m;
  double r = fma(md, -1.57079632673412561417e+00, (double)x);
  r = fma(md, -6.07710050650619224932e-11, r);
  const double s2 = r * r;
  double p = -7.34673622570819757e-13;
  p = fma(p, s2, 1.60458129180763398e-10);
  p = fma(p, s2, -2.50518043886916424e-08);
  p = fma(p, s2, 2.75573153848002669e-06);
  p = fma(p, s2, -1.98412698157051834e-04);
  p = fma(p, s2, 8.33333333325722396e-03);
  p = fma(p, s2, -1.66666666666660662e-01);
  const double v = fma(p * s2, r, r);
  const float f = (float)(want_cos ? -v : v);
  return as_f(as_u(f) ^ ((uint32_t)(int)n << 31));
}

static float exp_old(float x) {
  x = fminf(fmaxf(x, -104.0f), 89.0f);
  const double xd = (double)x;
  const double n = rint(xd * 1.4426950408889634);
  double r = fma(n, -6.93147180369123816490e-01, xd);
  r = fma(n, -1.90821492927058770002e-10, r);
  double p = 2.50521083854417187751e-08;
  p = fma(p, r, 2.75573192239858906526e-07);
  p = fma(p, r, 2.75573192239858906526e-06);
  p = fma(p, r, 2.48015873015873015873e-05);
  p = fma(p, r, 1.98412698412698412698e-04);
  p = fma(p, r, 1.38888888888888888889e-03);
  p = fma(p, r, 8.33333333333333333333e-03);
  p = fma(p, r, 4.16666666666666666667e-02);
  p = fma(p, r, 1.66666666666666666667e-01);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return (float)ldexp(p, (int)n);
}

static float exp_new(float x) {
  x = fminf(fmaxf(x, -104.0f), 89.0f);
  const double xd = (double)x;
  const double n = rint(xd * 1.4426950408889634);
  double r = fma(n, -6.93147180369123816490e-01, xd);
  r = fma(n, -1.90821492927058770002e-10, r);
  double p = 2.74715993357489975e-07;
  p = fma(p, r, 2.76351209779822652e-06);
  p = fma(p, r, 2.48019464013407408e-05);
  p = fma(p, r, 1.98411849339436464e-04);
  p = fma(p, r, 1.38888885022706824e-03);
  p = fma(p, r, 8.33333337108620349e-03);
  p = fma(p, r, 4.16666666681865250e-02);
  p = fma(p, r, 1.66666666666110797e-01);
  p = fma(p, r, 4.99999999999982736e-01);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return (float)ldexp(p, (int)n);
}


static float exp_d9(float x) {
  x = fminf(fmaxf(x, -104.0f), 89.0f);
  const double xd = (double)x;
  const double n = rint(xd * 1.4426950408889634);
  double r = fma(n, -6.93147180369123816490e-01, xd);
  r = fma(n, -1.90821492927058770002e-10, r);
  double p = 2.74930749914601988e-06;
  p = fma(p, r, 2.48808415869387003e-05);
  p = fma(p, r, 1.98415392254195396e-04);
  p = fma(p, r, 1.38888110820991131e-03);
  p = fma(p, r, 8.33333309485798264e-03);
  p = fma(p, r, 4.16666669626017602e-02);
  p = fma(p, r, 1.66666666672660641e-01);
  p = fma(p, r, 4.99999999996637579e-01);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return (float)ldexp(p, (int)n);
}

int main(void) {
  long long bad[7] = {0};
  long long total[3] = {0};
  // every float bit pattern; domains filtered
#pragma omp parallel for reduction(+ : bad[:7], total[:3]) schedule(dynamic, 1 << 16)
  for (long long u = 0; u < (1LL << 32); ++u) {
    const float x = as_f((uint32_t)u);
    if (!isfinite(x)) continue;
    if (fabsf(x) <= 105615.0f) {
      const float rs = (float)sin((double)x), rc = (float)cos((double)x);
      total[0] += 1;
      total[1] += 1;
      bad[0] += as_u(sincos_old(x, 0)) != as_u(rs) && !(rs == 0.0f && sincos_old(x, 0) == 0.0f);
      bad[1] += as_u(sincos_new(x, 0)) != as_u(rs) && !(rs == 0.0f && sincos_new(x, 0) == 0.0f);
      bad[2] += as_u(sincos_old(x, 1)) != as_u(rc) && !(rc == 0.0f && sincos_old(x, 1) == 0.0f);
      bad[3] += as_u(sincos_new(x, 1)) != as_u(rc) && !(rc == 0.0f && sincos_new(x, 1) == 0.0f);
    }
    if (x >= -104.0f && x <= 89.0f) {
      const float re = (float)exp((double)x);
      total[2] += 1;
      bad[4] += as_u(exp_old(x)) != as_u(re);
      bad[5] += as_u(exp_new(x)) != as_u(re);
      bad[6] += as_u(exp_d9(x)) != as_u(re);
    }
  }
  printf("sin: %lld floats, old %lld differ, new %lld differ\n", total[0], bad[0], bad[1]);
  printf("cos: %lld floats, old %lld differ, new %lld differ\n", total[1], bad[2], bad[3]);
  printf("exp: %lld floats, old %lld differ, new %lld differ, degree 9: %lld\n", total[2], bad[4], bad[5], bad[6]);
  return 0;
}
