/* Division by a constant c through its correctly rounded reciprocal
 * y = RN(1/c) and one FMA correction (Markstein):
 *     q = RN(a*y); r = fma(-c, q, a) (exact); q' = RN(r*y + q)
 * must equal the IEEE quotient RN(a/c) for |a|, |c| in [2^-60, 2^60]
 * (the range tree code admits; outside it the IEEE routine runs).
 * Checks every significand of a in one binade for a set of divisors,
 * plus random (a, c) pairs over the whole range. Exit 1 on a mismatch. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float fb(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t bf(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

static int check(float a, float c) {
  const float y = 1.0f / c;
  const float q = a * y;
  const float r = fmaf(-c, q, a);
  const float q1 = fmaf(r, y, q);
  const float ref = a / c;
  if (bf(q1) != bf(ref)) {
    printf("MISMATCH a=%a c=%a fast=%a ieee=%a\n", a, c, q1, ref);
    return 1;
  }
  return 0;
}

static uint64_t s = 88172645463325252ull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }

int main(int argc, char** argv) {
  long bad = 0, n = 0;
  const long nrand = argc > 1 ? atol(argv[1]) : 200000000L;
  /* exhaustive significands of a in [1, 2) (and the sign) for these divisors */
  const float divs[] = {3.0f, 7.0f, 0.1f, 1.7f, 2.9718f, -0.47f, 1.9999999f, 1.0000001f, 1.5f, 10.0f,
                        0x1.fffffep0f, 0x1.000002p0f, 0x1.555556p0f, 0x1.c71c72p-3f, 6.2831855f, 0.3183099f};
  for (size_t k = 0; k < sizeof divs / sizeof divs[0]; ++k) {
    for (uint32_t m = 0; m < (1u << 23); ++m) {
      const float a = fb(0x3f800000u | m);
      bad += check(a, divs[k]);
      bad += check(-a * 0x1p37f, divs[k]);
      n += 2;
      if (bad > 10) return 1;
    }
  }
  /* exhaustive significands of a for random divisor significands */
  const long nd = argc > 2 ? atol(argv[2]) : 0;
  for (long k = 0; k < nd; ++k) {
    const float c = fb(0x3f800000u | (uint32_t)(rnd() & 0x7fffff));
    for (uint32_t m = 0; m < (1u << 23); ++m) {
      bad += check(fb(0x3f800000u | m), c);
      ++n;
      if (bad > 10) return 1;
    }
  }
  /* random pairs over the admitted range */
  for (long i = 0; i < nrand; ++i) {
    const uint64_t r = rnd();
    const int ea = (int)(r % 121) - 60, ec = (int)((r >> 8) % 121) - 60;
    const float a = ldexpf(fb(0x3f800000u | (uint32_t)((r >> 16) & 0x7fffff)), ea) * ((r >> 40) & 1 ? -1.f : 1.f);
    const float c = ldexpf(fb(0x3f800000u | (uint32_t)((r >> 41) & 0x7fffff)), ec) * ((r >> 63) & 1 ? -1.f : 1.f);
    if (fabsf(a) >= 0x1p60f || fabsf(c) >= 0x1p60f) continue;
    bad += check(a, c);
    ++n;
    if (bad > 10) return 1;
  }
  printf("checked %ld quotients, %ld mismatches\n", n, bad);
  return bad != 0;
}
