/* Search for numel<16 serial-path draws whose double Box-Muller value lies within a few
 * double ulps of an fp32 rounding boundary (the midpoint between two floats), the only
 * place where a 1-ulp difference between glibc's log1p/sin/cos (the reference) and the
 * device's ocml ones could change z.  Test infrastructure (tests/test_gpu_serial_straddle.py
 * runs the device on the candidates against the oracle):
 *   gcc -O2 -fopenmp tools/straddle_search.c -lm -o /tmp/straddle && /tmp/straddle s0 s1 L
 * For seeds [s0, s1) and stream positions P = 16 m < L (a fast tensor of P elements in
 * front, then a 2-element tensor), prints "seed P idx dist" for the cos (idx 0) and sin
 * (idx 1) values with dist < 2 double ulps.  Follows DistributionsHelper.h:189-221 as
 * oracle/fks_oracle.c normal_double does. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { uint32_t s[624]; int i; } mt_t;
static void mt_seed(mt_t *m, uint32_t seed) {
  m->s[0] = seed;
  for (int j = 1; j < 624; j++) m->s[j] = 1812433253u * (m->s[j - 1] ^ (m->s[j - 1] >> 30)) + (uint32_t)j;
  m->i = 624;
}
static uint32_t mt_next(mt_t *m) {
  if (m->i == 624) {
    for (int k = 0; k < 624; k++) {
      uint32_t y = (m->s[k] & 0x80000000u) | (m->s[(k + 1) % 624] & 0x7fffffffu);
      m->s[k] = m->s[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    m->i = 0;
  }
  uint32_t y = m->s[m->i++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}
/* distance of v to the nearest midpoint between two adjacent floats, in ulps of v */
static double mid_dist(double v) {
  const float f = (float)v;
  const float nb = (double)f < v ? nextafterf(f, INFINITY) : nextafterf(f, -INFINITY);
  const double mid = 0.5 * ((double)f + (double)nb);
  const double ulp = nextafter(fabs(v), INFINITY) - fabs(v);
  return fabs(v - mid) / ulp;
}
int main(int argc, char **argv) {
  const long s0 = atol(argv[1]), s1 = atol(argv[2]);
  const long L = atol(argv[3]);
#pragma omp parallel for schedule(dynamic)
  for (long seed = s0; seed < s1; seed++) {
    mt_t m;
    mt_seed(&m, (uint32_t)seed);
    uint32_t w[4];
    for (int k = 0; k < 4; k++) w[k] = mt_next(&m);
    for (long P = 0; P + 16 < L; P += 16) {
      /* words P..P+3 are w[0..3]; advance the window by 16 words per step */
      const uint64_t a = ((uint64_t)w[0] << 32) | w[1], b = ((uint64_t)w[2] << 32) | w[3];
      const double u1 = (double)(a & ((1ULL << 53) - 1)) * (1.0 / 9007199254740992.0);
      const double u2 = (double)(b & ((1ULL << 53) - 1)) * (1.0 / 9007199254740992.0);
      const double r = sqrt(-2.0 * log1p(-u2));
      const double th = 2.0 * 3.14159265358979323846 * u1;
      const double vc = r * cos(th), vs = r * sin(th);
      const double dc = mid_dist(vc), ds = mid_dist(vs);
      const unsigned long long ma = a & ((1ULL << 53) - 1), mb = b & ((1ULL << 53) - 1);
      if (dc < 2.0) printf("%ld %ld 0 %.3f %llx %llx\n", seed, P, dc, ma, mb);
      if (ds < 2.0) printf("%ld %ld 1 %.3f %llx %llx\n", seed, P, ds, ma, mb);
      for (int k = 0; k < 12; k++) (void)mt_next(&m);  /* words P+4 .. P+15 */
      for (int k = 0; k < 4; k++) w[k] = mt_next(&m);   /* words P+16 .. P+19 */
    }
  }
  return 0;
}
