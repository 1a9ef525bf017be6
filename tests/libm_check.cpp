// Host checker for fate-llm_amd/csrc/fks_libm.h (test infrastructure, built by
// tests/test_libm_serial.py with g++ -O2 -ffp-contract=off): the header's log1p / sin /
// cos against this host's glibc, which is what the reference's CPU z stream calls.
//   libm_check log1p N      -> "bad <count>" over N inputs -u2, u2 = m 2^-53
//   libm_check sincos N     -> "bad <count>" then up to 256 "theta mine glibc" hex lines
//   libm_check z            -> stdin "a b which" (53-bit hex, which 0 = cos, 1 = sin);
//                              stdout the fp32 bits of the serial-path z, header and glibc
//   libm_check logf [fma]   -> "bad <count>": logf_glibc against logf on all 2^24 u1 = 1 - k 2^-24
//   libm_check sincosf [fma] -> "bad <count>": sincosf_glibc against sinf / cosf on all 2^24
//                              theta_k = (float)(2 pi_double k 2^-24)
//                              (fma: the fused evaluation form the device runs)
//   libm_check theta        -> "bad <count>": theta_of(k) against torch's expression, all 2^24 k
//   libm_check consts       -> the header's logf / sincosf constants, one %a per line, in the
//                              order tools/libm_float_consts.py lists glibc's
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../fate-llm_amd/csrc/fks_libm.h"

static uint64_t xs = 88172645463325252ull;
static uint64_t next() {
  xs ^= xs << 13;
  xs ^= xs >> 7;
  xs ^= xs << 17;
  return xs;
}
static double u53(uint64_t m) { return (double)(m & ((1ull << 53) - 1)) * (1.0 / 9007199254740992.0); }

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  if (!strcmp(argv[1], "log1p")) {
    const long n = atol(argv[2]);
    long bad = 0;
    for (long i = 0; i < n; i++) {
      uint64_t m = next() & ((1ull << 53) - 1);
      if (i % 4 == 1) m >>= (next() >> 58);  // small u2 as well
      const double x = -u53(m);
      if (fks_libm::bits(fks_libm::log1p(x)) != fks_libm::bits(log1p(x))) bad++;
    }
    printf("bad %ld\n", bad);
    return 0;
  }
  if (!strcmp(argv[1], "sincos")) {
    const long n = atol(argv[2]);
    long bad = 0;
    for (long i = 0; i < n; i++) {
      uint64_t m = next() & ((1ull << 53) - 1);
      if (i % 8 == 1) m >>= (next() >> 58);
      const double th = 2.0 * 3.14159265358979323846 * u53(m);
      for (int s = 0; s < 2; s++) {
        const double mine = fks_libm::sin_or_cos(th, s), ref = s ? sin(th) : cos(th);
        if (fks_libm::bits(mine) != fks_libm::bits(ref)) {
          if (bad < 256)
            fprintf(stderr, "%d %016llx %016llx %016llx\n", s, (unsigned long long)fks_libm::bits(th),
                    (unsigned long long)fks_libm::bits(mine), (unsigned long long)fks_libm::bits(ref));
          bad++;
        }
      }
    }
    printf("bad %ld\n", bad);
    return 0;
  }
  const bool fused = argc > 2 && !strcmp(argv[2], "fma");
  if (!strcmp(argv[1], "logf")) {
    long bad = 0;
    for (uint32_t k = 0; k < (1u << 24); k++) {
      const float u1 = 1.0f - (float)k * (1.0f / 16777216.0f);
      const float mine = fused ? fks_libm::logf_glibc<true>(u1) : fks_libm::logf_glibc<false>(u1);
      if (fks_libm::fbits(mine) != fks_libm::fbits(logf(u1))) bad++;
    }
    printf("bad %ld\n", bad);
    return 0;
  }
  if (!strcmp(argv[1], "sincosf")) {
    long bad = 0;
    for (uint32_t k = 0; k < (1u << 24); k++) {
      const float th = (float)(2.0f * 3.14159265358979323846 * (double)((float)k * (1.0f / 16777216.0f)));
      float s, c;
      if (fused) fks_libm::sincosf_glibc<true>(th, s, c);
      else fks_libm::sincosf_glibc<false>(th, s, c);
      if (fks_libm::fbits(s) != fks_libm::fbits(sinf(th))) bad++;
      if (fks_libm::fbits(c) != fks_libm::fbits(cosf(th))) bad++;
    }
    printf("bad %ld\n", bad);
    return 0;
  }
  if (!strcmp(argv[1], "theta")) {
    long bad = 0;
    for (uint32_t k = 0; k < (1u << 24); k++) {
      const float u2 = (float)k * (1.0f / 16777216.0f);
      const float ref = (float)(2.0f * 3.14159265358979323846 * (double)u2);
      if (fks_libm::fbits(fks_libm::theta_of(k)) != fks_libm::fbits(ref)) bad++;
    }
    printf("bad %ld\n", bad);
    return 0;
  }
  if (!strcmp(argv[1], "consts")) {
    for (int i = 0; i < 16; i++) printf("%a\n%a\n", fks_libm::kLogfTab[i][0], fks_libm::kLogfTab[i][1]);
    const double rest[] = {fks_libm::kLogfLn2, fks_libm::kLogfA0, fks_libm::kLogfA1, fks_libm::kLogfA2,
                           fks_libm::kScHpiInv, fks_libm::kScHpi, fks_libm::kScC0, fks_libm::kScC1,
                           fks_libm::kScS1, fks_libm::kScC2, fks_libm::kScS2, fks_libm::kScC3,
                           fks_libm::kScS3, fks_libm::kScC4};
    for (double v : rest) printf("%a\n", v);
    return 0;
  }
  if (!strcmp(argv[1], "z")) {
    unsigned long long a, b;
    int which;
    while (scanf("%llx %llx %d", &a, &b, &which) == 3) {
      const double u1 = u53(a), u2 = u53(b);
      const double th = 2.0 * 3.14159265358979323846 * u1;
      const double r1 = sqrt(-2.0 * fks_libm::log1p(-u2));
      const double v1 = r1 * fks_libm::sin_or_cos(th, which) * 1.0 + 0.0;
      const double r2 = sqrt(-2.0 * log1p(-u2));
      const double v2 = r2 * (which ? sin(th) : cos(th)) * 1.0 + 0.0;
      const float f1 = (float)v1, f2 = (float)v2;
      uint32_t b1, b2;
      memcpy(&b1, &f1, 4);
      memcpy(&b2, &f2, 4);
      printf("%08x %08x\n", b1, b2);
    }
    return 0;
  }
  return 2;
}
