// Double-precision log1p / sin / cos for the serial z path (tensors with numel < 16).
//
// The reference's CPU z stream draws those elements one at a time through
// at::normal_distribution<double> (ATen/core/DistributionsHelper.h: Box-Muller on two
// 53-bit uniforms, r = sqrt(-2 log1p(-u2)), r*cos / r*sin in double, then cast to the
// tensor dtype).  The double value is produced by the host libm the reference runs on --
// glibc 2.35 on x86_64 in this image -- and an fp32 element differs whenever the device's
// double lands on the other side of an fp32 rounding midpoint.  ocml's log1p / sin / cos
// are not glibc's, and such a midpoint case was found (tests/golden/serial_straddle.json,
// seed 48), so the serial path computes these three functions here instead:
//
//   log1p  restates glibc's sysdeps/ieee754/dbl-64/s_log1p.c (fdlibm's algorithm with the
//          polynomial split into four independent pairs): bit-identical to glibc on 5e7
//          inputs of the path's domain (-u2, u2 = m 2^-53), tests/test_libm_serial.py;
//   sin/cos  correctly rounded (double-double Cody-Waite reduction by pi/2 in three parts,
//          Taylor series to degree 31 / 30 in double-double): glibc's dbl-64 sin / cos are
//          correctly rounded on all but ~0.15% of inputs, and a double-ulp difference moves
//          the fp32 result only when the product r*sin sits within an ulp of a midpoint
//          (~2^-28 of those), i.e. below 1e-11 per draw.
//
// Every expression is evaluated in the order written: contraction into fma is off inside
// each function (clang pragma; g++ builds of the host checker pass -ffp-contract=off).
// The slow-but-exact double-double work costs a few hundred f64 operations per draw on a
// path that sees at most 15 elements per tensor.
#pragma once
#include <stdint.h>

#ifndef FKS_HD
#define FKS_HD inline
#endif

#if defined(__clang__)
#define FKS_NO_CONTRACT _Pragma("clang fp contract(off)")
#else
#define FKS_NO_CONTRACT
#endif

namespace fks_libm {

FKS_HD uint64_t bits(double x) { return __builtin_bit_cast(uint64_t, x); }
FKS_HD double from_bits(uint64_t u) { return __builtin_bit_cast(double, u); }

// glibc s_log1p.c (fdlibm): x = -u2 lies in (-1, 0], so the NaN / +inf / x >= 2^53 arms
// of the original are unreachable and kept only as far as they are cheap.  The algorithm
// and its constants are fdlibm's, whose notice follows:
//
//   ====================================================
//   Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
//
//   Developed at SunPro, a Sun Microsystems, Inc. business.
//   Permission to use, copy, modify, and distribute this
//   software is freely granted, provided that this notice
//   is preserved.
//   ====================================================
//
// (glibc's dbl-64 s_log1p.c carries the same notice; its "modified by" changes -- the
// split of the Lp polynomial evaluation -- are what the evaluation order below follows.)
FKS_HD double log1p(double x) {
  FKS_NO_CONTRACT
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01, Lp3 = 2.857142874366239149e-01,
               Lp4 = 2.222219843214978396e-01, Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
               Lp7 = 1.479819860511658591e-01;
  double f = 0.0, c = 0.0;
  const int32_t hx = (int32_t)(bits(x) >> 32), ax = hx & 0x7fffffff;
  int32_t k = 1, hu = 0;
  if (hx < 0x3FDA827A) {  // x < 0.41422
    if (ax >= 0x3ff00000) return x == -1.0 ? -__builtin_inf() : __builtin_nan("");
    if (ax < 0x3e200000) {  // |x| < 2^-29
      if (ax < 0x3c900000) return x;
      return x - x * x * 0.5;
    }
    if (hx > 0 || hx <= (int32_t)0xbfd2bec3) {  // -0.2929 < x < 0.41422
      k = 0;
      f = x;
      hu = 1;
    }
  }
  if (k != 0) {
    double u = 1.0 + x;
    hu = (int32_t)(bits(u) >> 32);
    k = (hu >> 20) - 1023;
    c = k > 0 ? 1.0 - (u - x) : x - (u - 1.0);  // correction term
    c /= u;
    hu &= 0x000fffff;
    const uint64_t lo = bits(u) & 0xffffffffull;
    if (hu < 0x6a09e) {
      u = from_bits(((uint64_t)(uint32_t)(hu | 0x3ff00000) << 32) | lo);  // normalize u
    } else {
      k += 1;
      u = from_bits(((uint64_t)(uint32_t)(hu | 0x3fe00000) << 32) | lo);  // normalize u/2
      hu = (0x00100000 - hu) >> 2;
    }
    f = u - 1.0;
  }
  const double hfsq = 0.5 * f * f;
  if (hu == 0) {  // |f| < 2^-20
    if (f == 0.0) {
      if (k == 0) return 0.0;
      c += k * ln2_lo;
      return k * ln2_hi + c;
    }
    const double R = hfsq * (1.0 - 0.66666666666666666 * f);
    if (k == 0) return f - R;
    return k * ln2_hi - ((R - (k * ln2_lo + c)) - f);
  }
  const double s = f / (2.0 + f);
  const double z = s * s;
  const double R1 = z * Lp1, z2 = z * z, R2 = Lp2 + z * Lp3, z4 = z2 * z2, R3 = Lp4 + z * Lp5, z6 = z4 * z2,
               R4 = Lp6 + z * Lp7;
  const double R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
  if (k == 0) return f - (hfsq - s * (hfsq + R));
  return k * ln2_hi - ((hfsq - (s * (hfsq + R) + (k * ln2_lo + c))) - f);
}

struct DD {
  double hi, lo;
};

FKS_HD DD two_sum(double a, double b) {
  FKS_NO_CONTRACT
  const double s = a + b, bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
FKS_HD DD fast_two_sum(double a, double b) {  // |a| >= |b|
  FKS_NO_CONTRACT
  const double s = a + b;
  return {s, b - (s - a)};
}
FKS_HD DD dd_add(DD x, DD y) {
  FKS_NO_CONTRACT
  const DD s = two_sum(x.hi, y.hi), t = two_sum(x.lo, y.lo);
  DD r = fast_two_sum(s.hi, s.lo + t.hi);
  return fast_two_sum(r.hi, r.lo + t.lo);
}
FKS_HD DD dd_mul(DD x, DD y) {
  FKS_NO_CONTRACT
  const double p = x.hi * y.hi;
  const double e = __builtin_fma(x.hi, y.hi, -p);
  return fast_two_sum(p, e + (x.hi * y.lo + x.lo * y.hi));
}

// (-1)^n / (2n+1)!  and  (-1)^n / (2n)!  as double-double, n = 0..15
constexpr double kSinC[16][2] = {
    {0x1.0000000000000p+0, 0x0.0p+0},           {-0x1.5555555555555p-3, -0x1.5555555555555p-57},
    {0x1.1111111111111p-7, 0x1.1111111111111p-63}, {-0x1.a01a01a01a01ap-13, -0x1.a01a01a01a01ap-73},
    {0x1.71de3a556c734p-19, -0x1.c154f8ddc6c00p-73}, {-0x1.ae64567f544e4p-26, 0x1.c062e06d1f209p-80},
    {0x1.6124613a86d09p-33, 0x1.f28e0cc748ebep-87}, {-0x1.ae7f3e733b81fp-41, -0x1.1d8656b0ee8cbp-97},
    {0x1.952c77030ad4ap-49, 0x1.ac981465ddc6cp-103}, {-0x1.2f49b46814157p-57, -0x1.2650f61dbdcb4p-112},
    {0x1.71b8ef6dcf572p-66, -0x1.d043ae40c4647p-120}, {-0x1.761b41316381ap-75, 0x1.3423c7d91404fp-130},
    {0x1.3f3ccdd165fa9p-84, -0x1.58ddadf344487p-139}, {-0x1.d1ab1c2dccea3p-94, -0x1.054d0c78aea14p-149},
    {0x1.259f98b4358adp-103, 0x1.eaf8c39dd9bc5p-157}, {-0x1.434d2e783f5bcp-113, -0x1.0b87b91be9affp-167}};
constexpr double kCosC[16][2] = {
    {0x1.0000000000000p+0, 0x0.0p+0},           {-0x1.0000000000000p-1, 0x0.0p+0},
    {0x1.5555555555555p-5, 0x1.5555555555555p-59}, {-0x1.6c16c16c16c17p-10, 0x1.f49f49f49f49fp-65},
    {0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-76}, {-0x1.27e4fb7789f5cp-22, -0x1.cbbc05b4fa99ap-76},
    {0x1.1eed8eff8d898p-29, -0x1.2aec959e14c06p-83}, {-0x1.93974a8c07c9dp-37, -0x1.05d6f8a2efd1fp-92},
    {0x1.ae7f3e733b81fp-45, 0x1.1d8656b0ee8cbp-101}, {-0x1.6827863b97d97p-53, -0x1.eec01221a8b0bp-107},
    {0x1.e542ba4020225p-62, 0x1.ea72b4afe3c2fp-120}, {-0x1.0ce396db7f853p-70, 0x1.aebcdbd20331cp-124},
    {0x1.f2cf01972f578p-80, -0x1.9ada5fcc1ab14p-135}, {-0x1.88e85fc6a4e5ap-89, 0x1.71c37ebd16540p-143},
    {0x1.0a18a2635085dp-98, 0x1.b9e2e28e1aa54p-153}, {-0x1.3932c5047d60ep-108, -0x1.832b7b530a627p-162}};

// sin(theta) or cos(theta), correctly rounded, for 0 <= theta < 8 (theta = 2 pi u1 here).
FKS_HD double sin_or_cos(double theta, bool want_sin) {
  FKS_NO_CONTRACT
  const double P1 = 0x1.921fb54442d18p+0, P2 = 0x1.1a62633145c07p-54, P3 = -0x1.f1976b7ed8fbcp-110;
  const int k = (int)__builtin_rint(theta * 0x1.45f306dc9c883p-1);  // nearest multiple of pi/2
  const double kd = (double)k;
  // y = theta - k pi/2: theta - k*P1 is exact (Sterbenz, k <= 5), then the two tails
  const double t1 = kd * P1;
  const double e1 = __builtin_fma(kd, P1, -t1);
  DD y = {theta - t1, 0.0};
  y = dd_add(y, {-e1, 0.0});
  const double t2 = kd * P2;
  y = dd_add(y, {-t2, -__builtin_fma(kd, P2, -t2)});
  y = dd_add(y, {-(kd * P3), 0.0});
  const DD y2 = dd_mul(y, y);
  // quadrant q: sin = [s, c, -s, -c][q], cos = [c, -s, -c, s][q]
  const int q = (k + (want_sin ? 0 : 1)) & 3;
  const bool use_sin = (q & 1) == 0;
  const double(*C)[2] = use_sin ? kSinC : kCosC;
  DD p = {C[15][0], C[15][1]};
  for (int n = 14; n >= 0; n--) p = dd_add(dd_mul(p, y2), {C[n][0], C[n][1]});
  if (use_sin) p = dd_mul(p, y);
  const double r = p.hi + p.lo;
  return (q & 2) ? -r : r;
}

// ---------------------------------------------------------------- fp32, libm flavour
// Under ATen's DEFAULT CPU capability (ATEN_CPU_CAPABILITY=default, or a host without
// AVX2) torch fills fp32 tensors of >= 16 elements with normal_fill_16<float>
// (DistributionTemplates.h:139-149) instead of normal_fill_16_AVX2: per pair
//   radius = sqrtf(-2 * logf(1 - u1)),  theta = (float)(2 pi_double * u2),
//   z_j = radius * cosf(theta) * std + mean,  z_{j+8} = radius * sinf(theta) * std + mean
// with glibc's single-precision logf / sinf / cosf (glibc >= 2.28: sysdeps/ieee754/flt-32
// e_logf.c, s_sinf.c, s_cosf.c, sincosf.h, from ARM's optimized-routines, evaluated in
// double).  Restated below for the inputs this path gives them -- logf on u1 = 1 - k 2^-24,
// sinf / cosf on theta_k, k < 2^24 -- where the special-value arms are unreachable.  The
// constants are glibc's __logf_data and __sincosf_table (tools/libm_float_consts.py reads
// them from this image's libm.so.6).  tests/test_libm_float.py compares every one of the
// 2^24 inputs of each function with the host's glibc, with its FMA dispatch on and off
// (the two builds agree on these inputs), in both evaluation forms below: FMA = false is
// glibc's source order with every product rounded (its non-FMA build); FMA = true fuses each
// "a * b + c" of the source into one fma, as its FMA build may, and is what the device runs
// (f64 arithmetic issues at half the f32 rate on gfx950: 7 instead of 11 f64 operations per
// logf, 14 instead of 21 per sine-cosine pair).  Both forms give glibc's value on every
// input of the domain -- the final rounding to float absorbs their difference there.
constexpr double kLogfTab[16][2] = {  // {invc, logc}: __logf_data.tab
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010b0p+0, -0x1.01eae7f513a67p-2}, {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8ea0p+0, -0x1.1aa2bc79c8100p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aa0p-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d224770p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2}};
constexpr double kLogfA0 = -0x1.00ea348b88334p-2, kLogfA1 = 0x1.5575b0be00b6ap-2, kLogfA2 = -0x1.ffffef20a4123p-2,
                 kLogfLn2 = 0x1.62e42fefa39efp-1;
// __sincosf_table[0]: 2/pi * 2^24, pi/2, the cosine and sine polynomials ([1] negates the
// cosine's coefficients, which negates its value exactly)
constexpr double kScHpiInv = 0x1.45f306dc9c883p+23, kScHpi = 0x1.921fb54442d18p+0, kScC0 = 1.0,
                 kScC1 = -0x1.ffffffd0c621cp-2, kScC2 = 0x1.55553e1068f19p-5, kScC3 = -0x1.6c087e89a359dp-10,
                 kScC4 = 0x1.99343027bf8c3p-16, kScS1 = -0x1.555545995a603p-3, kScS2 = 0x1.1107605230bc4p-7,
                 kScS3 = -0x1.994eb3774cf24p-13;

FKS_HD uint32_t fbits(float x) { return __builtin_bit_cast(uint32_t, x); }
FKS_HD float from_fbits(uint32_t u) { return __builtin_bit_cast(float, u); }

// e_logf.c's subinterval of a normal x > 0: x = 2^k z, z in [0x3f330000, 2 * that) as bits
FKS_HD int logf_index(float x) { return (int)(((fbits(x) - 0x3f330000u) >> 19) & 15u); }

// normal_fill_16<float>'s angle for the 24-bit uniform b: theta = (float)(2.0f *
// c10::pi<double> * u2) with u2 = b 2^-24, i.e. RN_float(RN_double(2 pi_double * u2)).  The
// double product equals RN_double((2 pi_double 2^-24) * b) -- a power-of-two scaling, exact
// in double -- so it is one conversion of b and one multiply (tests/libm_check.cpp "theta")
FKS_HD float theta_of(uint32_t b) { return (float)((double)b * 0x1.921fb54442d18p-22); }

// a * b + c, fused (FMA) or with the product rounded
template <bool FMA>
FKS_HD double mad(double a, double b, double c) {
  FKS_NO_CONTRACT
  if constexpr (FMA) return __builtin_fma(a, b, c);
  return a * b + c;
}

// e_logf.c for a normal x > 0 given its table entry (x = 1 takes glibc's early "return 0"
// arm there and +0 here as well: r = 0, y0 = 0)
template <bool FMA>
FKS_HD float logf_core(float x, double invc, double logc) {
  FKS_NO_CONTRACT
  const uint32_t ix = fbits(x), tmp = ix - 0x3f330000u;
  const int k = (int32_t)tmp >> 23;
  const double z = (double)from_fbits(ix - (tmp & 0xff800000u));
  const double r = mad<FMA>(z, invc, -1.0);  // log(x) = log1p(z/c - 1) + log(c) + k ln2
  const double y0 = mad<FMA>((double)k, kLogfLn2, logc);
  const double r2 = r * r;
  double y = mad<FMA>(kLogfA1, r, kLogfA2);
  y = mad<FMA>(kLogfA0, r2, y);
  y = mad<FMA>(y, r2, y0 + r);
  return (float)y;
}

template <bool FMA>
FKS_HD float logf_glibc(float x) {
  const int i = logf_index(x);
  return logf_core<FMA>(x, kLogfTab[i][0], kLogfTab[i][1]);
}

// sinf(y) and cosf(y) for 0 <= y < 120: s_sinf.c / s_cosf.c's first two arms.  Their
// reduce_fast gives n = 0 and x unchanged for y < pi/4, which is the small-argument arm, so
// one evaluation serves both; only |y| < 2^-12 is special (sin y = y, cos y = 1), and for
// y >= 0 not even that (below).
template <bool FMA>
FKS_HD void sincosf_glibc(float y, float& s, float& c) {
  FKS_NO_CONTRACT
  const double x = (double)y;
  const double r = x * kScHpiInv;                 // reduce_fast without TOINT_INTRINSICS
  const int n = ((int32_t)r + 0x800000) >> 24;
  const double xr = mad<FMA>(-(double)n, kScHpi, x);
  // x * sign[n & 3], sign = {1, -1, -1, 1}: the sign bit flipped for n & 3 in {1, 2}
  const double xs = from_bits(bits(xr) ^ ((uint64_t)((uint32_t)(n + 1) & 2u) << 62));
  const double x2 = xs * xs;
  const double x3 = xs * x2;                      // sinf_poly, even quadrant
  const double s1 = mad<FMA>(x2, kScS3, kScS2);
  const double x7 = x3 * x2;
  const double sp = mad<FMA>(x3, kScS1, xs);
  const float ps = (float)mad<FMA>(x7, s1, sp);
  const double x4 = x2 * x2;                      // sinf_poly, odd quadrant (table n & 2)
  const double c2 = mad<FMA>(x2, kScC4, kScC3);
  const double c1 = mad<FMA>(x2, kScC1, kScC0);
  const double x6 = x4 * x2;
  const double cp = mad<FMA>(x4, kScC2, c1);
  const float pc0 = (float)mad<FMA>(x6, c2, cp);
  const float pc = from_fbits(fbits(pc0) ^ (((uint32_t)n & 2u) << 30));  // table n & 2: negated
  const bool odd = (n & 1) != 0;  // sinf takes the cosine polynomial in odd quadrants, cosf in even
  s = odd ? pc : ps;
  c = odd ? ps : pc;
  // |y| < 2^-12 (abstop12(y) < abstop12(0x1p-12f)): glibc returns y and 1.0f.  For y >= 0
  // that is what the polynomials round to there as well -- sin: y (1 - y^2/6 ...) is within
  // 2^-26.6 y of y, below half an ulp; cos: 1 - y^2/2 with y^2/2 < 2^-25, below half the
  // spacing under 1 -- so the fused form drops the arm (the exhaustive checks cover both)
  if constexpr (!FMA) {
    if ((fbits(y) >> 20) < 0x398u) {
      s = y;
      c = 1.0f;
    }
  }
}

}  // namespace fks_libm
