// fks_tables.cpp -- Box-Muller tables for the reduced-precision z streams.
//
// For bf16 (f16) parameters torch draws an 8-bit (11-bit) uniform per element
// (uniform_real_distribution<scalar_t>, TransformationHelper.h:84-90, digits = 8 / 11)
// and runs normal_fill_16<scalar_t> (DistributionTemplates.h:139-149) in c10 reduced
// arithmetic: every op is a float op rounded to the 16-bit type.  Hence
//   radius = R[a]   (a = u32 & 0xFF, u1 = 1 - a/256)
//   cos/sin(theta) = C[b], S[b]   (b = the uniform of element j+8)
//   z_j = round16(R[a] * C[b]) + 0,  z_{j+8} = round16(R[a] * S[b]) + 0
// with R, C, S computed here once, with the same libm (glibc logf/cosf/sinf/sqrtf)
// torch's CPU kernel calls.  The device kernel only multiplies and rounds.
#include <cmath>
#include <cstring>
#include <mutex>

#include "fks_internal.h"

namespace fks {
namespace {

inline uint32_t fbits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
inline float bitsf(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

// c10::detail::round_to_nearest_even (torch/headeronly/util/BFloat16.h:100-114)
inline float bf(float f) {
  if (f != f) return f;
  uint32_t u = fbits(f);
  u = (u + (((u >> 16) & 1u) + 0x7FFFu)) & 0xFFFF0000u;
  return bitsf(u);
}

// float -> binary16 -> float, round to nearest even (c10::Half)
inline float hf(float f) {
  if (f != f) return f;
  uint32_t x = fbits(f);
  uint32_t sign = x & 0x80000000u, ax = x & 0x7fffffffu;
  if (ax >= 0x477ff000u) return bitsf(sign | 0x7f800000u);
  if (ax < 0x38800000u) {  // half subnormal: quantum 2^-24
    float q = std::nearbyint(bitsf(ax) * 16777216.0f) / 16777216.0f;
    return bitsf(sign | fbits(q));
  }
  uint32_t mant = ax & 0x7fffffu, rem = mant & 0x1fffu;
  uint32_t keep = ax & ~0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (keep & 0x2000u))) keep += 0x2000u;
  return bitsf(sign | keep);
}

constexpr double kPi = 3.14159265358979323846;  // c10::pi<double>

Tables* build() {
  auto* t = new Tables();
  for (int a = 0; a < 256; a++) {
    const float u = bf((float)a * (1.0f / 256.0f));
    const float u1 = bf(1.0f - u);                       // 1 - data[j]
    t->r_bf16[a] = bf(std::sqrt(bf(-2.0f * bf(std::log(u1)))));
    const float theta = bf((float)(2.0f * kPi * (double)u));  // double -> float -> bf16
    t->c_bf16[a] = bf(std::cos(theta));
    t->s_bf16[a] = bf(std::sin(theta));
  }
  for (int a = 0; a < 2048; a++) {
    const float u = hf((float)a * (1.0f / 2048.0f));
    const float u1 = hf(1.0f - u);
    t->r_f16[a] = hf(std::sqrt(hf(-2.0f * hf(std::log(u1)))));
    const float theta = hf((float)(2.0f * kPi * (double)u));
    t->c_f16[a] = hf(std::cos(theta));
    t->s_f16[a] = hf(std::sin(theta));
  }
  return t;
}

}  // namespace

const Tables& tables() {
  static std::once_flag once;
  static Tables* t = nullptr;
  std::call_once(once, [] { t = build(); });
  return *t;
}

}  // namespace fks
