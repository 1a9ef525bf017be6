// fks_bitslice.h -- bit-sliced MT19937 primitives of the bf16 slice kernel
// (fks_apply_bs_kernel, fks_device.hip).  Host + device: the host build is only used by
// tools/bs_selftest.cpp to check every primitive against the scalar generator.
//
// A SLICE is 32 seeds.  Their generator states are held transposed: ROW i (i < 624)
// is the 624-word state position i of all 32 seeds as 32 bit PLANES, plane b bit k =
// bit b of seed k's word i.  In that form the MT19937 twist (MT19937RNGEngine.h:164-175)
// is one 2- or 3-input xor per plane -- shifts and masks become plane renaming --, and
// the tempering (:141-145) of the 8 bits the bf16 uniform uses (random() & 0xFF,
// uniform_real_distribution<BFloat16>, 8 mantissa digits) is a fixed GF(2) map: each
// of the 8 output planes is the xor of 3 to 9 input planes.  A 3-stage bit-matrix
// transpose turns the 8 output planes of a row back into one byte per seed.
#pragma once
#include <stdint.h>

namespace fks {
namespace bs {

constexpr int kSeeds = 32;                 // seeds per slice (bits of a plane word)
constexpr int kRows = 624;                 // MT19937 state words
constexpr uint32_t kMatrixA = 0x9908b0dfu;

#if defined(__HIPCC__)
#define FKS_BS_FN __host__ __device__ __forceinline__
#else
#define FKS_BS_FN inline
#endif

// v_bitop3_b32 (LOP3 truth-table convention: IMM = f(0xF0, 0xCC, 0xAA))
template <unsigned IMM>
FKS_BS_FN uint32_t bitop3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, IMM);
#else
  uint32_t r = 0;
  for (unsigned m = 0; m < 8; m++)
    if ((IMM >> m) & 1u) r |= ((m & 4) ? a : ~a) & ((m & 2) ? b : ~b) & ((m & 1) ? c : ~c);
  return r;
#endif
}
FKS_BS_FN uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return bitop3<0x96>(a, b, c); }
// bitwise select: m ? a : b
FKS_BS_FN uint32_t mux(uint32_t m, uint32_t a, uint32_t b) { return bitop3<0xCA>(m, a, b); }

// two 32-bit words shifted as ONE 64-bit value (v_lshrrev_b64 / v_lshlrev_b64, full
// rate on gfx950): lo = x0, hi = x1
struct W2 {
  uint32_t lo, hi;
};
template <int S>
FKS_BS_FN W2 shr2(uint32_t lo, uint32_t hi) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef uint32_t v2 __attribute__((ext_vector_type(2)));
  v2 x = {lo, hi}, r;
  asm("v_lshrrev_b64 %0, %2, %1" : "=v"(r) : "v"(x), "i"(S));
  return W2{r.x, r.y};
#else
  const uint64_t v = ((uint64_t)hi << 32 | lo) >> S;
  return W2{(uint32_t)v, (uint32_t)(v >> 32)};
#endif
}
template <int S>
FKS_BS_FN W2 shl2(uint32_t lo, uint32_t hi) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef uint32_t v2 __attribute__((ext_vector_type(2)));
  v2 x = {lo, hi}, r;
  asm("v_lshlrev_b64 %0, %2, %1" : "=v"(r) : "v"(x), "i"(S));
  return W2{r.x, r.y};
#else
  const uint64_t v = ((uint64_t)hi << 32 | lo) << S;
  return W2{(uint32_t)v, (uint32_t)(v >> 32)};
#endif
}

// One twisted row: N = the new word i of every seed, from V = old row i+1 (the NEW
// row 0 for i = 623), M = old row i+397 (i < 227) or the new row i-227, and U31 =
// plane 31 of the old row i.  y = (U & UPPER) | (V & LOWER); N = M ^ (y >> 1) ^
// (V & 1 ? A : 0):  plane b of y >> 1 is V[b+1] (b < 30), U[31] (b = 30), 0 (b = 31).
FKS_BS_FN void twist_row(const uint32_t (&V)[32], const uint32_t (&M)[32], uint32_t U31, uint32_t (&N)[32]) {
#pragma unroll
  for (int b = 0; b < 30; b++) N[b] = ((kMatrixA >> b) & 1u) ? xor3(M[b], V[b + 1], V[0]) : (M[b] ^ V[b + 1]);
  N[30] = ((kMatrixA >> 30) & 1u) ? xor3(M[30], U31, V[0]) : (M[30] ^ U31);
  N[31] = ((kMatrixA >> 31) & 1u) ? (M[31] ^ V[0]) : M[31];
}
// the same, the new row written over M (plane b of the new row needs only M[b]): no
// third 32-register row array in the twist wave
FKS_BS_FN void twist_row_inplace(const uint32_t (&V)[32], uint32_t (&M)[32], uint32_t U31) {
#pragma unroll
  for (int b = 0; b < 30; b++) M[b] = ((kMatrixA >> b) & 1u) ? xor3(M[b], V[b + 1], V[0]) : (M[b] ^ V[b + 1]);
  M[30] = ((kMatrixA >> 30) & 1u) ? xor3(M[30], U31, V[0]) : (M[30] ^ U31);
  M[31] = ((kMatrixA >> 31) & 1u) ? (M[31] ^ V[0]) : M[31];
}

// Planes 0..7 of the tempered row (tempering restricted to its low byte, a GF(2) map:
// out bit b = xor of the input bits listed; generated from the scalar tempering and
// checked by tools/bs_selftest.cpp).
FKS_BS_FN void temper_low8(const uint32_t (&x)[32], uint32_t (&o)[8]) {
  const uint32_t s03 = x[0] ^ x[3];
  const uint32_t t0 = xor3(s03, x[14], x[18]);        // 0 3 14 18
  o[0] = xor3(t0, x[22], x[29]);                      // 0 3 14 18 22 29
  o[1] = xor3(x[1], x[19], x[23]) ^ x[30];            // 1 19 23 30
  o[2] = xor3(x[2], x[13], x[20]) ^ x[31];            // 2 13 20 31
  const uint32_t s2125 = x[21] ^ x[25];
  o[3] = x[3] ^ s2125;                                // 3 21 25
  o[4] = xor3(xor3(x[0], x[4], x[7]), xor3(x[11], x[15], x[18]), x[22]);  // 0 4 7 11 15 18 22
  o[5] = xor3(xor3(x[5], x[8], x[16]), x[19], x[23]);                    // 5 8 16 19 23
  o[6] = xor3(xor3(x[2], x[6], x[9]), xor3(x[13], x[20], x[24]), x[28]); // 2 6 9 13 20 24 28
  o[7] = xor3(xor3(t0, x[7], x[10]), x[11], s2125);   // 0 3 7 10 11 14 18 21 25
}

// 8 planes -> 8 words of 4 bytes: byte c of W[j] = bits (8c + j) of planes 0..7, i.e.
// the tempered low byte of seed 8c + j.  Three delta-swap stages of the four 8x8 bit
// blocks (one per byte column); each stage exchanges bits between planes r and r + d as
//   x' = (m << d) ? (y << d) : x,   y' = m ? (x >> d) : y,
// with the shifts done on two words at a time (their spilled bits fall outside the
// stage's mask).  In place: P becomes W.
template <int D>
FKS_BS_FN void swap_stage(uint32_t& x0, uint32_t& x1, uint32_t& y0, uint32_t& y1, uint32_t m) {
  const W2 xs = shr2<D>(x0, x1);
  const W2 ys = shl2<D>(y0, y1);
  const uint32_t mh = m << D;
  const uint32_t nx0 = mux(mh, ys.lo, x0), nx1 = mux(mh, ys.hi, x1);
  y0 = mux(m, xs.lo, y0);
  y1 = mux(m, xs.hi, y1);
  x0 = nx0;
  x1 = nx1;
}
FKS_BS_FN void transpose8(uint32_t (&P)[8]) {
  swap_stage<4>(P[0], P[1], P[4], P[5], 0x0F0F0F0Fu);
  swap_stage<4>(P[2], P[3], P[6], P[7], 0x0F0F0F0Fu);
  swap_stage<2>(P[0], P[1], P[2], P[3], 0x33333333u);
  swap_stage<2>(P[4], P[5], P[6], P[7], 0x33333333u);
  swap_stage<1>(P[0], P[2], P[1], P[3], 0x55555555u);
  swap_stage<1>(P[4], P[6], P[5], P[7], 0x55555555u);
}

// 32 words (one per seed) -> 32 planes, plane b bit k = bit b of w[k] (five stages, the
// kernel prologue only).  In place.
template <int D>
FKS_BS_FN void swap1(uint32_t& x, uint32_t& y, uint32_t m) {
  const uint32_t t = ((x >> D) ^ y) & m;
  y ^= t;
  x ^= t << D;
}
FKS_BS_FN void transpose32(uint32_t (&w)[32]) {
#pragma unroll
  for (int r = 0; r < 32; r++)
    if (!(r & 16)) swap1<16>(w[r], w[r + 16], 0x0000FFFFu);
#pragma unroll
  for (int r = 0; r < 32; r++)
    if (!(r & 8)) swap1<8>(w[r], w[r + 8], 0x00FF00FFu);
#pragma unroll
  for (int r = 0; r < 32; r++)
    if (!(r & 4)) swap1<4>(w[r], w[r + 4], 0x0F0F0F0Fu);
#pragma unroll
  for (int r = 0; r < 32; r++)
    if (!(r & 2)) swap1<2>(w[r], w[r + 2], 0x33333333u);
#pragma unroll
  for (int r = 0; r < 32; r++)
    if (!(r & 1)) swap1<1>(w[r], w[r + 1], 0x55555555u);
}

// byte c of w times 2^S: one SDWA shift (src1_sel BYTE_c) on the device
template <int C, int S>
FKS_BS_FN uint32_t byte_x(uint32_t w) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_lshlrev_b32_sdwa %0, %2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_%3"
      : "=v"(r)
      : "v"(w), "i"(S), "i"(C));
  return r;
#else
  return ((w >> (8 * C)) & 0xFFu) << S;
#endif
}

}  // namespace bs
}  // namespace fks
