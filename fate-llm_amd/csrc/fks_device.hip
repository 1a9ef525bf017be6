// fks_device.hip -- gfx950 kernels of the FedKSeed codec.
//
// Work decomposition (DESIGN.md "Kernels"):
//   * the parameter stream (all tensors in param-group order, the order
//     zo_utils.directional_derivative_step draws z in, zo_utils.py:43-47) is cut into
//     `nchunks` runs of whole 624-word MT19937 blocks, one workgroup each;
//   * fks_jump_kernel gives every (seed, chunk) its generator window at the chunk
//     start (GF(2) jump-ahead, see fks_gf2.cpp);
//   * fks_apply_kernel holds up to kMaxSeedsPerPass seed windows in LDS, and for each
//     MT block twists them all (in place, 3 dependency phases), then lets thread q
//     own Box-Muller pair q of the block: it loads its two parameters once, runs
//     every seed in order (temper -> uniform -> z -> update, all in registers), and
//     stores them once.  Seeds run sequentially per element, exactly as the
//     reference's per-seed loop rounds them (fedkseed.py:136-141).
//
// Numerics are restated op for op from torch's CPU kernels (file:line in the
// comments); -ffp-contract=off is required, every fused multiply-add is explicit.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <atomic>
#include <type_traits>
#include <mutex>

#include "fks_internal.h"
#include "fks_bitslice.h"
#define FKS_HD __device__ __forceinline__
#include "fks_libm.h"

// Design choices measured on MI355X in rounds 1-2 are fixed in the code; the A/B knobs
// and the wrong-result timing diagnostics of those rounds were removed (their logs are
// under profiles/, their code in the git history).
constexpr int kDbMinWaves = 4;   // launch-bounds waves per SIMD of the double-buffered small-K kernel (6 WGs/CU measured 19 % slower than 5)
constexpr int kZrUnroll = 2;     // z-index replay: tiles per loop iteration (in flight per wave)
constexpr int kSm2MinWaves = 8;  // launch-bounds waves per SIMD of fks_small2_kernel (8 workgroups of 4 waves per CU: <= 64 VGPRs)
constexpr int kBsFence = 8;      // slice kernel: compiler fence after every 8 seeds' table lookups
#ifndef FKS_BS_LAG               // slice kernel, two-slice passes: half 0 twists task n only once half 1
#define FKS_BS_LAG 36            // has applied task n - FKS_BS_LAG (0: unbounded; must exceed 12)
#endif
#ifndef FKS_F32_SEED_PAIRS       // fp32 19-seed kernel: seed PAIRS sharing packed float ops, this many
#define FKS_F32_SEED_PAIRS 0     // interleaved per step (0: one seed per z computation).  Measured
#endif                           // 7-9 % SLOWER for 1-3 (profiles/r05c_f32_seedpair_ab.log)
#ifndef FKS_LOG_INTMASK          // fp32 Cephes log: the x < sqrt(1/2) select as integer arithmetic
#define FKS_LOG_INTMASK 1
#endif
#ifndef FKS_F32_TRIM             // fp32 Cephes z: the uniforms' scalings folded, the sincos signs
#define FKS_F32_TRIM 1           // as one v_bitop3 each (same values; 0 = the round-5 form, for A/B)
#endif

namespace fks {
namespace {

// ------------------------------------------------------------------ MT19937 pieces
__device__ __forceinline__ uint32_t mt_twist(uint32_t u, uint32_t v) {
  return (((u & 0x80000000u) | (v & 0x7fffffffu)) >> 1) ^ ((v & 1u) ? kMatrixA : 0u);
}

// v_bitop3_b32 truth tables (LOP3 convention: f(0xF0, 0xCC, 0xAA))
constexpr unsigned kXorAnd = 0x78;  // a ^ (b & c)
constexpr unsigned kXorMask = 0x28; // (a ^ b) & c
constexpr unsigned kXorNotAnd = 0xD2;  // a ^ (~b & c)

// tempering, MT19937RNGEngine.h:141-145; each "y ^= (y << s) & M" is one shift + one bitop3
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y = __builtin_amdgcn_bitop3_b32(y, y << 7, 0x9d2c5680u, kXorAnd);
  y = __builtin_amdgcn_bitop3_b32(y, y << 15, 0xefc60000u, kXorAnd);
  y ^= (y >> 18);
  return y;
}


// ------------------------------------------------------------------ rounding
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
// RNE to bf16, result kept as the f32 with the same value: ONE v_cvt_pk_bf16_f32 with
// a zero low half (hi = bf16(x), lo = bf16(0) = 0x0000).  NaN stays NaN.
__device__ __forceinline__ float rbf_cvt(float x) {
  const f32x2_t v = {0.0f, x};
  return __builtin_bit_cast(float, __builtin_convertvector(v, bf16x2_t));
}
__device__ __forceinline__ float rbf(float x) { return rbf_cvt(x); }
__device__ __forceinline__ float rhf(float x) {  // RNE to f16 and back
  // The empty asm pins x as an f32 VALUE: without it the backend folds the producing
  // f32 multiply into v_fma_mixlo_f16 (one rounding of the exact product straight to
  // f16), while c10::Half rounds the f32 product first (double rounding).
  asm volatile("" : "+v"(x));
  return static_cast<float>(static_cast<_Float16>(x));
}

// value of the adjacent lane (lane ^ 1): DPP quad_perm [1,0,3,2]
__device__ __forceinline__ uint32_t swap_adjacent(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}

// ------------------------------------------------------------------ fp32 Box-Muller
// normal_fill_16_AVX2 (DistributionTemplates.h:88-106) with log256_ps / sincos256_ps
// (avx_mathfun.h:90-160, 426-520) restated lane by lane; the fmaf()s are the
// contractions GCC applies in libtorch's AVX2/AVX512 build (pinned bit-exact by
// oracle/fks_oracle.c against the reference's golden streams).
__device__ __forceinline__ float cephes_logf(float x) {  // x in [2^-24, 1]
#if FKS_LOG_INTMASK
  // the "x < sqrt(1/2)" select as integer arithmetic: x is a normal float in [0.5, 1)
  // (ordered like its bits), the mask the sign of bits(x) - bits(0.70710678f); "mask ? x :
  // 0" is bits(x) & mask and e = float(imm0 - 126 + mask) the exact integer
  // (imm0 - 0x7f) + 1 - (mask ? 1 : 0): no compare, no select, no hazard wait
  const uint32_t xb0 = __float_as_uint(x);
  const uint32_t xb = (xb0 & ~0x7f800000u) | 0x3f000000u;
  const int32_t m = (int32_t)(xb - 0x3F3504F3u) >> 31;
  const float e = (float)((int32_t)(xb0 >> 23) - 126 + m);
  const float tmp = __uint_as_float(xb & (uint32_t)m);
  x = __uint_as_float(xb) - 1.0f;
#else
  int32_t imm0 = (int32_t)(__float_as_uint(x) >> 23);
  x = __uint_as_float((__float_as_uint(x) & ~0x7f800000u) | 0x3f000000u);
  imm0 -= 0x7f;
  float e = (float)imm0;
  e = e + 1.0f;
  const bool mask = x < 0.707106781186547524f;
  const float tmp = mask ? x : 0.0f;
  x = x - 1.0f;
  e = e - (mask ? 1.0f : 0.0f);
#endif
  x = x + tmp;
  const float z = x * x;
  float y = 7.0376836292E-2f;
  y = __fmaf_rn(y, x, -1.1514610310E-1f);
  y = __fmaf_rn(y, x, 1.1676998740E-1f);
  y = __fmaf_rn(y, x, -1.2420140846E-1f);
  y = __fmaf_rn(y, x, +1.4249322787E-1f);
  y = __fmaf_rn(y, x, -1.6668057665E-1f);
  y = __fmaf_rn(y, x, +2.0000714765E-1f);
  y = __fmaf_rn(y, x, -2.4999993993E-1f);
  y = __fmaf_rn(y, x, +3.3333331174E-1f);
  y = y * x;
  y = __fmaf_rn(y, z, e * -2.12194440e-4f);
  y = __fmaf_rn(-z, 0.5f, y);
  x = x + y;
  x = __fmaf_rn(e, 0.693359375f, x);
  return x;
}


// ------------------------------------------------------------------ per-dtype traits
template <int DT>
struct Traits;

typedef __attribute__((address_space(1))) float gf32;
typedef __attribute__((address_space(1))) uint16_t gu16;
typedef __attribute__((address_space(1))) _Float16 gf16;

// load_raw returns the element's bits (kept raw in the software pipeline so that the
// load's wait lands at first use, a block later); cvt turns them into the f32 value.
typedef __attribute__((address_space(1))) uint32_t gu32;

typedef __attribute__((address_space(1))) uint64_t gu64;

template <>
struct Traits<FKS_F32> {
  typedef uint64_t Pair;  // two adjacent elements
  __device__ static Pair load_pair(uint64_t a) { return *reinterpret_cast<const gu64*>(a); }
  __device__ static void store_pair(uint64_t a, Pair v) { *reinterpret_cast<gu64*>(a) = v; }
  __device__ static uint32_t lo(Pair v) { return (uint32_t)v; }
  __device__ static uint32_t hi(Pair v) { return (uint32_t)(v >> 32); }
  __device__ static Pair pack(uint32_t l, uint32_t h) { return (uint64_t)l | ((uint64_t)h << 32); }
  __device__ static uint32_t bits(float v) { return __float_as_uint(v); }
  __device__ static uint32_t load_raw(uint64_t p, int64_t i) { return reinterpret_cast<const gu32*>(p)[i]; }
  __device__ static float cvt(uint32_t r) { return __uint_as_float(r); }
  __device__ static float load(uint64_t p, int64_t i) { return reinterpret_cast<const gf32*>(p)[i]; }
  __device__ static void store(uint64_t p, int64_t i, float v) { reinterpret_cast<gf32*>(p)[i] = v; }
  __device__ static float rnd(float x) { return x; }
};

template <>
struct Traits<FKS_BF16> {
  typedef uint32_t Pair;  // two adjacent elements
  __device__ static Pair load_pair(uint64_t a) { return *reinterpret_cast<const gu32*>(a); }
  __device__ static void store_pair(uint64_t a, Pair v) { *reinterpret_cast<gu32*>(a) = v; }
  __device__ static uint32_t lo(Pair v) { return v & 0xffffu; }
  __device__ static uint32_t hi(Pair v) { return v >> 16; }
  __device__ static Pair pack(uint32_t l, uint32_t h) { return (l & 0xffffu) | (h << 16); }
  __device__ static uint32_t bits(float v) { return __float_as_uint(v) >> 16; }  // v is bf16-exact
  __device__ static uint32_t load_raw(uint64_t p, int64_t i) { return reinterpret_cast<const gu16*>(p)[i]; }
  __device__ static float cvt(uint32_t r) { return __uint_as_float(r << 16); }
  __device__ static float load(uint64_t p, int64_t i) {
    return __uint_as_float((uint32_t)reinterpret_cast<const gu16*>(p)[i] << 16);
  }
  __device__ static void store(uint64_t p, int64_t i, float v) {  // v is bf16-exact
    reinterpret_cast<gu16*>(p)[i] = (uint16_t)(__float_as_uint(v) >> 16);
  }
  __device__ static float rnd(float x) { return rbf(x); }
};

template <>
struct Traits<FKS_F16> {
  typedef uint32_t Pair;
  __device__ static Pair load_pair(uint64_t a) { return *reinterpret_cast<const gu32*>(a); }
  __device__ static void store_pair(uint64_t a, Pair v) { *reinterpret_cast<gu32*>(a) = v; }
  __device__ static uint32_t lo(Pair v) { return v & 0xffffu; }
  __device__ static uint32_t hi(Pair v) { return v >> 16; }
  __device__ static Pair pack(uint32_t l, uint32_t h) { return (l & 0xffffu) | (h << 16); }
  __device__ static uint32_t bits(float v) { return __builtin_bit_cast(uint16_t, static_cast<_Float16>(v)); }
  __device__ static uint32_t load_raw(uint64_t p, int64_t i) { return reinterpret_cast<const gu16*>(p)[i]; }
  __device__ static float cvt(uint32_t r) { return static_cast<float>(__builtin_bit_cast(_Float16, (uint16_t)r)); }
  __device__ static float load(uint64_t p, int64_t i) { return static_cast<float>(reinterpret_cast<const gf16*>(p)[i]); }
  __device__ static void store(uint64_t p, int64_t i, float v) { reinterpret_cast<gf16*>(p)[i] = static_cast<_Float16>(v); }
  __device__ static float rnd(float x) { return rhf(x); }
};

// fp32 tensors of the libm flavour (kDtF32Libm): fp32 in every respect but their z
template <>
struct Traits<kDtF32Libm> : Traits<FKS_F32> {};
constexpr bool is_f32(int dt) { return dt == FKS_F32 || dt == kDtF32Libm; }

// One parameter through one seed.  zo_utils.py:49 (has_wd) / :52 ; optimizer.py:173
// (perturb: p + ps*z, ps = f32(scaling_factor * eps)).
// Each statement is one torch op rounded to the parameter dtype (fp32 opmath).
template <int DT>
__device__ __forceinline__ float apply_one(float p, float z, float g, float lr, float wd, bool has_wd, int mode,
                                           float ps, bool upd = true) {
  using TR = Traits<DT>;
  if (mode == kModeDelta) return __fmaf_rn(g, z, p);   // seed-sharded variant: delta += c_k * z (f32)
  if (mode == kModePerturb || mode == kModePerturbUpdate) {
    p = TR::rnd(p + TR::rnd(ps * z));                  // param.data + scaling_factor * eps * z
    if (mode == kModePerturb || !upd) return p;         // (upd: the device-side apply decision)
  }
  if (mode == kModeUpdate || mode == kModePerturbUpdate) {
    const float gz = TR::rnd(g * z);                    // directional_derivative_value * z
    const float t2 = TR::rnd(gz + TR::rnd(wd * p));     // + weight_decay * param.data
    const float t = has_wd ? t2 : gz;                   // (select: keeps the seed loop branch-free)
    return TR::rnd(p - TR::rnd(lr * t));                // param.data - lr * (...)
  }
  return z;
}

// The directional value of a device-side perturb_step (fks_perturb_step_dev): v[0] = g
// (f32) rounded to the parameter dtype like a VALUE_TENSOR host value, v[1] != 0 applies
// the update.  Read once per workgroup, wave-uniform.
template <int DT>
__device__ __forceinline__ float dev_value_g(const float* v) {
  const float g = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v[0])));
  return is_f32(DT) ? g : Traits<DT>::rnd(g);
}
__device__ __forceinline__ bool dev_value_apply(const float* v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v[1]))) != 0.0f;
}

// ------------------------------------------------------------------ jump kernel
// grid (nseeds, ceil(nchunks / chunks_per_wg)); block kJumpThreads (16 waves).
// LDS holds one phase of the seed's x words (below) at a 3-word offset, so that
// y = x + 1 is 16-byte aligned.  Each wave evaluates the jump
// of one chunk at a time: lane l < 63 owns window words w = 10l .. 10l+9 and sweeps
// the 19937 coefficients of c(t) = t^J mod phi four at a time (jump_quad_step10; the
// 2-bit pair step it replaced and the one-phase kernel are in git history (commit
// 9dd4861); A/B logs profiles/r04n_jump_quad_ab.log, r04x_jump_2phase_ab.log), keeping
// y[i + 10l .. i + 10l + 15] in a 16-register sliding window fed by two ds_read_b64
// per step:  acc[j] ^= y[i + d + 10l + j] & -c[i + d]   (d = 0..3, j = 0..9).
constexpr int kJumpXOff = 3;            // x at word 3 -> y = x + 1 at word 4 (16 B aligned)

// acc[j] ^= XOR over the set bits d of the wave-uniform 4-bit code of w[d + j] (j < 10):
// coefficients 4 at a time.  A binary tree of scalar bit tests picks one of 16 bodies
// (none, one v_xor_b32, one v_bitop3_b32, or two of them per word), so a random polynomial
// costs 1.25 VALU ops per word per 4 coefficients -- 0.3125 per coefficient against the
// pair step's 0.375 -- and 4 scalar tests instead of 2 x (1-3) compares.
__device__ __forceinline__ void jump_quad_step10(uint32_t (&acc)[10], const uint32_t (&w)[13], uint32_t code) {
  asm volatile(
      "s_bitcmp1_b32 %[c], 3\n"
      "s_cbranch_scc1 .Lqb3k8x%=\n"
      "s_bitcmp1_b32 %[c], 2\n"
      "s_cbranch_scc1 .Lqb2k4x%=\n"
      "s_bitcmp1_b32 %[c], 1\n"
      "s_cbranch_scc1 .Lqb1k2x%=\n"
      "s_bitcmp1_b32 %[c], 0\n"
      "s_cbranch_scc1 .Lqb0k1x%=\n"
      "s_branch .Lqendx%=\n"
      ".Lqb0k1x%=:\n"
      "v_xor_b32 %[a0], %[a0], %[w0]\n"
      "v_xor_b32 %[a1], %[a1], %[w1]\n"
      "v_xor_b32 %[a2], %[a2], %[w2]\n"
      "v_xor_b32 %[a3], %[a3], %[w3]\n"
      "v_xor_b32 %[a4], %[a4], %[w4]\n"
      "v_xor_b32 %[a5], %[a5], %[w5]\n"
      "v_xor_b32 %[a6], %[a6], %[w6]\n"
      "v_xor_b32 %[a7], %[a7], %[w7]\n"
      "v_xor_b32 %[a8], %[a8], %[w8]\n"
      "v_xor_b32 %[a9], %[a9], %[w9]\n"
      "s_branch .Lqendx%=\n"
      ".Lqb1k2x%=:\n"
      "s_bitcmp1_b32 %[c], 0\n"
      "s_cbranch_scc1 .Lqb0k3x%=\n"
      "v_xor_b32 %[a0], %[a0], %[w1]\n"
      "v_xor_b32 %[a1], %[a1], %[w2]\n"
      "v_xor_b32 %[a2], %[a2], %[w3]\n"
      "v_xor_b32 %[a3], %[a3], %[w4]\n"
      "v_xor_b32 %[a4], %[a4], %[w5]\n"
      "v_xor_b32 %[a5], %[a5], %[w6]\n"
      "v_xor_b32 %[a6], %[a6], %[w7]\n"
      "v_xor_b32 %[a7], %[a7], %[w8]\n"
      "v_xor_b32 %[a8], %[a8], %[w9]\n"
      "v_xor_b32 %[a9], %[a9], %[w10]\n"
      "s_branch .Lqendx%=\n"
      ".Lqb0k3x%=:\n"
      "v_bitop3_b32 %[a0], %[a0], %[w0], %[w1] bitop3:0x96\n"
      "v_bitop3_b32 %[a1], %[a1], %[w1], %[w2] bitop3:0x96\n"
      "v_bitop3_b32 %[a2], %[a2], %[w2], %[w3] bitop3:0x96\n"
      "v_bitop3_b32 %[a3], %[a3], %[w3], %[w4] bitop3:0x96\n"
      "v_bitop3_b32 %[a4], %[a4], %[w4], %[w5] bitop3:0x96\n"
      "v_bitop3_b32 %[a5], %[a5], %[w5], %[w6] bitop3:0x96\n"
      "v_bitop3_b32 %[a6], %[a6], %[w6], %[w7] bitop3:0x96\n"
      "v_bitop3_b32 %[a7], %[a7], %[w7], %[w8] bitop3:0x96\n"
      "v_bitop3_b32 %[a8], %[a8], %[w8], %[w9] bitop3:0x96\n"
      "v_bitop3_b32 %[a9], %[a9], %[w9], %[w10] bitop3:0x96\n"
      "s_branch .Lqendx%=\n"
      ".Lqb2k4x%=:\n"
      "s_bitcmp1_b32 %[c], 1\n"
      "s_cbranch_scc1 .Lqb1k6x%=\n"
      "s_bitcmp1_b32 %[c], 0\n"
      "s_cbranch_scc1 .Lqb0k5x%=\n"
      "v_xor_b32 %[a0], %[a0], %[w2]\n"
      "v_xor_b32 %[a1], %[a1], %[w3]\n"
      "v_xor_b32 %[a2], %[a2], %[w4]\n"
      "v_xor_b32 %[a3], %[a3], %[w5]\n"
      "v_xor_b32 %[a4], %[a4], %[w6]\n"
      "v_xor_b32 %[a5], %[a5], %[w7]\n"
      "v_xor_b32 %[a6], %[a6], %[w8]\n"
      "v_xor_b32 %[a7], %[a7], %[w9]\n"
      "v_xor_b32 %[a8], %[a8], %[w10]\n"
      "v_xor_b32 %[a9], %[a9], %[w11]\n"
      "s_branch .Lqendx%=\n"
      ".Lqb0k5x%=:\n"
      "v_bitop3_b32 %[a0], %[a0], %[w0], %[w2] bitop3:0x96\n"
      "v_bitop3_b32 %[a1], %[a1], %[w1], %[w3] bitop3:0x96\n"
      "v_bitop3_b32 %[a2], %[a2], %[w2], %[w4] bitop3:0x96\n"
      "v_bitop3_b32 %[a3], %[a3], %[w3], %[w5] bitop3:0x96\n"
      "v_bitop3_b32 %[a4], %[a4], %[w4], %[w6] bitop3:0x96\n"
      "v_bitop3_b32 %[a5], %[a5], %[w5], %[w7] bitop3:0x96\n"
      "v_bitop3_b32 %[a6], %[a6], %[w6], %[w8] bitop3:0x96\n"
      "v_bitop3_b32 %[a7], %[a7], %[w7], %[w9] bitop3:0x96\n"
      "v_bitop3_b32 %[a8], %[a8], %[w8], %[w10] bitop3:0x96\n"
      "v_bitop3_b32 %[a9], %[a9], %[w9], %[w11] bitop3:0x96\n"
      "s_branch .Lqendx%=\n"
      ".Lqb1k6x%=:\n"
      "s_bitcmp1_b32 %[c], 0\n"
      "s_cbranch_scc1 .Lqb0k7x%=\n"
      "v_bitop3_b32 %[a0], %[a0], %[w1], %[w2] bitop3:0x96\n"
      "v_bitop3_b32 %[a1], %[a1], %[w2], %[w3] bitop3:0x96\n"
      "v_bitop3_b32 %[a2], %[a2], %[w3], %[w4] bitop3:0x96\n"
      "v_bitop3_b32 %[a3], %[a3], %[w4], %[w5] bitop3:0x96\n"
      "v_bitop3_b32 %[a4], %[a4], %[w5], %[w6] bitop3:0x96\n"
      "v_bitop3_b32 %[a5], %[a5], %[w6], %[w7] bitop3:0x96\n"
      "v_bitop3_b32 %[a6], %[a6], %[w7], %[w8] bitop3:0x96\n"
      "v_bitop3_b32 %[a7], %[a7], %[w8], %[w9] bitop3:0x96\n"
      "v_bitop3_b32 %[a8], %[a8], %[w9], %[w10] bitop3:0x96\n"
      "v_bitop3_b32 %[a9], %[a9], %[w10], %[w11] bitop3:0x96\n"
      "s_branch .Lqendx%=\n"
      ".Lqb0k7x%=:\n"
      "v_bitop3_b32 %[a0], %[a0], %[w0], %[w1] bitop3:0x96\n"
      "v_xor_b32 %[a0], %[a0], %[w2]\n"
      "v_bitop3_b32 %[a1], %[a1], %[w1], %[w2] bitop3:0x96\n"
      "v_xor_b32 %[a1], %[a1], %[w3]\n"
      "v_bitop3_b32 %[a2], %[a2], %[w2], %[w3] bitop3:0x96\n"
      "v_xor_b32 %[a2], %[a2], %[w4]\n"
      "v_bitop3_b32 %[a3], %[a3], %[w3], %[w4] bitop3:0x96\n"
      "v_xor_b32 %[a3], %[a3], %[w5]\n"
      "v_bitop3_b32 %[a4], %[a4], %[w4], %[w5] bitop3:0x96\n"
      "v_xor_b32 %[a4], %[a4], %[w6]\n"
      "v_bitop3_b32 %[a5], %[a5], %[w5], %[w6] bitop3:0x96\n"
      "v_xor_b32 %[a5], %[a5], %[w7]\n"
      "v_bitop3_b32 %[a6], %[a6], %[w6], %[w7] bitop3:0x96\n"
      "v_xor_b32 %[a6], %[a6], %[w8]\n"
      "v_bitop3_b32 %[a7], %[a7], %[w7], %[w8] bitop3:0x96\n"
      "v_xor_b32 %[a7], %[a7], %[w9]\n"
      "v_bitop3_b32 %[a8], %[a8], %[w8], %[w9] bitop3:0x96\n"
      "v_xor_b32 %[a8], %[a8], %[w10]\n"
      "v_bitop3_b32 %[a9], %[a9], %[w9], %[w10] bitop3:0x96\n"
      "v_xor_b32 %[a9], %[a9], %[w11]\n"
      "s_branch .Lqendx%=\n"
      ".Lqb3k8x%=:\n"
      "s_bitcmp1_b32 %[c], 2\n"
      "s_cbranch_scc1 .Lqb2k12x%=\n"
      "s_bitcmp1_b32 %[c], 1\n"
      "s_cbranch_scc1 .Lqb1k10x%=\n"
      "s_bitcmp1_b32 %[c], 0\n"
      "s_cbranch_scc1 .Lqb0k9x%=\n"
      "v_xor_b32 %[a0], %[a0], %[w3]\n"
      "v_xor_b32 %[a1], %[a1], %[w4]\n"
      "v_xor_b32 %[a2], %[a2], %[w5]\n"
      "v_xor_b32 %[a3], %[a3], %[w6]\n"
      "v_xor_b32 %[a4], %[a4], %[w7]\n"
      "v_xor_b32 %[a5], %[a5], %[w8]\n"
      "v_xor_b32 %[a6], %[a6], %[w9]\n"
      "v_xor_b32 %[a7], %[a7], %[w10]\n"
      "v_xor_b32 %[a8], %[a8], %[w11]\n"
      "v_xor_b32 %[a9], %[a9], %[w12]\n"
      "s_branch .Lqendx%=\n"
      ".Lqb0k9x%=:\n"
      "v_bitop3_b32 %[a0], %[a0], %[w0], %[w3] bitop3:0x96\n"
      "v_bitop3_b32 %[a1], %[a1], %[w1], %[w4] bitop3:0x96\n"
      "v_bitop3_b32 %[a2], %[a2], %[w2], %[w5] bitop3:0x96\n"
      "v_bitop3_b32 %[a3], %[a3], %[w3], %[w6] bitop3:0x96\n"
      "v_bitop3_b32 %[a4], %[a4], %[w4], %[w7] bitop3:0x96\n"
      "v_bitop3_b32 %[a5], %[a5], %[w5], %[w8] bitop3:0x96\n"
      "v_bitop3_b32 %[a6], %[a6], %[w6], %[w9] bitop3:0x96\n"
      "v_bitop3_b32 %[a7], %[a7], %[w7], %[w10] bitop3:0x96\n"
      "v_bitop3_b32 %[a8], %[a8], %[w8], %[w11] bitop3:0x96\n"
      "v_bitop3_b32 %[a9], %[a9], %[w9], %[w12] bitop3:0x96\n"
      "s_branch .Lqendx%=\n"
      ".Lqb1k10x%=:\n"
      "s_bitcmp1_b32 %[c], 0\n"
      "s_cbranch_scc1 .Lqb0k11x%=\n"
      "v_bitop3_b32 %[a0], %[a0], %[w1], %[w3] bitop3:0x96\n"
      "v_bitop3_b32 %[a1], %[a1], %[w2], %[w4] bitop3:0x96\n"
      "v_bitop3_b32 %[a2], %[a2], %[w3], %[w5] bitop3:0x96\n"
      "v_bitop3_b32 %[a3], %[a3], %[w4], %[w6] bitop3:0x96\n"
      "v_bitop3_b32 %[a4], %[a4], %[w5], %[w7] bitop3:0x96\n"
      "v_bitop3_b32 %[a5], %[a5], %[w6], %[w8] bitop3:0x96\n"
      "v_bitop3_b32 %[a6], %[a6], %[w7], %[w9] bitop3:0x96\n"
      "v_bitop3_b32 %[a7], %[a7], %[w8], %[w10] bitop3:0x96\n"
      "v_bitop3_b32 %[a8], %[a8], %[w9], %[w11] bitop3:0x96\n"
      "v_bitop3_b32 %[a9], %[a9], %[w10], %[w12] bitop3:0x96\n"
      "s_branch .Lqendx%=\n"
      ".Lqb0k11x%=:\n"
      "v_bitop3_b32 %[a0], %[a0], %[w0], %[w1] bitop3:0x96\n"
      "v_xor_b32 %[a0], %[a0], %[w3]\n"
      "v_bitop3_b32 %[a1], %[a1], %[w1], %[w2] bitop3:0x96\n"
      "v_xor_b32 %[a1], %[a1], %[w4]\n"
      "v_bitop3_b32 %[a2], %[a2], %[w2], %[w3] bitop3:0x96\n"
      "v_xor_b32 %[a2], %[a2], %[w5]\n"
      "v_bitop3_b32 %[a3], %[a3], %[w3], %[w4] bitop3:0x96\n"
      "v_xor_b32 %[a3], %[a3], %[w6]\n"
      "v_bitop3_b32 %[a4], %[a4], %[w4], %[w5] bitop3:0x96\n"
      "v_xor_b32 %[a4], %[a4], %[w7]\n"
      "v_bitop3_b32 %[a5], %[a5], %[w5], %[w6] bitop3:0x96\n"
      "v_xor_b32 %[a5], %[a5], %[w8]\n"
      "v_bitop3_b32 %[a6], %[a6], %[w6], %[w7] bitop3:0x96\n"
      "v_xor_b32 %[a6], %[a6], %[w9]\n"
      "v_bitop3_b32 %[a7], %[a7], %[w7], %[w8] bitop3:0x96\n"
      "v_xor_b32 %[a7], %[a7], %[w10]\n"
      "v_bitop3_b32 %[a8], %[a8], %[w8], %[w9] bitop3:0x96\n"
      "v_xor_b32 %[a8], %[a8], %[w11]\n"
      "v_bitop3_b32 %[a9], %[a9], %[w9], %[w10] bitop3:0x96\n"
      "v_xor_b32 %[a9], %[a9], %[w12]\n"
      "s_branch .Lqendx%=\n"
      ".Lqb2k12x%=:\n"
      "s_bitcmp1_b32 %[c], 1\n"
      "s_cbranch_scc1 .Lqb1k14x%=\n"
      "s_bitcmp1_b32 %[c], 0\n"
      "s_cbranch_scc1 .Lqb0k13x%=\n"
      "v_bitop3_b32 %[a0], %[a0], %[w2], %[w3] bitop3:0x96\n"
      "v_bitop3_b32 %[a1], %[a1], %[w3], %[w4] bitop3:0x96\n"
      "v_bitop3_b32 %[a2], %[a2], %[w4], %[w5] bitop3:0x96\n"
      "v_bitop3_b32 %[a3], %[a3], %[w5], %[w6] bitop3:0x96\n"
      "v_bitop3_b32 %[a4], %[a4], %[w6], %[w7] bitop3:0x96\n"
      "v_bitop3_b32 %[a5], %[a5], %[w7], %[w8] bitop3:0x96\n"
      "v_bitop3_b32 %[a6], %[a6], %[w8], %[w9] bitop3:0x96\n"
      "v_bitop3_b32 %[a7], %[a7], %[w9], %[w10] bitop3:0x96\n"
      "v_bitop3_b32 %[a8], %[a8], %[w10], %[w11] bitop3:0x96\n"
      "v_bitop3_b32 %[a9], %[a9], %[w11], %[w12] bitop3:0x96\n"
      "s_branch .Lqendx%=\n"
      ".Lqb0k13x%=:\n"
      "v_bitop3_b32 %[a0], %[a0], %[w0], %[w2] bitop3:0x96\n"
      "v_xor_b32 %[a0], %[a0], %[w3]\n"
      "v_bitop3_b32 %[a1], %[a1], %[w1], %[w3] bitop3:0x96\n"
      "v_xor_b32 %[a1], %[a1], %[w4]\n"
      "v_bitop3_b32 %[a2], %[a2], %[w2], %[w4] bitop3:0x96\n"
      "v_xor_b32 %[a2], %[a2], %[w5]\n"
      "v_bitop3_b32 %[a3], %[a3], %[w3], %[w5] bitop3:0x96\n"
      "v_xor_b32 %[a3], %[a3], %[w6]\n"
      "v_bitop3_b32 %[a4], %[a4], %[w4], %[w6] bitop3:0x96\n"
      "v_xor_b32 %[a4], %[a4], %[w7]\n"
      "v_bitop3_b32 %[a5], %[a5], %[w5], %[w7] bitop3:0x96\n"
      "v_xor_b32 %[a5], %[a5], %[w8]\n"
      "v_bitop3_b32 %[a6], %[a6], %[w6], %[w8] bitop3:0x96\n"
      "v_xor_b32 %[a6], %[a6], %[w9]\n"
      "v_bitop3_b32 %[a7], %[a7], %[w7], %[w9] bitop3:0x96\n"
      "v_xor_b32 %[a7], %[a7], %[w10]\n"
      "v_bitop3_b32 %[a8], %[a8], %[w8], %[w10] bitop3:0x96\n"
      "v_xor_b32 %[a8], %[a8], %[w11]\n"
      "v_bitop3_b32 %[a9], %[a9], %[w9], %[w11] bitop3:0x96\n"
      "v_xor_b32 %[a9], %[a9], %[w12]\n"
      "s_branch .Lqendx%=\n"
      ".Lqb1k14x%=:\n"
      "s_bitcmp1_b32 %[c], 0\n"
      "s_cbranch_scc1 .Lqb0k15x%=\n"
      "v_bitop3_b32 %[a0], %[a0], %[w1], %[w2] bitop3:0x96\n"
      "v_xor_b32 %[a0], %[a0], %[w3]\n"
      "v_bitop3_b32 %[a1], %[a1], %[w2], %[w3] bitop3:0x96\n"
      "v_xor_b32 %[a1], %[a1], %[w4]\n"
      "v_bitop3_b32 %[a2], %[a2], %[w3], %[w4] bitop3:0x96\n"
      "v_xor_b32 %[a2], %[a2], %[w5]\n"
      "v_bitop3_b32 %[a3], %[a3], %[w4], %[w5] bitop3:0x96\n"
      "v_xor_b32 %[a3], %[a3], %[w6]\n"
      "v_bitop3_b32 %[a4], %[a4], %[w5], %[w6] bitop3:0x96\n"
      "v_xor_b32 %[a4], %[a4], %[w7]\n"
      "v_bitop3_b32 %[a5], %[a5], %[w6], %[w7] bitop3:0x96\n"
      "v_xor_b32 %[a5], %[a5], %[w8]\n"
      "v_bitop3_b32 %[a6], %[a6], %[w7], %[w8] bitop3:0x96\n"
      "v_xor_b32 %[a6], %[a6], %[w9]\n"
      "v_bitop3_b32 %[a7], %[a7], %[w8], %[w9] bitop3:0x96\n"
      "v_xor_b32 %[a7], %[a7], %[w10]\n"
      "v_bitop3_b32 %[a8], %[a8], %[w9], %[w10] bitop3:0x96\n"
      "v_xor_b32 %[a8], %[a8], %[w11]\n"
      "v_bitop3_b32 %[a9], %[a9], %[w10], %[w11] bitop3:0x96\n"
      "v_xor_b32 %[a9], %[a9], %[w12]\n"
      "s_branch .Lqendx%=\n"
      ".Lqb0k15x%=:\n"
      "v_bitop3_b32 %[a0], %[a0], %[w0], %[w1] bitop3:0x96\n"
      "v_bitop3_b32 %[a0], %[a0], %[w2], %[w3] bitop3:0x96\n"
      "v_bitop3_b32 %[a1], %[a1], %[w1], %[w2] bitop3:0x96\n"
      "v_bitop3_b32 %[a1], %[a1], %[w3], %[w4] bitop3:0x96\n"
      "v_bitop3_b32 %[a2], %[a2], %[w2], %[w3] bitop3:0x96\n"
      "v_bitop3_b32 %[a2], %[a2], %[w4], %[w5] bitop3:0x96\n"
      "v_bitop3_b32 %[a3], %[a3], %[w3], %[w4] bitop3:0x96\n"
      "v_bitop3_b32 %[a3], %[a3], %[w5], %[w6] bitop3:0x96\n"
      "v_bitop3_b32 %[a4], %[a4], %[w4], %[w5] bitop3:0x96\n"
      "v_bitop3_b32 %[a4], %[a4], %[w6], %[w7] bitop3:0x96\n"
      "v_bitop3_b32 %[a5], %[a5], %[w5], %[w6] bitop3:0x96\n"
      "v_bitop3_b32 %[a5], %[a5], %[w7], %[w8] bitop3:0x96\n"
      "v_bitop3_b32 %[a6], %[a6], %[w6], %[w7] bitop3:0x96\n"
      "v_bitop3_b32 %[a6], %[a6], %[w8], %[w9] bitop3:0x96\n"
      "v_bitop3_b32 %[a7], %[a7], %[w7], %[w8] bitop3:0x96\n"
      "v_bitop3_b32 %[a7], %[a7], %[w9], %[w10] bitop3:0x96\n"
      "v_bitop3_b32 %[a8], %[a8], %[w8], %[w9] bitop3:0x96\n"
      "v_bitop3_b32 %[a8], %[a8], %[w10], %[w11] bitop3:0x96\n"
      "v_bitop3_b32 %[a9], %[a9], %[w9], %[w10] bitop3:0x96\n"
      "v_bitop3_b32 %[a9], %[a9], %[w11], %[w12] bitop3:0x96\n"
      ".Lqendx%=:\n"
      : [a0] "+v"(acc[0]), [a1] "+v"(acc[1]), [a2] "+v"(acc[2]), [a3] "+v"(acc[3]), [a4] "+v"(acc[4]), [a5] "+v"(acc[5]), [a6] "+v"(acc[6]), [a7] "+v"(acc[7]), [a8] "+v"(acc[8]), [a9] "+v"(acc[9])
      : [w0] "v"(w[0]), [w1] "v"(w[1]), [w2] "v"(w[2]), [w3] "v"(w[3]), [w4] "v"(w[4]), [w5] "v"(w[5]), [w6] "v"(w[6]), [w7] "v"(w[7]), [w8] "v"(w[8]), [w9] "v"(w[9]), [w10] "v"(w[10]), [w11] "v"(w[11]), [w12] "v"(w[12]), [c] "s"(code)
      : "scc");
}
__device__ __forceinline__ uint4 lds_b64x2(const uint32_t* p) {  // 8-byte aligned: two ds_read_b64
  const uint2 lo = *reinterpret_cast<const uint2*>(p), hi = *reinterpret_cast<const uint2*>(p + 2);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}

// The sweep in two phases of 156 coefficient words (9984 coefficients) each, so that LDS
// holds only the x words one phase's windows read (10,624 words, 42.5 KB, plus the 624
// seeding words) instead of all 20,561: two workgroups per CU instead of one, 8 waves per
// SIMD to hide the scalar branches of the 4-bit steps.  The phases take turns in LDS
// between a wave's jobs (A B, B A, ...): the accumulation is an xor, so their order does
// not matter, and each switch regenerates the other phase's words from 624 saved ones.
constexpr int kJumpPhaseWd = 156;                     // coefficient words (of 312) per phase
constexpr int kJumpPhaseX = 64 * kJumpPhaseWd + 640;  // x words a phase reads: 9984 + 10 x 62 + 19 + 1, rounded up
constexpr int kJumpInitOff = kJumpXOff + kJumpPhaseX;  // the 624 seeding words, kept for phase A
constexpr int kJumpLds2Words = kJumpInitOff + kMtN;

__global__ __launch_bounds__(kJumpThreads) void fks_jump_kernel(JumpArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_j[];
  uint32_t* lx = lds_j + kJumpXOff;  // phase P: lx[t] = x[9984 P + t]
  uint32_t* x0 = lds_j + kJumpInitOff;
  const int tid = threadIdx.x;
  const int k = blockIdx.x;
  const uint64_t seed = a.seeds[k];
  // mt19937::init_with_uint32 (MT19937RNGEngine.h:156-162): a serial recurrence
  if (tid == 0) {
    uint32_t s = (uint32_t)(seed & 0xffffffffu);
    x0[0] = s;
    for (int j = 1; j < kMtN; j++) {
      s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)j;
      x0[j] = s;
    }
  }
  __syncthreads();
  // fill LDS with phase P's words: its first 624 (the seeding words, or x[9984..10607]
  // from phase A's words in place), then x[n] = x[n-227] ^ twist(x[n-624], x[n-623]) in
  // steps of 227 independent words.  Callers are past a barrier that ends every read of
  // the other phase.
  auto fill = [&](const int P) {
    if (tid < kMtN) lx[tid] = P == 0 ? x0[tid] : lx[64 * kJumpPhaseWd + tid];
    __syncthreads();
    for (int base = kMtN; base < kJumpPhaseX; base += kMtN - kMtM) {
      const int n = base + tid;
      if (tid < kMtN - kMtM && n < kJumpPhaseX) lx[n] = lx[n - (kMtN - kMtM)] ^ mt_twist(lx[n - kMtN], lx[n - kMtN + 1]);
      __syncthreads();
    }
  };
  fill(0);
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  constexpr int kW = 10, kLanes = 63;  // 63 lanes x 10 words (lane 62 keeps words 620..623)
  const uint32_t* yb = lx + 1 + kW * lane;  // y[9984 P + kW lane]
  const int c0 = blockIdx.y * a.chunks_per_wg;
  const int c1 = min(c0 + a.chunks_per_wg, a.nchunks);
  const int st = a.stride > 0 ? a.stride : 1;
  constexpr int kWaves = kJumpThreads / 64;
  const int nround = (c1 - c0 + kWaves - 1) / kWaves;  // workgroup-uniform
  int P = 0;  // the phase in LDS
  for (int r = 0; r < nround; r++) {
    const int c = c0 + wave + kWaves * r;
    const bool job = c < c1 && lane < kLanes;
    const int64_t b = c < c1 ? a.chunk_block[(size_t)c * st] : 0;
    const bool sweep = c < c1 && b != 0;  // wave-uniform
    const uint64_t* poly = a.polys + (size_t)(c < c1 ? c : c0) * st * 312;  // wave-uniform: scalar loads
    uint32_t acc[kW];
#pragma unroll
    for (int j = 0; j < kW; j++) acc[j] = 0u;
    if (job && b == 0) {
#pragma unroll
      for (int j = 0; j < kW; j++) acc[j] = kW * lane + j < kMtN ? x0[kW * lane + j] : 0u;
    }
    for (int h = 0; h < 2; h++) {
      if (h == 1) {  // switch the phase in LDS
        __syncthreads();
        P ^= 1;
        fill(P);
      }
      if (sweep && lane < kLanes) {
        uint32_t win[16];
        {
          const uint4 q0 = lds_b64x2(yb), q1 = lds_b64x2(yb + 4), q2 = lds_b64x2(yb + 8), q3 = lds_b64x2(yb + 12);
          win[0] = q0.x; win[1] = q0.y; win[2] = q0.z; win[3] = q0.w;
          win[4] = q1.x; win[5] = q1.y; win[6] = q1.z; win[7] = q1.w;
          win[8] = q2.x; win[9] = q2.y; win[10] = q2.z; win[11] = q2.w;
          win[12] = q3.x; win[13] = q3.y; win[14] = q3.z; win[15] = q3.w;
        }
        const uint64_t* pw = poly + kJumpPhaseWd * P;
        uint64_t next = pw[0];
        for (int wd = 0; wd < kJumpPhaseWd; wd++) {
          const uint64_t bits = next;
          if (wd + 1 < kJumpPhaseWd) next = pw[wd + 1];  // prefetch the next 64 coefficients
          const uint32_t lo = (uint32_t)bits, hi = (uint32_t)(bits >> 32);
          const uint32_t* yw = yb + 64 * wd;
#pragma unroll
          for (int q = 0; q < 16; q++) {
            // window = y[9984 P + 64 wd + 4q + kW lane + 0..15], stored rotated by 4q (mod 16)
            const uint4 nx = lds_b64x2(yw + 4 * q + 16);
            const int rot = (4 * q) & 15;
            const uint32_t word = q < 8 ? lo : hi;
            const uint32_t quad = (word >> ((4 * q) & 31)) & 15u;
            uint32_t w13[13];
#pragma unroll
            for (int t = 0; t < 13; t++) w13[t] = win[(rot + t) & 15];
            jump_quad_step10(acc, w13, quad);
            win[(rot + 0) & 15] = nx.x;
            win[(rot + 1) & 15] = nx.y;
            win[(rot + 2) & 15] = nx.z;
            win[(rot + 3) & 15] = nx.w;
          }
        }
      }
    }
    if (job) {
      uint32_t* out = a.states + ((size_t)(a.use_slot ? a.slot[k] : (uint32_t)k) * a.nchunks + c) * kMtN + kW * lane;
#pragma unroll
      for (int j = 0; j < kW; j += 2)
        if (kW * lane + j < kMtN) *reinterpret_cast<uint2*>(out + j) = make_uint2(acc[j], acc[j + 1]);
    }
  }
}

// ------------------------------------------------------------------ apply kernel
// LDS accessors by byte offset.  The apply kernel's only LDS is its dynamic block,
// which starts at LDS address 0 (no static __shared__; checked at kernel entry), so an
// offset IS the address: immediates fold into ds_read/ds_write and no base add is
// spent per access.
typedef __attribute__((address_space(3))) uint32_t lds_u32_t;
typedef __attribute__((address_space(3))) uint64_t lds_u64_t;
typedef __attribute__((address_space(3))) float lds_f32_t;
typedef __attribute__((address_space(3))) f32x2_t lds_f32x2_t;
__device__ __forceinline__ uint32_t lds_u32(int off) { return *(const lds_u32_t*)(size_t)off; }
__device__ __forceinline__ uint64_t lds_u64(int off) { return *(const lds_u64_t*)(size_t)off; }
__device__ __forceinline__ void lds_st(int off, uint32_t v) { *(lds_u32_t*)(size_t)off = v; }
__device__ __forceinline__ float lds_f32(uint32_t off) { return *(const lds_f32_t*)(size_t)off; }
__device__ __forceinline__ f32x2_t lds_f32x2(uint32_t off) { return *(const lds_f32x2_t*)(size_t)off; }

// next raw MT word from old words u = x[i], v = x[i+1] and m = x[i+397] (or the new
// x[i-227]): m ^ (((u & UPPER) | (v & LOWER)) >> 1) ^ (v & 1 ? MATRIX_A : 0)
// (MT19937RNGEngine.h:172-175), as 5 VALU ops: bitop3 mux, shift, 1-bit sign
// extract, bitop3 "(s & A) ^ m", xor.
constexpr unsigned kMux = 0xCA;     // a ? b : c, bitwise
constexpr unsigned kAndXor = 0x6A;  // (a & b) ^ c
__device__ __forceinline__ uint32_t mt_next(uint32_t u, uint32_t v, uint32_t m) {
  const uint32_t y = __builtin_amdgcn_bitop3_b32(0x80000000u, u, v, kMux);
  const uint32_t s = (uint32_t)__builtin_amdgcn_sbfe((int)v, 0, 1);
  return __builtin_amdgcn_bitop3_b32(s, kMatrixA, m, kAndXor) ^ (y >> 1);
}

// Seed windows in LDS: window k at kLdsTabBytes + 2496 k, its words PERMUTED inside each
// 16-block so that the Box-Muller pair (j, j+8) is one aligned 8-byte word pair: one
// conflict-free ds_read_b64 per seed and lane in the pair phase.
__host__ __device__ constexpr int wperm(int i) { return (i & ~15) | ((i & 7) << 1) | ((i >> 3) & 1); }
constexpr int kWinBytes = kMtN * 4;

// In-place twist of the windows (MT19937RNGEngine.h:164-175), WAVE-LOCAL: wave w owns
// windows w, w+5, w+10, w+15.  Word i of the new block needs OLD words i, i+1 and
// i+397 (i < 227) or the NEW word i-227, so the 624 words form 3 dependency phases
// [0,227) [227,454) [454,624); word 623 pairs with the NEW word 0.  A wave reads all
// its items of a phase into registers before writing any, and a wave's LDS
// operations execute in order, so no workgroup barrier is needed inside the twist.
// Lane l handles i = lo + l + 64 j: wperm(i + 64 j) = wperm(i) + 64 j, so each phase
// needs three per-lane byte offsets (u, v, m) and immediates for j and the window.
constexpr int kWaves = kApplyThreads / 64;
constexpr int kWinPerWave = (kMaxSeedsPerPass + kWaves - 1) / kWaves;

struct TwistPlan {
  int u[3], v[3], m[3];  // byte offsets in window 0 of words i, i+1, m-index for j = 0
  int v3last;            // phase 3, j = 2: lane 41 (i = 623) pairs with the new x[0]
  int wave;
  int lane;
};

__device__ __forceinline__ void twist_plan(TwistPlan& P, int tid, int st_base) {
  P.wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  P.lane = tid & 63;
  const int lo[3] = {0, 227, 454};
#pragma unroll
  for (int ph = 0; ph < 3; ph++) {
    const int i = lo[ph] + P.lane;
    P.u[ph] = st_base + 4 * wperm(i);
    P.v[ph] = st_base + 4 * wperm(i + 1);
    P.m[ph] = st_base + 4 * wperm(ph == 0 ? i + kMtM : i - (kMtN - kMtM));
  }
  // i = 454 + 41 + 128 = 623: its next word is the new x[0]; expressed relative to j = 2
  P.v3last = P.lane == 41 ? st_base + 4 * wperm(0) - 2 * 256 : P.v[2];
}

template <int PH>
__device__ __forceinline__ void twist_phase(const TwistPlan& P, int nseeds) {
  constexpr int len = PH == 2 ? kMtN - 454 : 227;
  constexpr int nj = (len + 63) / 64;
  uint32_t nv[kWinPerWave][nj];
#pragma unroll
  for (int t = 0; t < kWinPerWave; t++) {
    const int k = P.wave + kWaves * t;
    if (k < nseeds) {  // wave-uniform
#pragma unroll
      for (int j = 0; j < nj; j++) {
        const int w = k * kWinBytes + 256 * j;
        const int vo = (PH == 2 && j == nj - 1) ? P.v3last : P.v[PH];
        nv[t][j] = mt_next(lds_u32(P.u[PH] + w), lds_u32(vo + w), lds_u32(P.m[PH] + w));
      }
    }
  }
  asm volatile("" ::: "memory");  // every read of the phase is issued before any write
#pragma unroll
  for (int t = 0; t < kWinPerWave; t++) {
    const int k = P.wave + kWaves * t;
    if (k < nseeds) {
#pragma unroll
      for (int j = 0; j < nj; j++) {
        if (j < nj - 1 || P.lane + 64 * j < len) lds_st(P.u[PH] + k * kWinBytes + 256 * j, nv[t][j]);
      }
    }
  }
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void twist_all(const TwistPlan& P, int nseeds) {
  twist_phase<0>(P, nseeds);
  twist_phase<1>(P, nseeds);
  twist_phase<2>(P, nseeds);
}

// Out-of-place twist of ONE window by its owner wave (double-buffered small-K kernel):
// old words from the window at byte offset `src`, new words to the window at `dst`
// (offsets relative to window 0 of the plan).  Phase 0 reads old words only; phases 1
// and 2 read the new words i-227 (and word 623 the new word 0) that this wave wrote in
// earlier phases -- a wave's LDS operations execute in order, so no barrier.  Nothing
// else reads `dst` or writes `src` while this runs.
template <int PH>
__device__ __forceinline__ void twist_phase_oop(const TwistPlan& P, int src, int dst) {
  constexpr int len = PH == 2 ? kMtN - 454 : 227;
  constexpr int nj = (len + 63) / 64;
  uint32_t nv[nj];
#pragma unroll
  for (int j = 0; j < nj; j++) {
    const int vo = (PH == 2 && j == nj - 1 && P.lane == 41) ? P.v3last + dst : P.v[PH] + src;
    const int mo = P.m[PH] + (PH == 0 ? src : dst);
    nv[j] = mt_next(lds_u32(P.u[PH] + src + 256 * j), lds_u32(vo + 256 * j), lds_u32(mo + 256 * j));
  }
#pragma unroll
  for (int j = 0; j < nj; j++)
    if (j < nj - 1 || P.lane + 64 * j < len) lds_st(P.u[PH] + dst + 256 * j, nv[j]);
}

__device__ __forceinline__ void twist_oop(const TwistPlan& P, int src, int dst) {
  twist_phase_oop<0>(P, src, dst);
  twist_phase_oop<1>(P, src, dst);
  twist_phase_oop<2>(P, src, dst);
}

// The same out-of-place twist with the phases chained in REGISTERS: lane l's word
// i = lo + l + 64 j of phase 1 (2) takes as m the new word i - 227, which is this lane's
// own word (l, j) of phase 0 (1); only word 623's partner, the new word 0, crosses lanes
// (lane 0's first word, broadcast with v_readlane).  So every LDS read of the window is
// issued up front, against the old words only, and there is one LDS round trip per
// window instead of three dependent ones.
__device__ __forceinline__ void twist_oop_reg(const TwistPlan& P, int src, int dst) {
  uint32_t u0[4], v0[4], m0[4], u1[4], v1[4], u2[3], v2[3];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    u0[j] = lds_u32(P.u[0] + src + 256 * j);
    v0[j] = lds_u32(P.v[0] + src + 256 * j);
    m0[j] = lds_u32(P.m[0] + src + 256 * j);
    u1[j] = lds_u32(P.u[1] + src + 256 * j);
    v1[j] = lds_u32(P.v[1] + src + 256 * j);
  }
#pragma unroll
  for (int j = 0; j < 3; j++) {
    u2[j] = lds_u32(P.u[2] + src + 256 * j);
    v2[j] = lds_u32(P.v[2] + src + 256 * j);  // lane 41, j = 2 (i = 623): replaced below
  }
  uint32_t n0[4], n1[4], n2[3];
#pragma unroll
  for (int j = 0; j < 4; j++) n0[j] = mt_next(u0[j], v0[j], m0[j]);
#pragma unroll
  for (int j = 0; j < 4; j++) n1[j] = mt_next(u1[j], v1[j], n0[j]);
  const uint32_t x0 = __builtin_amdgcn_readlane(n0[0], 0);
#pragma unroll
  for (int j = 0; j < 3; j++) n2[j] = mt_next(u2[j], (j == 2 && P.lane == 41) ? x0 : v2[j], n1[j]);
#pragma unroll
  for (int j = 0; j < 4; j++) {
    if (j < 3 || P.lane + 192 < 227) {
      lds_st(P.u[0] + dst + 256 * j, n0[j]);
      lds_st(P.u[1] + dst + 256 * j, n1[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < 3; j++)
    if (j < 2 || P.lane + 128 < kMtN - 454) lds_st(P.u[2] + dst + 256 * j, n2[j]);
}

__constant__ float c_tab_bf16[3 * 256];  // R | C | S, set once from fks::tables()

// LDS: [R[256] f32 | (C,S)[256] f32x2 | windows (kMaxSeedsPerPass + 1) x 624 u32]
// ((R,R) pairs at the (C,S) index scale measured 8 % slower: the radius lookup moves
// twice the LDS bytes)
constexpr int kLdsRBytes = 256 * 4;
constexpr int kLdsTabBytes = kLdsRBytes + 256 * 8;
constexpr int kLdsCsOff = kLdsRBytes;
constexpr int kLdsStBytes = (kMaxSeedsPerPass + 1) * kMtN * 4;

// 64-bit shifts of a word pair held in one VGPR pair (full rate on gfx950, measured
// tools/ubench): the bits one word shifts into the other are masked off afterwards
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
template <int S>
__device__ __forceinline__ u32x2_t shr64(u32x2_t x) {
  u32x2_t r;
  asm("v_lshrrev_b64 %0, %2, %1" : "=v"(r) : "v"(x), "i"(S));
  return r;
}
template <int S>
__device__ __forceinline__ u32x2_t shl64(u32x2_t x) {
  u32x2_t r;
  asm("v_lshlrev_b64 %0, %2, %1" : "=v"(r) : "v"(x), "i"(S));
  return r;
}

// Both table byte offsets (x8) of a Box-Muller word pair y = (word j, word j+8):
// MT19937RNGEngine.h:141-145 tempering of both words, then ((y ^ (y >> 18)) & 0xFF) << 3,
// 13 VALU ops for the two words instead of 18.  y >> 11 pulls 11 bits of the high word
// into the top of the low one (mask 0x001FFFFF); y << 7 and y << 15 push the low word's
// top bits into the high word's bits 0..6 / 0..14, which the tempering masks already
// clear; the final shifts' spill lies outside 0x7F8.
__device__ __forceinline__ u32x2_t temper_pair_u8x8(u32x2_t y) {
  u32x2_t t = shr64<11>(y);
  y.x = __builtin_amdgcn_bitop3_b32(y.x, t.x, 0x001FFFFFu, kXorAnd);
  y.y ^= t.y;
  t = shl64<7>(y);
  y.x = __builtin_amdgcn_bitop3_b32(y.x, t.x, 0x9d2c5680u, kXorAnd);
  y.y = __builtin_amdgcn_bitop3_b32(y.y, t.y, 0x9d2c5680u, kXorAnd);
  // the third step y ^= (y << 15) & 0xefc60000 changes bits 17..31 only; of those the
  // index reads bits 18..25, where it adds y bits 3..10 under 0xF1 (= 0xefc60000 >> 18):
  // idx8 = ((y << 3) ^ (y >> 15) ^ (y & 0x788)) & 0x7F8 on the second step's y -- 6 ops
  // for the pair instead of 7 (checked against the four-step tempering in
  // tests/test_temper_fold.py)
  const u32x2_t t1 = shl64<3>(y), t2 = shr64<15>(y);
  u32x2_t o;
  o.x = __builtin_amdgcn_bitop3_b32(t1.x, t2.x, 0x7F8u, kXorMask);
  o.y = __builtin_amdgcn_bitop3_b32(t1.y, t2.y, 0x7F8u, kXorMask);
  o.x = __builtin_amdgcn_bitop3_b32(o.x, y.x, 0x788u, kXorAnd);
  o.y = __builtin_amdgcn_bitop3_b32(o.y, y.y, 0x788u, kXorAnd);
  return o;
}

// fp32 z pair from the two RAW words of a 16-block: normal_fill_16_AVX2
// (DistributionTemplates.h:88-106) with log256_ps / sincos256_ps (avx_mathfun.h:90-160,
// 426-520), as oracle/fks_oracle.c restates it literally, with fewer instructions -- all
// exact rewrites on this input domain (pinned by the golden fp32 streams):
//   * both words tempered on the 64-bit pair (masks clear the bits one word shifts into
//     the other; only the low 24 bits are kept);
//   * theta = 2*pi*d2 >= +0, so sincos256_ps's sign extraction and abs are identities;
//   * its select-and-add merge of the two polynomials is a swap (the adds involve an
//     exact zero; a zero's sign cannot reach z, which is rounded as radius*s + 0);
//   * radius*c + 0 (mul, then the fmadd with std 1, mean 0) is fma(radius, c, 0): the
//     exact product is never a nonzero below the subnormal range here.
__device__ __forceinline__ u32x2_t temper_pair_u24(u32x2_t y) {
  u32x2_t t = shr64<11>(y);
  y.x = __builtin_amdgcn_bitop3_b32(y.x, t.x, 0x001FFFFFu, kXorAnd);
  y.y ^= t.y;
  t = shl64<7>(y);
  y.x = __builtin_amdgcn_bitop3_b32(y.x, t.x, 0x9d2c5680u, kXorAnd);
  y.y = __builtin_amdgcn_bitop3_b32(y.y, t.y, 0x9d2c5680u, kXorAnd);
  t = shl64<15>(y);
  y.x = __builtin_amdgcn_bitop3_b32(y.x, t.x, 0xefc60000u, kXorAnd);
  y.y = __builtin_amdgcn_bitop3_b32(y.y, t.y, 0xefc60000u, kXorAnd);
  t = shr64<18>(y);
  y.x = __builtin_amdgcn_bitop3_b32(y.x, t.x, 0x3FFFu, kXorAnd) & 0xFFFFFFu;
  y.y = __builtin_amdgcn_bitop3_b32(y.y, t.y, 0xFFFFFFu, kXorMask);
  return y;
}

__device__ __forceinline__ void cephes_sincosf_nonneg(float x, float& s, float& c) {
  float y = x * 1.27323954473516f;
  int32_t imm2 = (int32_t)y;
  imm2 = (imm2 + 1) & ~1;
  y = (float)imm2;
  const uint32_t sign_bit_sin = ((uint32_t)(imm2 & 4)) << 29;
  const uint32_t sign_bit_cos = ((uint32_t)(~(imm2 - 2) & 4)) << 29;
  const bool poly_mask = (imm2 & 2) == 0;
  x = __fmaf_rn(y, -0.78515625f, x);
  x = __fmaf_rn(y, -2.4187564849853515625e-4f, x);
  x = __fmaf_rn(y, -3.77489497744594108e-8f, x);
  const float z = x * x;
  float yc = 2.443315711809948E-005f;
  yc = __fmaf_rn(yc, z, -1.388731625493765E-003f);
  yc = __fmaf_rn(yc, z, 4.166664568298827E-002f);
  yc = yc * z;
  yc = __fmaf_rn(yc, z, -(z * 0.5f));
  yc = yc + 1.0f;
  float ys = -1.9515295891E-4f;
  ys = __fmaf_rn(ys, z, 8.3321608736E-3f);
  ys = __fmaf_rn(ys, z, -1.6666654611E-1f);
  ys = ys * z;
  ys = __fmaf_rn(ys, x, x);
  const float xmm1 = poly_mask ? ys : yc;
  const float xmm2 = poly_mask ? yc : ys;
#if FKS_F32_TRIM
  // sign_bit_sin = bit 2 of imm2 at bit 31; sign_bit_cos = bit 2 of ~(imm2 - 2), i.e. the
  // complement of bit 31 of (imm2 << 29) - (2 << 29): one v_bitop3 each
  (void)sign_bit_sin;
  (void)sign_bit_cos;
  const uint32_t sh = (uint32_t)imm2 << 29;
  s = __uint_as_float(__builtin_amdgcn_bitop3_b32(__float_as_uint(xmm1), sh, 0x80000000u, kXorAnd));
  c = __uint_as_float(__builtin_amdgcn_bitop3_b32(__float_as_uint(xmm2), sh - 0x40000000u, 0x80000000u, kXorNotAnd));
#else
  s = __uint_as_float(__float_as_uint(xmm1) ^ sign_bit_sin);
  c = __uint_as_float(__float_as_uint(xmm2) ^ sign_bit_cos);
#endif
}

// Correctly rounded sqrt of the radius input x = -2 log(u1), as _mm256_sqrt_ps: the
// compiler's correctly rounded expansion (a bare v_sqrt_f32 is NOT correctly rounded on
// this domain), checked on all 2^24 inputs against the exact midpoint criterion
// (fks_device_selfcheck FKS_CHECK_SQRT_DOMAIN, a GPU test).  (Restricting it to the
// domain -- x is +-0 or in [1.19e-7, 33.3], so the rescaling and class select are dead,
// as phx_radius2 does for the Philox stream -- issues 14 % fewer VALU instructions in the
// fp32 19-seed kernel but 50 % more hazard s_nops between its compares and selects, and
// measured 3 % slower: profiles/r04h_sqrt_ab.log.  v_sqrt_f64 rounded to f32 -- three
// instructions, no select -- is 4.7 % faster but NOT correctly rounded: the self check
// counts 1,326,243 of the 2^24 inputs wrong, profiles/r04i_sqrt64.log.)
#ifndef FKS_SQRT_F64NR
#define FKS_SQRT_F64NR 0
#endif
#if FKS_SQRT_F64NR
// (A/B) the root in double: v_rsq_f64 (relative error <= 2^-22), two Newton steps with the
// fixed half-reciprocal (error ~1.5 e^3 < 2^-60, then one f64 rounding), one rounding to
// float -- the correctly rounded root, as sqrt of a 24-bit float lies at least ~2^-49
// (relative) from an f32 rounding midpoint; +-0 passes through (sqrt(+-0) = +-0)
__device__ __forceinline__ float radius_sqrt(float x) {
  const double d = (double)x;
  const double t = __builtin_amdgcn_rsq(d);
  const double h = 0.5 * t;
  double s = d * t;
  s = __builtin_fma(__builtin_fma(-s, s, d), h, s);
  s = __builtin_fma(__builtin_fma(-s, s, d), h, s);
  return x == 0.0f ? x : (float)s;
}
#elif defined(FKS_SQRT_INTFIX) && FKS_SQRT_INTFIX
// (A/B) ocml's correctly rounded expansion restricted to this domain (x is +-0 or a normal
// float in [1.19e-7, 33.3]: no rescaling, no class select), its two compare-selects
// replaced by integer arithmetic on the residuals' bits: with vm = fma(-(s-1ulp), s, x) and
// vp = fma(-(s+1ulp), s, x) (never -0: an exact zero sum rounds to +0), "vm <= 0" is
// 1 - [vm > 0] and [v > 0] is the sign bit of -bits(v), so the root's bits are
// bits(s) - 1 + [vp > 0] + [vm > 0]; x = +-0 keeps s (= x)
__device__ __forceinline__ float radius_sqrt(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const uint32_t sm = __float_as_uint(s) - 1u, sp = __float_as_uint(s) + 1u;
  const float vm = __fmaf_rn(-__uint_as_float(sm), s, x);
  const float vp = __fmaf_rn(-__uint_as_float(sp), s, x);
  const uint32_t r = sm + ((0u - __float_as_uint(vp)) >> 31) + ((0u - __float_as_uint(vm)) >> 31);
  return x == 0.0f ? s : __uint_as_float(r);
}
#else
__device__ __forceinline__ float radius_sqrt(float x) { return sqrtf(x); }
#endif

__device__ __forceinline__ void z_pair_f32_raw(uint32_t r1, uint32_t r2, float& z1, float& z2) {
  u32x2_t w;
  w.x = r1;
  w.y = r2;
  const u32x2_t t = temper_pair_u24(w);
#if FKS_F32_TRIM
  // u1 = 1 - d1 (exact: d1 = t.x 2^-24) as one fma; theta = RN(2pi_f * t.y 2^-24) =
  // RN((2pi_f 2^-24) * t.y), the power-of-two scaling exact: one multiply
  const float u1 = __fmaf_rn((float)t.x, -1.0f / 16777216.0f, 1.0f);
  const float theta = (float)t.y * (6.28318548202514648438f / 16777216.0f);
#else
  const float d1 = (float)t.x * (1.0f / 16777216.0f);
  const float d2 = (float)t.y * (1.0f / 16777216.0f);
  const float u1 = 1.0f - d1;
  const float theta = 6.28318548202514648438f * d2;
#endif
  const float radius = radius_sqrt(-2.0f * cephes_logf(u1));
  float s, c;
  cephes_sincosf_nonneg(theta, s, c);
  z1 = __fmaf_rn(radius, c, 0.0f);
  z2 = __fmaf_rn(radius, s, 0.0f);
}

// The libm flavour of the same pair (kDtF32Libm; normal_fill_16<float>,
// DistributionTemplates.h:139-149, under ATen's DEFAULT CPU capability): glibc's logf / sinf
// / cosf in double as fks_libm.h restates them, e_logf.c's 16 {invc, logc} pairs read from
// LDS at byte `tab`; radius * cos(theta) * std + mean with std 1, mean 0 is one rounding of
// the product and -0 -> +0, the fma with a +0 addend.
typedef double f64x2_t __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) f64x2_t lds_f64x2_t;
constexpr int kLdsLogfBytes = 16 * 16;
__device__ __forceinline__ void logf_tab_fill(uint32_t tab, int tid, int nthreads) {
  for (int i = tid; i < 16; i += nthreads)
    *(lds_f64x2_t*)(size_t)(tab + 16u * (uint32_t)i) = (f64x2_t){fks_libm::kLogfTab[i][0], fks_libm::kLogfTab[i][1]};
}
__device__ __forceinline__ void z_pair_f32_libm(uint32_t tab, uint32_t r1, uint32_t r2, float& z1, float& z2) {
  u32x2_t w;
  w.x = r1;
  w.y = r2;
  const u32x2_t t = temper_pair_u24(w);
  const float u1 = __fmaf_rn((float)t.x, -1.0f / 16777216.0f, 1.0f);  // 1 - data[j], exact
  const f64x2_t e = *(const lds_f64x2_t*)(size_t)(tab + 16u * (uint32_t)fks_libm::logf_index(u1));
  const float radius = radius_sqrt(-2.0f * fks_libm::logf_core<true>(u1, e.x, e.y));
  const float theta = fks_libm::theta_of(t.y);  // 2.0f * c10::pi<double> * data[j + 8]
  float s, c;
  fks_libm::sincosf_glibc<true>(theta, s, c);
  z1 = __fmaf_rn(radius, c, 0.0f);
  z2 = __fmaf_rn(radius, s, 0.0f);
}

// The same z pairs for TWO seeds at once (the fp32 19-seed kernel's full passes): every
// float operation of cephes_logf / the radius / cephes_sincosf_nonneg runs on the two
// seeds' values as one packed f32 instruction (v_pk_mul/add/fma_f32: per element the same
// IEEE operation, so the same bits); the integer work stays per seed.  cephes_logf's
// "x < sqrt(1/2)" select becomes integer arithmetic on the bits -- the mask is the sign of
// bits(x) - bits(0.70710678f) (x is a normal float in [0.5, 1): ordered like its bits);
// "mask ? x : 0" is bits(x) & mask and e = float(imm0 - 126 + mask) is the exact integer
// e + 1 - (mask ? 1 : 0) -- no compare, no select, no hazard wait.
__device__ __forceinline__ f32x2_t pk(float a, float b) { return (f32x2_t){a, b}; }
__device__ __forceinline__ f32x2_t pk1(float a) { return (f32x2_t){a, a}; }
// Q packed pairs side by side, every step issued for all Q before the next: a dependent
// v_pk_*_f32 right after its producer costs a wait state on gfx950, so the Horner chains
// of the Q pairs are interleaved in the source (each step's Q ops are independent).
#define FKS_Q for (int q = 0; q < Q; q++)
template <int Q>
__device__ __forceinline__ void cephes_logf2(f32x2_t (&x)[Q]) {  // every value in [2^-24, 1]
  f32x2_t e[Q], z[Q], y[Q], tm[Q];
#pragma unroll
  FKS_Q {
    float xm[2], tmv[2], ef[2];
    const uint32_t b[2] = {__float_as_uint(x[q].x), __float_as_uint(x[q].y)};
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const uint32_t xb = (b[i] & ~0x7f800000u) | 0x3f000000u;  // mantissa in [0.5, 1)
      const int32_t m = (int32_t)(xb - 0x3F3504F3u) >> 31;      // -1 iff x < 0.707106781186547524f
      xm[i] = __uint_as_float(xb);
      tmv[i] = __uint_as_float(xb & (uint32_t)m);               // mask ? x : 0
      ef[i] = (float)((int32_t)(b[i] >> 23) - 126 + m);         // (imm0 - 0x7f) + 1 - (mask ? 1 : 0)
    }
    x[q] = pk(xm[0], xm[1]);
    tm[q] = pk(tmv[0], tmv[1]);
    e[q] = pk(ef[0], ef[1]);
  }
#pragma unroll
  FKS_Q x[q] = x[q] - pk1(1.0f);
#pragma unroll
  FKS_Q x[q] = x[q] + tm[q];
#pragma unroll
  FKS_Q z[q] = x[q] * x[q];
#pragma unroll
  FKS_Q y[q] = __builtin_elementwise_fma(pk1(7.0376836292E-2f), x[q], pk1(-1.1514610310E-1f));
  constexpr float kC[7] = {1.1676998740E-1f, -1.2420140846E-1f, +1.4249322787E-1f, -1.6668057665E-1f,
                           +2.0000714765E-1f, -2.4999993993E-1f, +3.3333331174E-1f};
#pragma unroll
  for (int t = 0; t < 7; t++) {
#pragma unroll
    FKS_Q y[q] = __builtin_elementwise_fma(y[q], x[q], pk1(kC[t]));
  }
#pragma unroll
  FKS_Q y[q] = y[q] * x[q];
#pragma unroll
  FKS_Q y[q] = __builtin_elementwise_fma(y[q], z[q], e[q] * pk1(-2.12194440e-4f));
#pragma unroll
  FKS_Q y[q] = __builtin_elementwise_fma(-z[q], pk1(0.5f), y[q]);
#pragma unroll
  FKS_Q x[q] = x[q] + y[q];
#pragma unroll
  FKS_Q x[q] = __builtin_elementwise_fma(e[q], pk1(0.693359375f), x[q]);
}

template <int Q>
__device__ __forceinline__ void cephes_sincosf2_nonneg(f32x2_t (&x)[Q], f32x2_t (&s)[Q], f32x2_t (&c)[Q]) {
  f32x2_t y[Q], z[Q], yc[Q], ys[Q];
  int32_t imm2[Q][2];
#pragma unroll
  FKS_Q y[q] = x[q] * pk1(1.27323954473516f);
#pragma unroll
  FKS_Q {
    imm2[q][0] = ((int32_t)y[q].x + 1) & ~1;
    imm2[q][1] = ((int32_t)y[q].y + 1) & ~1;
    y[q] = pk((float)imm2[q][0], (float)imm2[q][1]);
  }
#pragma unroll
  FKS_Q x[q] = __builtin_elementwise_fma(y[q], pk1(-0.78515625f), x[q]);
#pragma unroll
  FKS_Q x[q] = __builtin_elementwise_fma(y[q], pk1(-2.4187564849853515625e-4f), x[q]);
#pragma unroll
  FKS_Q x[q] = __builtin_elementwise_fma(y[q], pk1(-3.77489497744594108e-8f), x[q]);
#pragma unroll
  FKS_Q z[q] = x[q] * x[q];
#pragma unroll
  FKS_Q {
    yc[q] = __builtin_elementwise_fma(pk1(2.443315711809948E-005f), z[q], pk1(-1.388731625493765E-003f));
    ys[q] = __builtin_elementwise_fma(pk1(-1.9515295891E-4f), z[q], pk1(8.3321608736E-3f));
  }
#pragma unroll
  FKS_Q {
    yc[q] = __builtin_elementwise_fma(yc[q], z[q], pk1(4.166664568298827E-002f));
    ys[q] = __builtin_elementwise_fma(ys[q], z[q], pk1(-1.6666654611E-1f));
  }
#pragma unroll
  FKS_Q {
    yc[q] = yc[q] * z[q];
    ys[q] = ys[q] * z[q];
  }
#pragma unroll
  FKS_Q {
    yc[q] = __builtin_elementwise_fma(yc[q], z[q], -(z[q] * pk1(0.5f)));
    ys[q] = __builtin_elementwise_fma(ys[q], x[q], x[q]);
  }
#pragma unroll
  FKS_Q yc[q] = yc[q] + pk1(1.0f);
#pragma unroll
  FKS_Q {
    float so[2], co[2];
    const float ysv[2] = {ys[q].x, ys[q].y}, ycv[2] = {yc[q].x, yc[q].y};
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const uint32_t sign_bit_sin = ((uint32_t)(imm2[q][i] & 4)) << 29;
      const uint32_t sign_bit_cos = ((uint32_t)(~(imm2[q][i] - 2) & 4)) << 29;
      const bool poly_mask = (imm2[q][i] & 2) == 0;
      so[i] = __uint_as_float(__float_as_uint(poly_mask ? ysv[i] : ycv[i]) ^ sign_bit_sin);
      co[i] = __uint_as_float(__float_as_uint(poly_mask ? ycv[i] : ysv[i]) ^ sign_bit_cos);
    }
    s[q] = pk(so[0], so[1]);
    c[q] = pk(co[0], co[1]);
  }
}

// z pairs (z_j, z_{j+8}) of 2Q seeds from their raw word pairs w[0..2Q) (as
// z_pair_f32_raw; seeds 2q and 2q+1 share packed float instructions)
template <int Q>
__device__ __forceinline__ void z_pair_f32x2_raw(const u32x2_t (&w)[2 * Q], f32x2_t (&zo)[2 * Q]) {
  f32x2_t d1[Q], d2[Q], v[Q], s[Q], c[Q];
#pragma unroll
  FKS_Q {
    const u32x2_t ta = temper_pair_u24(w[2 * q]), tb = temper_pair_u24(w[2 * q + 1]);
    d1[q] = pk((float)ta.x, (float)tb.x) * pk1(1.0f / 16777216.0f);
    d2[q] = pk((float)ta.y, (float)tb.y) * pk1(1.0f / 16777216.0f);
  }
#pragma unroll
  FKS_Q v[q] = pk1(1.0f) - d1[q];
  cephes_logf2<Q>(v);
#pragma unroll
  FKS_Q v[q] = pk1(-2.0f) * v[q];
  float r[2 * Q];
#pragma unroll
  FKS_Q {
    r[2 * q] = radius_sqrt(v[q].x);
    r[2 * q + 1] = radius_sqrt(v[q].y);
  }
#pragma unroll
  FKS_Q v[q] = pk1(6.28318548202514648438f) * d2[q];
  cephes_sincosf2_nonneg<Q>(v, s, c);
#pragma unroll
  FKS_Q {
    zo[2 * q] = __builtin_elementwise_fma(pk1(r[2 * q]), pk(c[q].x, s[q].x), pk1(0.0f));
    zo[2 * q + 1] = __builtin_elementwise_fma(pk1(r[2 * q + 1]), pk(c[q].y, s[q].y), pk1(0.0f));
  }
}
#undef FKS_Q

// bf16 Box-Muller pair before the final rounding: (R[a] * C[b], R[a] * S[b]) + 0 as ONE
// v_pk_fma_f32 (R*C is exact in f32: 8-bit x 8-bit significands; the +0 addend turns
// -0 into +0 like normal_fill_16's "+ mean").  (R,R) pairs at LDS 0, (C,S) pairs at 2048.
__device__ __forceinline__ f32x2_t z_pair_bf16_raw(uint32_t r1, uint32_t r2) {
  u32x2_t w;
  w.x = r1;
  w.y = r2;
  const u32x2_t ab = temper_pair_u8x8(w);
  const float r = lds_f32(ab.x >> 1);
  const f32x2_t rr = {r, r};
  const f32x2_t cs = lds_f32x2(kLdsCsOff + ab.y);
  const f32x2_t zero = {0.0f, 0.0f};
  return __builtin_elementwise_fma(rr, cs, zero);
}

// z pair of seed k for this lane's 16-block slot: raw words j1, j1+8 -> (z_j, z_{j+8})
template <int DT>
__device__ __forceinline__ void z_pair(const uint8_t* lds, uint32_t r1, uint32_t r2, float& z1, float& z2) {
  if constexpr (DT == FKS_F32) {
    z_pair_f32_raw(r1, r2, z1, z2);
  } else if constexpr (DT == kDtF32Libm) {  // the logf table at `lds` (kernels of this dtype: LDS 0)
    z_pair_f32_libm((uint32_t)(size_t)(const __attribute__((address_space(3))) uint8_t*)lds, r1, r2, z1, z2);
  } else {
    // normal_fill_16<BFloat16>: z = bf16(R[a] * C[b]) * 1 + 0 (std, mean).  R*C is exact
    // in f32 (8-bit x 8-bit significands) and fma(R, C, +0) turns -0 into +0 like "+ mean".
    const f32x2_t zz = z_pair_bf16_raw(r1, r2);
    z1 = rbf(zz.x);
    z2 = rbf(zz.y);
  }
}

// The update of an element PAIR (p1, p2) through one seed, zo_utils.py:49 / :52 and
// optimizer.py:173, in packed f32 (v_pk_mul_f32 / v_pk_add_f32: both elements per
// instruction); every op is still rounded to the parameter dtype per element, so the
// values are those of apply_one.
template <int DT>
__device__ __forceinline__ f32x2_t rnd2(f32x2_t x) {
  f32x2_t r;
  r.x = Traits<DT>::rnd(x.x);
  r.y = Traits<DT>::rnd(x.y);
  return r;
}

// The update modes' p-dependent part, given gz = rnd(g z): t = gz + rnd(wd p) (or the
// form the launch's weight decay allows), p - rnd(lr t), each op rounded to the dtype.
template <int DT, int MODE>
__device__ __forceinline__ f32x2_t apply_tail(f32x2_t p, f32x2_t gz, float lr, float wd, bool has_wd) {
  f32x2_t t;
  if (MODE == kModeUpdateNoWd || MODE == kModeUpdateWdPos0) {
    t = gz;
  } else if (MODE == kModeUpdateWd0) {
    // wd = +-0: rnd(gz + rnd(wd*p)) == fma(wd, p, gz) (fks_internal.h)
    const f32x2_t ww = {wd, wd};
    t = __builtin_elementwise_fma(ww, p, gz);
  } else {
    const f32x2_t t2 = rnd2<DT>(gz + rnd2<DT>(wd * p));
    if (MODE == kModeUpdateWd) {
      t = t2;
    } else {
      t.x = has_wd ? t2.x : gz.x;
      t.y = has_wd ? t2.y : gz.y;
    }
  }
  return rnd2<DT>(p - rnd2<DT>(lr * t));
}

template <int DT, int MODE>
__device__ __forceinline__ f32x2_t apply_pair(f32x2_t p, f32x2_t z, float g, float lr, float wd, bool has_wd,
                                              float ps, bool upd = true) {
  if (MODE == kModeDelta) {  // delta += c_k * z: one v_pk_fma_f32 per element pair and seed
    const f32x2_t gg = {g, g};
    return __builtin_elementwise_fma(gg, z, p);
  }
  if (MODE == kModePerturb || MODE == kModePerturbUpdate) {
    p = rnd2<DT>(p + rnd2<DT>(ps * z));
    if (MODE == kModePerturb || !upd) return p;
  }
  if (MODE == kModeUpdate || MODE == kModeUpdateWd || MODE == kModeUpdateNoWd || MODE == kModePerturbUpdate ||
      MODE == kModeUpdateWd0 || MODE == kModeUpdateWdPos0)
    return apply_tail<DT, MODE>(p, rnd2<DT>(g * z), lr, wd, has_wd);
  return z;
}

// f16 parameters in the torch_rocm stream.  The reference then runs torch's DEVICE
// elementwise kernels (ATen/native/cuda/CUDALoops.cuh), and how those round a Half
// "f32 scalar * f16 tensor" product depends on the code path (measured on this image,
// tools/diag_f16_tail.py, profiles/r05_f16_rounding.log):
//   * the 8-wide vectorized path -- every pointer 16-byte aligned, elements below
//     N - N % 2048 (full blocks of 256 threads x 8) -- rounds the f32 product to f16:
//     TWICE, like c10::Half on the CPU;
//   * the unrolled path -- the partial last block, or a tensor that is not 16-byte aligned
//     -- is compiled to v_fma_mixlo_f16 a, b, 0: ONE rounding of the exact product.
// The two differ when the f32 product lands on an f16 rounding midpoint (and in the sign of
// a zero product).  The chain's products: g z, lr t and the perturbation's ps z read fresh,
// aligned tensors (z, t); wd p reads the parameter -- its own alignment at the call's first
// seed, a fresh aligned tensor after it (the reference rebinds param.data every step,
// zo_utils.py:49).  The sums of two f16 values round the same either way.
__device__ __forceinline__ float mul_f16_ref(float a, float b, bool once) {  // b f16-exact
  if (once) {
    uint32_t r = 0;
    asm volatile("v_fma_mixlo_f16 %0, %1, %2, 0" : "+v"(r) : "v"(a), "v"(b));
    return (float)__builtin_bit_cast(_Float16, (uint16_t)(r & 0xffffu));
  }
  return rhf(a * b);
}
template <int MODE>
__device__ __forceinline__ f32x2_t apply_pair_f16dev(f32x2_t p, f32x2_t z, float g, float lr, float wd, bool has_wd,
                                                     float ps, bool upd, const bool (&once)[2],
                                                     const bool (&wd_once)[2]) {
  float q[2] = {p.x, p.y};
  const float zz[2] = {z.x, z.y};
  const bool use_wd = MODE == kModeUpdateNoWd ? false
                      : (MODE == kModeUpdateWd || MODE == kModeUpdateWd0 || MODE == kModeUpdateWdPos0) ? true
                                                                                                          : has_wd;
#pragma unroll
  for (int i = 0; i < 2; i++) {
    if (MODE == kModePerturb || MODE == kModePerturbUpdate) {
      q[i] = rhf(q[i] + mul_f16_ref(ps, zz[i], once[i]));
      if (MODE == kModePerturb || !upd) continue;
    }
    const float gz = mul_f16_ref(g, zz[i], once[i]);
    const float t = use_wd ? rhf(gz + mul_f16_ref(wd, q[i], wd_once[i])) : gz;
    q[i] = rhf(q[i] - mul_f16_ref(lr, t, once[i]));
  }
  return (f32x2_t){q[0], q[1]};
}

template <int DT>
__device__ __forceinline__ f32x2_t z_pair2(const uint8_t* lds, uint32_t r1, uint32_t r2) {
  f32x2_t z;
  if constexpr (DT == FKS_BF16) {
    z = rnd2<DT>(z_pair_bf16_raw(r1, r2));
  } else {
    float z1, z2;
    z_pair<DT>(lds, r1, r2, z1, z2);
    z.x = z1;
    z.y = z2;
  }
  return z;
}

// All seeds of the pass: every state-word read of the block is issued up front
// (latency hidden behind the z math of earlier seeds), z for every seed next, then
// the sequential per-element update chain in seed order.  (Staging every table index,
// then every lookup, then the products measured no faster.)
template <int DT, int MODE, int NS>
__device__ __forceinline__ void pair_all(const uint8_t* lds, int st_off, const float* g, float lr, float wd,
                                         bool has_wd, float ps, float& p1, float& p2) {
  uint32_t r1[NS], r2[NS];
#pragma unroll
  for (int k = 0; k < NS; k++) {
    const uint64_t w = lds_u64(st_off + k * kWinBytes);  // (word j, word j+8), permuted window
    r1[k] = (uint32_t)w;
    r2[k] = (uint32_t)(w >> 32);
  }
  f32x2_t z[NS];
  if constexpr (DT == FKS_F32 && FKS_F32_SEED_PAIRS > 0) {  // seed pairs share packed float ops
    constexpr int Q = FKS_F32_SEED_PAIRS > 0 ? FKS_F32_SEED_PAIRS : 1;  // pairs interleaved per step
#pragma unroll
    for (int k = 0; k + 2 * Q <= NS; k += 2 * Q) {
      u32x2_t w[2 * Q];
      f32x2_t zz[2 * Q];
#pragma unroll
      for (int i = 0; i < 2 * Q; i++) w[i] = (u32x2_t){r1[k + i], r2[k + i]};
      z_pair_f32x2_raw<Q>(w, zz);
#pragma unroll
      for (int i = 0; i < 2 * Q; i++) z[k + i] = zz[i];
    }
#pragma unroll
    for (int k = NS - NS % (2 * Q); k < NS; k++) z[k] = z_pair2<DT>(lds, r1[k], r2[k]);
  } else {
#pragma unroll
    for (int k = 0; k < NS; k++) z[k] = z_pair2<DT>(lds, r1[k], r2[k]);
  }
  f32x2_t p = {p1, p2};
#pragma unroll
  for (int k = 0; k < NS; k++) p = apply_pair<DT, MODE>(p, z[k], g[k], lr, wd, has_wd, ps);
  p1 = p.x;
  p2 = p.y;
}

// one seed (partial passes)
template <int DT, int MODE>
__device__ __forceinline__ void pair_one(const uint8_t* lds, int st_off, int k, float g, float lr, float wd,
                                         bool has_wd, float ps, float& p1, float& p2, bool upd = true) {
  const uint64_t w = lds_u64(st_off + k * kWinBytes);
  const f32x2_t z = z_pair2<DT>(lds, (uint32_t)w, (uint32_t)(w >> 32));
  f32x2_t p = {p1, p2};
  p = apply_pair<DT, MODE>(p, z, g, lr, wd, has_wd, ps, upd);
  p1 = p.x;
  p2 = p.y;
}

// DB (partial passes of <= kSmallK seeds): the windows are double-buffered -- window k
// of buffer s at kLdsTabBytes + (s * nseeds + k) * kWinBytes, + one spare for the twist's
// over-read -- and a sixth wave (kDbThreads) twists window 0 of block b+1 out of place
// while the five pair waves run block b (windows 1..3 are twisted by pair waves 4..2):
// one barrier per block instead of two, and for K=1 the twist leaves the pair waves'
// critical path (it was a third of a K=1 pass).
constexpr int kDbThreads = kApplyThreads + 64;
template <int DT, int MODE, bool FULL, bool DB = false>
__global__ __launch_bounds__(DB ? kDbThreads : kApplyThreads,
                             DB ? kDbMinWaves : (kApplyWgPerCu * kApplyThreads + 255) / 256) void fks_apply_kernel(ApplyArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds32[];
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds32);
  // the lds_* accessors address LDS by offset from 0: the dynamic block must start there
  if ((uint32_t)(size_t)(lds_u32_t*)lds32 != 0u) __builtin_trap();
  const int tid = threadIdx.x;
  const int c = blockIdx.x;
  const int nseeds = FULL ? kMaxSeedsPerPass : a.nseeds;
  const int64_t b0 = a.chunk_block[c], b1 = a.chunk_block[c + 1];

  if constexpr (DT == FKS_BF16) {
    float2* tabCS = reinterpret_cast<float2*>(lds + kLdsCsOff);
    for (int i = tid; i < 256; i += kApplyThreads) {
      reinterpret_cast<float*>(lds)[i] = c_tab_bf16[i];
      tabCS[i] = make_float2(c_tab_bf16[256 + i], c_tab_bf16[512 + i]);
    }
  } else if constexpr (DT == kDtF32Libm) {
    logf_tab_fill(0u, tid, DB ? kDbThreads : kApplyThreads);
  }
  const int buf1 = DB ? nseeds * kWinBytes : 0;  // DB: the jump windows go to buffer 1
  for (int idx = tid; idx < nseeds * kMtN; idx += (DB ? kDbThreads : kApplyThreads)) {
    const int k = idx / kMtN, i = idx - k * kMtN;
    lds_st(kLdsTabBytes + buf1 + k * kWinBytes + 4 * wperm(i), a.states[((size_t)k * a.nchunks + c) * kMtN + i]);
  }
  TwistPlan plan;
  twist_plan(plan, tid, kLdsTabBytes);
  // per-seed multipliers: wave-uniform, kept in SGPRs for the whole kernel
  float gk[kMaxSeedsPerPass];
#pragma unroll
  for (int k = 0; k < kMaxSeedsPerPass; k++)
    gk[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(k < nseeds ? a.g[k] : 0.0f)));
  // a device-side perturb_step (one seed): g and the apply decision from device memory
  bool upd = true;
  float g0 = gk[0];
  if (MODE == kModePerturbUpdate && a.gdev) {
    g0 = dev_value_g<DT == FKS_F16 ? FKS_F16 : DT>(a.gdev);
    upd = dev_value_apply(a.gdev);
  }
  __syncthreads();
  // DB: window tw is twisted by wave kWaves - tw (window 0 by the sixth, twist-only wave)
  const int tw = kWaves - plan.wave;
  const bool twister = DB && tw >= 0 && tw < nseeds;
  if constexpr (DB) {  // block b0 into buffer 0
    if (twister && b0 < b1) twist_oop(plan, buf1 + tw * kWinBytes, tw * kWinBytes);
    __syncthreads();
  }

  // Thread q < 312 owns Box-Muller pair q of every block: 16-block q/8, slot q%8,
  // i.e. block words j1 = 16*(q/8) + q%8 and j1 + 8 (DistributionTemplates.h:141-146).
  const bool lane_on = tid < kMtN / 2;
  const int j1 = 16 * (tid >> 3) + (tid & 7);
  const int st_off = kLdsTabBytes + 4 * wperm(j1);  // the (j1, j1 + 8) word pair

  // The lane's current segment, cached in registers; positions only grow.
  int cur;
  {
    const int64_t s1 = (int64_t)kMtN * b0 + j1;
    int lo = 0, hi = a.nsegs;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (a.segs[mid].start + a.segs[mid].numel <= s1) lo = mid + 1; else hi = mid;
    }
    cur = lo;
  }
  int64_t seg_start = INT64_MAX, seg_end = INT64_MAX;
  uint64_t seg_ptr = 0;
  float seg_lr = 0.0f, seg_wd = 0.0f, seg_ps = 0.0f;
  bool seg_wdf = false;
  auto load_seg = [&]() {
    if (cur < a.nsegs) {
      const DevSeg sg = a.segs[cur];
      seg_start = sg.start;
      seg_end = sg.start + sg.numel;
      seg_ptr = sg.ptr;
      seg_lr = sg.lr;
      seg_ps = sg.ps;
      seg_wd = sg.wd;
      seg_wdf = (sg.flags & FKS_HAS_WD) != 0;
    } else {
      seg_start = seg_end = INT64_MAX;
    }
    // Drain here (rare: once per segment change), so the cached segment registers are
    // never "possibly pending" later: otherwise every block's address computation would
    // carry a vmcnt(0) that also waits for the previous block's stores.
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt/lgkmcnt untouched
  };
  load_seg();

  // software pipeline: block b+1's parameters are fetched before block b's Box-Muller
  // Parameter traffic in pairs of ADJACENT elements: lane q (slot r = q%8 of its
  // 16-block) owns elements j1 = 16m + r and j1 + 8; an even lane moves the pair
  // (j1, j1+1), an odd lane the pair (j1+7, j1+8), and the two lanes swap the halves
  // that belong to each other (one DPP op) -- one dword (bf16) / dwordx2 (f32) access
  // per lane instead of two scattered ones.
  const bool odd = (tid & 1) != 0;
  // storage: the parameters, or (kModeDelta) the f32 delta buffer the z of dtype DT is
  // accumulated into
  using ST = Traits<MODE == kModeDelta ? FKS_F32 : DT>;
  constexpr int kEs = (is_f32(DT) || MODE == kModeDelta) ? 4 : 2;
  typedef typename ST::Pair Pair;
  struct Slot { uint64_t addr; float lr, wd, ps; uint32_t wdf, on; Pair raw; };
  auto fetch = [&](int64_t b) -> Slot {
    Slot sl;
    const int64_t s1 = (int64_t)kMtN * b + j1;
    while (s1 >= seg_end) { cur++; load_seg(); }
    const bool on = lane_on && s1 >= seg_start;
    sl.on = on;
    sl.lr = seg_lr; sl.wd = seg_wd; sl.ps = seg_ps; sl.wdf = seg_wdf;
    // off lanes read and write a workspace sink, so the load and the store are
    // unconditional: the store is then always counted in vmcnt and the next wait for a
    // prefetched pair can leave it outstanding (a maybe-executed store makes the
    // compiler wait for it)
    sl.addr = on ? seg_ptr + (uint64_t)(s1 - seg_start + (odd ? 7 : 0)) * kEs : (uint64_t)(uintptr_t)a.sink;
    sl.raw = 0;
    if (MODE != kModeWriteZ) sl.raw = ST::load_pair(sl.addr);
    return sl;
  };
  // One block: twist, prefetch block b+1 (returned), Box-Muller + update chain, store.
  auto step = [&](Slot sl, int64_t b) -> Slot {
    int buf = 0;  // byte offset of the buffer holding block b (DB)
    if constexpr (DB) {
      buf = (int)((b - b0) & 1) * nseeds * kWinBytes;
      const int other = nseeds * kWinBytes - buf;
      if (twister && b + 1 < b1)  // block b+1, out of place
        twist_oop(plan, buf + tw * kWinBytes, other + tw * kWinBytes);
      if (plan.wave == kWaves) {  // the twist-only wave
        __syncthreads();
        return sl;
      }
    } else {
      __syncthreads();  // every wave is done reading block b-1's words
      twist_all(plan, nseeds);  // the raw words of stream block b
      __syncthreads();  // every window holds block b
    }
    const Slot nxt = fetch(b + 1 < b1 ? b + 1 : b);  // (the last block re-reads itself, unused)
    {  // every lane: off lanes compute garbage into the sink
      // even lane holds (p1, partner's p1), odd lane (partner's p2, p2)
      const uint32_t keep = odd ? ST::hi(sl.raw) : ST::lo(sl.raw);
      const uint32_t got = swap_adjacent(odd ? ST::lo(sl.raw) : ST::hi(sl.raw));
      float p1 = ST::cvt(odd ? got : keep), p2 = ST::cvt(odd ? keep : got);
      if constexpr (FULL) {
        pair_all<DT, MODE, kMaxSeedsPerPass>(lds, st_off, gk, sl.lr, sl.wd, sl.wdf != 0, sl.ps, p1, p2);
      } else {
        // a.g[k] straight from the kernel-argument segment (one s_load per seed): a
        // dynamically indexed gk[] would be copied to VGPRs and indexed per seed
        for (int k = 0; k < nseeds; k++)
          pair_one<DT, MODE>(lds, st_off + buf, k, MODE == kModePerturbUpdate ? g0 : a.g[k], sl.lr, sl.wd,
                             sl.wdf != 0, sl.ps, p1, p2, upd);
      }
      const uint32_t b1v = ST::bits(p1), b2v = ST::bits(p2);
      const uint32_t back = swap_adjacent(odd ? b1v : b2v);  // even gets partner's p1, odd partner's p2
      const Pair out = odd ? ST::pack(back, b2v) : ST::pack(b1v, back);
      ST::store_pair(sl.addr, out);
    }
    if constexpr (DB) __syncthreads();  // block b+1 is twisted; block b's buffer is free
    return nxt;
  };
  Slot sa = fetch(b0);
  // a store after the first prefetch, so the loop is entered with the same pending
  // (load, store) shape as the back edge and the first wait can leave a store in flight
  *reinterpret_cast<volatile uint32_t*>(a.sink + 1) = 0u;
  for (int64_t b = b0; b < b1; b++) sa = step(sa, b);
}

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4_t lds_u4_t;
__device__ __forceinline__ u32x4_t lds_u4(uint32_t off) { return *(const lds_u4_t*)(size_t)off; }
__device__ __forceinline__ void lds_st4(uint32_t off, u32x4_t v) { *(lds_u4_t*)(size_t)off = v; }

// ------------------------------------------------------------------ small-K kernel v2
// (Other bf16 table layouts for the small-K kernel -- R|C|S f32, (C,S) packed as bf16 --
// measured within noise or slower: profiles/r02_smallk_ab.log.)
// bf16 z pair from the two table byte offsets (x8) of temper_pair_u8x8: the lookups and
// the rounding of z_pair_bf16_raw (default table layout)
__device__ __forceinline__ f32x2_t z_bf16_idx8(uint32_t a8, uint32_t b8) {
  const float r = lds_f32(a8 >> 1);
  const f32x2_t rr = {r, r}, zero = {0.0f, 0.0f};
  return rnd2<FKS_BF16>(__builtin_elementwise_fma(rr, lds_f32x2(kLdsCsOff + b8), zero));
}

// fks_small2_kernel<DT, MODE>: passes of <= kSmallK seeds over fast segments (the ZO
// step's perturb / restore + update / K=1 update, optimizer.py:152-173, :146-148).
// 3 pair waves + 1 twist wave per chunk.  Pair lane q < 156 owns TWO Box-Muller pairs of
// every block, (j, j+8) and (j+1, j+9) with j = 16 (q/4) + 2 (q%4):
//   * the four raw words are adjacent in the permuted window (wperm): one ds_read_b128
//     per seed;
//   * the four parameters are two aligned element pairs (j, j+1) and (j+8, j+9): two
//     dword (bf16) / dwordx2 (f32) accesses, no exchange between lanes.
// The twist wave twists every window of block b+1 out of place while the pair waves
// run block b (double-buffered windows, one barrier per block).  Window k of buffer B
// sits at window slot 2k + B and the loops are unrolled by two blocks, so every LDS
// offset of a block is an immediate.
// Segment walk: a block lying inside one segment (all but a few hundred blocks of a
// model) is addressed from a WAVE-UNIFORM base (scalar registers: segment cursor, block
// range, base address and the segment's scalars) plus the lane's fixed byte offset, so
// it costs no vector instruction; a block that straddles segments or a gap takes a
// per-lane path (segment scan, no prefetch).  Lanes q >= 156 mirror lane 155 (same
// loads, same values stored to the same addresses).
constexpr int kSm2Threads = 256;
constexpr int kSm2PairLanes = kMtN / 4;  // 156
constexpr int kSm2TwistWave = 3;

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
  return (uint64_t)rfl((uint32_t)v) | ((uint64_t)rfl((uint32_t)(v >> 32)) << 32);
}
__device__ __forceinline__ float rflf(float v) { return __uint_as_float(rfl(__float_as_uint(v))); }

// ZM 1 (bf16, one seed): also store every block's table indices, one u32 per pair lane
// (bytes a_j, b_j, a_j+1, b_j+1: 1 B per parameter) at zidx[(block - zlo) * 156 + q],
// for fks_zreplay_kernel to replay (the ZO step's second and third calls).  (A replay
// through this kernel's own structure -- ZM 2, 3 waves, no twist -- streamed at 3.8
// TB/s against 5.6 for the flat kernel: profiles/r02_smallk_ab.log.)
constexpr int kZidxPerBlock = kSm2ZidxPerBlock;  // u32 per block
static_assert(kSm2ZidxPerBlock == kSm2PairLanes, "one z-index word per pair lane");
template <int DT, int MODE, int ZM = 0>
__global__ __launch_bounds__(kSm2Threads, kSm2MinWaves) void fks_small2_kernel(ApplyArgs a) {
  static_assert(ZM == 0 || (ZM == 1 && DT == FKS_BF16), "z-index store: bf16");
  extern __shared__ __attribute__((aligned(16))) uint32_t lds32[];
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds32);
  if ((uint32_t)(size_t)(lds_u32_t*)lds32 != 0u) __builtin_trap();
  const int tid = threadIdx.x;
  const int c = blockIdx.x;
  const int nseeds = a.nseeds;
  const int64_t b0 = a.chunk_block[c];
  const int nblk = (int)(a.chunk_block[c + 1] - b0);  // host: a chunk is far below 2^31 blocks

  if constexpr (DT == FKS_BF16) {
    for (int i = tid; i < 256; i += (int)blockDim.x) {
      reinterpret_cast<float*>(lds)[i] = c_tab_bf16[i];
      reinterpret_cast<float2*>(lds + kLdsCsOff)[i] = make_float2(c_tab_bf16[256 + i], c_tab_bf16[512 + i]);
    }
  } else if constexpr (DT == kDtF32Libm) {
    logf_tab_fill(0u, tid, kSm2Threads);
  }
  // the chunk-start windows go to buffer 1, twisted into buffer 0 for block b0
  for (int idx = tid; idx < nseeds * kMtN; idx += kSm2Threads) {
    const int k = idx / kMtN, i = idx - k * kMtN;
    lds_st(kLdsTabBytes + (2 * k + 1) * kWinBytes + 4 * wperm(i), a.states[((size_t)k * a.nchunks + c) * kMtN + i]);
  }
  TwistPlan plan;
  twist_plan(plan, tid, kLdsTabBytes);
  // (rotating the twist role across the workgroups' waves, so that twist waves do not
  // share a SIMD, measured no different: profiles/r02_smallk_ab.log)
  const int vw = plan.wave;
  __syncthreads();
  if (vw == kSm2TwistWave) {
    auto twist_into = [&](auto dst_c) __attribute__((always_inline)) {
      constexpr int D = decltype(dst_c)::value;
#pragma unroll
      for (int k = 0; k < kSmallK; k++)
        if (k < nseeds) twist_oop_reg(plan, (2 * k + 1 - D) * kWinBytes, (2 * k + D) * kWinBytes);
    };
    if (nblk > 0) twist_into(std::integral_constant<int, 0>{});
    __syncthreads();
    for (int t = 0; t < nblk; t += 2) {
      if (t + 1 < nblk) twist_into(std::integral_constant<int, 1>{});
      __syncthreads();  // block t+1 is in buffer 1; block t's buffer 0 is free
      if (t + 1 >= nblk) break;
      if (t + 2 < nblk) twist_into(std::integral_constant<int, 0>{});
      __syncthreads();
    }
    return;
  }
  __syncthreads();  // block b0 is in buffer 0

  const int vt = 64 * vw + (tid & 63);
  const int q = vt < kSm2PairLanes ? vt : kSm2PairLanes - 1;
  const int j = 16 * (q >> 2) + 2 * (q & 3);
  const uint32_t st_off = kLdsTabBytes + 4 * wperm(j);  // words (j, j+8, j+1, j+9), 16-byte aligned
  float gk[kSmallK];
#pragma unroll
  for (int k = 0; k < kSmallK; k++) gk[k] = rflf(k < nseeds ? a.g[k] : 0.0f);
  bool upd = true;  // a device-side perturb_step: g and the apply decision from device memory
  if (MODE == kModePerturbUpdate && a.gdev) {
    gk[0] = dev_value_g<DT>(a.gdev);
    upd = dev_value_apply(a.gdev);
  }

  using ST = Traits<MODE == kModeDelta ? FKS_F32 : DT>;
  constexpr int kEs = (is_f32(DT) || MODE == kModeDelta) ? 4 : 2;
  constexpr uint32_t kBlockBytes = kMtN * kEs;
  typedef typename ST::Pair Pair;
  const uint32_t joff = (uint32_t)j * kEs;

  // wave-uniform segment cursor; block t of the chunk (t relative to b0) is fast when
  // t in [fb, eb): it starts at or after the segment's start and ends within it
  int cur = 0;
  {
    const int64_t s0 = (int64_t)kMtN * b0;
    int lo = 0, hi = a.nsegs;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      const DevSeg& sm = a.segs[mid];
      if ((int64_t)rfl64((uint64_t)(sm.start + sm.numel)) <= s0) lo = mid + 1; else hi = mid;
    }
    cur = lo;
  }
  int fb = 0, eb = 0, nb = 0;
  uint64_t base0 = 0;
  float u_lr = 0.0f, u_wd = 0.0f, u_ps = 0.0f;
  bool u_wdf = false;
  auto load_seg = [&]() __attribute__((always_inline)) {
    if (cur < a.nsegs) {
      const DevSeg& sg = a.segs[cur];
      const int64_t st = (int64_t)rfl64((uint64_t)sg.start);
      const int64_t en = st + (int64_t)rfl64((uint64_t)sg.numel);
      const int64_t lim = (int64_t)nblk + 1;
      auto rel = [&](int64_t blk) __attribute__((always_inline)) -> int { const int64_t r = blk - b0; return (int)(r < -1 ? -1 : (r > lim ? lim : r)); };
      fb = rel((st + kMtN - 1) / kMtN);
      eb = rel(en / kMtN);
      nb = rel((en + kMtN - 1) / kMtN);
      base0 = rfl64(sg.ptr) + (uint64_t)((int64_t)kMtN * b0 - st) * kEs;
      u_lr = rflf(sg.lr);
      u_wd = rflf(sg.wd);
      u_ps = rflf(sg.ps);
      u_wdf = (rfl(sg.flags) & FKS_HAS_WD) != 0;
    } else {
      fb = eb = 0;
      nb = INT32_MAX;
    }
  };
  load_seg();

  // (cur at fetch time: the first segment ending after block t's start, where a
  // straddling block's lanes start their scan; fetching block t+1 may move cur on)
  struct Slot { uint64_t base; int cur; bool fast; Pair r0, r1; };
  auto fetch = [&](int t) __attribute__((always_inline)) -> Slot {
    Slot sl;
    while (t >= nb) { cur++; load_seg(); }
    sl.cur = cur;
    sl.fast = t >= fb && t < eb;
    // a block that is not fast prefetches from the sink (4 KB, any lane's offset fits):
    // the loads stay unconditional, so no register is reset under a pending load
    sl.base = sl.fast ? base0 + (uint64_t)(uint32_t)t * kBlockBytes : (uint64_t)(uintptr_t)a.sink;
    if (MODE != kModeWriteZ) {
      sl.r0 = ST::load_pair(sl.base + joff);
      sl.r1 = ST::load_pair(sl.base + joff + 8 * kEs);
    } else {
      sl.r0 = 0;
      sl.r1 = 0;
    }
    return sl;
  };

  // the block's four parameters through every seed of the pass, in seed order
  // ZM 1: the block's seed-0 table offsets, computed once per block for every lane
  u32x2_t zab = {0u, 0u}, zcd = {0u, 0u};
  auto run = [&](auto buf_c, Pair& r0, Pair& r1, float lr, float wd, bool wdf, float ps) __attribute__((always_inline)) {
    constexpr int B = decltype(buf_c)::value;
    // pA = (p_j, p_j+8), pB = (p_j+1, p_j+9): the two Box-Muller pairs' parameters
    f32x2_t pA = {ST::cvt(ST::lo(r0)), ST::cvt(ST::lo(r1))};
    f32x2_t pB = {ST::cvt(ST::hi(r0)), ST::cvt(ST::hi(r1))};
#pragma unroll
    for (int k = 0; k < kSmallK; k++) {
      if (k < nseeds) {  // wave-uniform
        f32x2_t zA, zB;
        if (ZM == 1 && k == 0) {
          zA = z_bf16_idx8(zab.x, zab.y);
          zB = z_bf16_idx8(zcd.x, zcd.y);
        } else {
          const u32x4_t w = lds_u4(st_off + (uint32_t)((2 * k + B) * kWinBytes));
          zA = z_pair2<DT>(lds, w.x, w.y);
          zB = z_pair2<DT>(lds, w.z, w.w);
        }
        pA = apply_pair<DT, MODE>(pA, zA, gk[k], lr, wd, wdf, ps, upd);
        pB = apply_pair<DT, MODE>(pB, zB, gk[k], lr, wd, wdf, ps, upd);
      }
    }
    if constexpr (sizeof(Pair) == 4) {  // bf16: the high halves of the bf16-exact results
      r0 = __builtin_amdgcn_perm(__float_as_uint(pB.x), __float_as_uint(pA.x), 0x07060302u);
      r1 = __builtin_amdgcn_perm(__float_as_uint(pB.y), __float_as_uint(pA.y), 0x07060302u);
    } else {
      r0 = ST::pack(ST::bits(pA.x), ST::bits(pB.x));
      r1 = ST::pack(ST::bits(pA.y), ST::bits(pB.y));
    }
  };

  auto block = [&](auto buf_c, Slot& sl, int t) __attribute__((always_inline)) {
    if constexpr (ZM == 1) {
      constexpr int B = decltype(buf_c)::value;
      const u32x4_t w = lds_u4(st_off + (uint32_t)(B * kWinBytes));
      u32x2_t w0, w1;
      w0.x = w.x;
      w0.y = w.y;
      w1.x = w.z;
      w1.y = w.w;
      zab = temper_pair_u8x8(w0);
      zcd = temper_pair_u8x8(w1);
      a.zidx[((size_t)(b0 + t - a.zlo)) * kZidxPerBlock + q] =
          (zab.x >> 3) | (zab.y << 5) | (zcd.x << 13) | (zcd.y << 21);
    }
    {
      if (sl.fast) {
        run(buf_c, sl.r0, sl.r1, u_lr, u_wd, u_wdf, u_ps);
        ST::store_pair(sl.base + joff, sl.r0);
        ST::store_pair(sl.base + joff + 8 * kEs, sl.r1);
      } else {
        // straddling block: each lane finds its own segment from the cursor on
        const int64_t s1 = (int64_t)kMtN * (b0 + t) + j;
        int cc = sl.cur;
        bool in = false;
        DevSeg sg;
        while (cc < a.nsegs) {
          sg = a.segs[cc];
          if (s1 < sg.start + sg.numel) { in = s1 >= sg.start; break; }
          cc++;
        }
        if (in) {
          const uint64_t addr = sg.ptr + (uint64_t)(s1 - sg.start) * kEs;
          Pair r0 = 0, r1 = 0;
          if (MODE != kModeWriteZ) {
            r0 = ST::load_pair(addr);
            r1 = ST::load_pair(addr + 8 * kEs);
          }
          run(buf_c, r0, r1, sg.lr, sg.wd, (sg.flags & FKS_HAS_WD) != 0, sg.ps);
          ST::store_pair(addr, r0);
          ST::store_pair(addr + 8 * kEs, r1);
        }
      }
    }
    __syncthreads();  // the twist wave has block t+1 in place
  };

  // (fetching two blocks ahead measured slower: profiles/r02_smallk_ab.log)
  Slot s0 = fetch(0);
  // a store after the first prefetch, so the loop is entered with the same pending
  // (load, store) shape as the back edge
  *reinterpret_cast<volatile uint32_t*>(a.sink + 1) = 0u;
  for (int t = 0; t < nblk; t += 2) {
    Slot s1 = fetch(t + 1 < nblk ? t + 1 : t);  // (the last block re-reads itself, unused)
    block(std::integral_constant<int, 0>{}, s0, t);
    if (t + 1 >= nblk) break;
    s0 = fetch(t + 2 < nblk ? t + 2 : t + 1);
    block(std::integral_constant<int, 1>{}, s1, t + 1);
  }
}

// ------------------------------------------------------------------ z-index replay
// fks_zreplay_kernel<MODE>: a one-seed bf16 pass whose z comes from the table indices a
// fks_small2_kernel<.., ZM 1> pass stored for the same seed (ZCache): no generator, no
// windows, no barriers -- a streaming pass.  Each thread takes 8 consecutive stream
// positions (half a 16-block: 16 B of parameters, one dwordx4 load and store; a wave
// covers 1 KB contiguously) and the 16-block's index record (16 B: a_i, b_i for its 8
// Box-Muller pairs, at the record's stream offset: 1 byte per position), which both
// halves of the 16-block read.  The first half takes z_i = R[a_i] C[b_i], the second
// z_{i+8} = R[a_i] S[b_i] (DistributionTemplates.h:141-146), each rounded once as
// z_pair_bf16_raw; then the update chain of apply_pair, element pairs (i, i+1).
// Workgroup c walks the stream positions of chunk c in tiles of 256 x 8; a tile inside
// one segment is addressed from a wave-uniform base, a straddling tile per lane.
constexpr int kZrThreads = 256;
typedef __attribute__((address_space(1))) u32x4_t gu32x4_t;
__device__ __forceinline__ u32x4_t gload4(uint64_t addr) { return *reinterpret_cast<const gu32x4_t*>(addr); }
__device__ __forceinline__ void gstore4(uint64_t addr, u32x4_t v) { *reinterpret_cast<gu32x4_t*>(addr) = v; }
constexpr int kZrTile = kZrThreads * 8;  // stream positions per tile

template <int MODE>
__global__ __launch_bounds__(kZrThreads) void fks_zreplay_kernel(ApplyArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds32[];
  if ((uint32_t)(size_t)(lds_u32_t*)lds32 != 0u) __builtin_trap();
  const int tid = threadIdx.x;
  const int c = blockIdx.x;
  // R | C | S as three f32[256]: one b32 lookup per table
  for (int i = tid; i < 256; i += kZrThreads) {
    reinterpret_cast<float*>(lds32)[i] = c_tab_bf16[i];
    reinterpret_cast<float*>(lds32)[256 + i] = c_tab_bf16[256 + i];
    reinterpret_cast<float*>(lds32)[512 + i] = c_tab_bf16[512 + i];
  }
  __syncthreads();
  // tiles of the whole call are dealt round-robin over the workgroups, so the workgroups
  // in flight stream neighbouring addresses (few pages live at a time, as a grid-stride
  // elementwise kernel; one chunk per workgroup measured slower)
  const int64_t p0 = (int64_t)kMtN * a.chunk_block[0] + (int64_t)c * kZrTile;
  const int64_t p1 = (int64_t)kMtN * a.chunk_block[a.nchunks];
  const int64_t tstep = (int64_t)gridDim.x * kZrTile;
  const int64_t zbase = (int64_t)kMtN * a.zlo;
  const uint64_t zb = (uint64_t)(uintptr_t)a.zidx;
  float g = rflf(a.g[0]);
  bool upd = true;
  if (MODE == kModePerturbUpdate && a.gdev) {
    g = dev_value_g<FKS_BF16>(a.gdev);
    upd = dev_value_apply(a.gdev);
  }
  const uint32_t half = (uint32_t)tid & 1u;  // 0: first half of the 16-block (cos), 1: second (sin)
  const uint32_t cs_tab = half ? 2048u : 1024u;

  int cur = 0;
  {
    int lo = 0, hi = a.nsegs;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      const DevSeg& sm = a.segs[mid];
      if ((int64_t)rfl64((uint64_t)(sm.start + sm.numel)) <= p0) lo = mid + 1; else hi = mid;
    }
    cur = lo;
  }
  // the 8 elements e[0..7] through the seed; z from the record's bytes
  auto chain = [&](u32x4_t pv, u32x4_t rec, float lr, float wd, bool wdf, float ps) __attribute__((always_inline)) -> u32x4_t {
    const uint32_t w[4] = {pv.x, pv.y, pv.z, pv.w};
    const uint32_t r[4] = {rec.x, rec.y, rec.z, rec.w};
    uint32_t o[4];
#pragma unroll
    for (int m = 0; m < 4; m++) {  // elements 2m, 2m+1: pairs 2m (bytes 0,1 of r[m]) and 2m+1 (bytes 2,3)
      const uint32_t ri = r[m];
      const float ra = lds_f32((ri << 2) & 0x3FCu), rb = lds_f32((ri >> 14) & 0x3FCu);
      const float ca = lds_f32(cs_tab + ((ri >> 6) & 0x3FCu)), cb = lds_f32(cs_tab + ((ri >> 22) & 0x3FCu));
      const f32x2_t rr = {ra, rb}, cc = {ca, cb}, zero = {0.0f, 0.0f};
      const f32x2_t z = rnd2<FKS_BF16>(__builtin_elementwise_fma(rr, cc, zero));
      f32x2_t pe = {__uint_as_float(w[m] << 16), __uint_as_float(w[m] & 0xffff0000u)};
      pe = apply_pair<FKS_BF16, MODE>(pe, z, g, lr, wd, wdf, ps, upd);
      o[m] = __builtin_amdgcn_perm(__float_as_uint(pe.y), __float_as_uint(pe.x), 0x07060302u);
    }
    const u32x4_t out = {o[0], o[1], o[2], o[3]};
    return out;
  };
  const u32x4_t zero4 = {0u, 0u, 0u, 0u};
  // kZrUnroll tiles per iteration: every tile's index records and parameters are
  // loaded before the first is computed, so a wave keeps that many tiles in flight (a
  // straddling tile loads its parameters when it runs)
  struct ZSlot { int64_t t0; uint64_t base; float lr, wd, ps; int cur; bool fast, wdf; u32x4_t rec, pv; };
  // the current segment's scalars, re-read only when the walk moves on (a global load
  // here would wait for every load in flight, the prefetched tile's included)
  int64_t seg_st = INT64_MAX, seg_en = INT64_MAX;
  uint64_t seg_ptr = 0;
  float seg_lr = 0.0f, seg_wd = 0.0f, seg_ps = 0.0f;
  bool seg_wdf = false;
  auto load_seg = [&]() __attribute__((always_inline)) {
    if (cur < a.nsegs) {
      const DevSeg& sg = a.segs[cur];
      seg_st = (int64_t)rfl64((uint64_t)sg.start);
      seg_en = seg_st + (int64_t)rfl64((uint64_t)sg.numel);
      seg_ptr = rfl64(sg.ptr);
      seg_lr = rflf(sg.lr);
      seg_wd = rflf(sg.wd);
      seg_ps = rflf(sg.ps);
      seg_wdf = (rfl(sg.flags) & FKS_HAS_WD) != 0;
    } else {
      seg_st = seg_en = INT64_MAX;
    }
  };
  load_seg();
  auto zfetch = [&](int64_t t0) __attribute__((always_inline)) -> ZSlot {
    ZSlot z;
    z.t0 = t0;
    while (seg_en <= t0) {  // wave-uniform: the first segment ending after the tile's start
      cur++;
      load_seg();
    }
    z.cur = cur;
    const int64_t tend = t0 + kZrTile < p1 ? t0 + kZrTile : p1;
    z.fast = seg_st <= t0 && tend <= seg_en;
    z.base = seg_ptr + (uint64_t)(t0 - seg_st) * 2u;
    z.lr = seg_lr;
    z.wd = seg_wd;
    z.ps = seg_ps;
    z.wdf = seg_wdf;
    const int64_t pos = t0 + 8 * (int64_t)tid;
    const bool live = pos < p1;  // (lanes past the chunk's end load lane 0's addresses)
    z.rec = zero4;
    z.pv = zero4;
    if (t0 < p1) {  // wave-uniform
      z.rec = gload4(zb + (uint64_t)(((live ? pos : t0) - zbase) & ~(int64_t)15));
      if (MODE != kModeWriteZ && z.fast) z.pv = gload4(z.base + (live ? 16u * (uint32_t)tid : 0u));
    }
    return z;
  };
  auto zblock = [&](ZSlot& z) __attribute__((always_inline)) {
    const int64_t pos = z.t0 + 8 * (int64_t)tid;
    if (pos >= p1) return;
    if (z.fast) {
      gstore4(z.base + 16u * (uint32_t)tid, chain(z.pv, z.rec, z.lr, z.wd, z.wdf, z.ps));
    } else {
      int cc = z.cur;
      bool in = false;
      DevSeg sg;
      while (cc < a.nsegs) {
        sg = a.segs[cc];
        if (pos < sg.start + sg.numel) { in = pos >= sg.start; break; }
        cc++;
      }
      if (in) {
        const uint64_t ptr = sg.ptr + (uint64_t)(pos - sg.start) * 2u;
        const u32x4_t pv = MODE == kModeWriteZ ? zero4 : gload4(ptr);
        gstore4(ptr, chain(pv, z.rec, sg.lr, sg.wd, (sg.flags & FKS_HAS_WD) != 0, sg.ps));
      }
    }
  };
  constexpr int kU = kZrUnroll;
  for (int64_t t0 = p0; t0 < p1; t0 += kU * tstep) {
    ZSlot z[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) z[u] = zfetch(t0 + u * tstep);
#pragma unroll
    for (int u = 0; u < kU; u++) zblock(z[u]);
  }
}

// ------------------------------------------------------------------ bf16 slice kernel
// fks_apply_bs_kernel<MODE>: the bf16 fast segments of a reconstruct, 64 seeds per pass
// as two SLICES of 32, generator state BIT-SLICED (fks_bitslice.h): row i of a slice's
// state is state word i of its 32 seeds as 32 bit planes.  One workgroup per CU takes one
// chunk and holds both slices' states in LDS, one per half.  The work of a chunk is cut
// into TASKS of 128 consecutive stream words (64 Box-Muller pairs: one wave), and the six
// waves of a half take the half's tasks round-robin.  A wave runs the whole of its task:
//   * twist: lane L owns the pair (j, j+8), j = 16 (L >> 3) + (L & 7) of the task, and
//     twists exactly those two rows in place, block b -> b+1 (MT19937RNGEngine.h:164-175
//     on 32 seeds at once): word u of the stream is f(word u-624 (plane 31 only: U31),
//     word u-623 (V, the next slot), word u-227 (M));
//   * the two new rows are still in registers: temper their low bytes (temper_low8),
//     transpose them to one byte per seed, and run the 32-seed update chain of the lane's
//     two parameters (thread owns Box-Muller pair (j, j+8): two table lookups, the z
//     product and its rounding, the per-op-rounded update chain).
// The twists of a half form one serial chain -- M of a task's last 29 words are words the
// previous task wrote -- so a wave waits until the half's LDS flag counts n twisted
// tasks, twists task n, and publishes n+1; the chains of different tasks overlap freely.
// Half 1 applies its seeds to what half 0 stored: its wave for task n waits until the
// half-0 wave of task n+6 has published that store as complete before it prefetches
// task n+6's parameters (half 0 publishes task m at its task m+6, after s_waitcnt
// vmcnt(0): workgroup-scope release; half 0 never waits for half 1).  Two slices per
// workgroup instead of two chunks halve the jumps (one per seed and chunk) and the HBM
// passes of a reconstruct.
// Against the round-2 form (five pair waves + one twist wave per half, two workgroup
// barriers per MT block): no pair wave re-reads the rows the twist wave wrote (a quarter
// of the LDS traffic), every wave carries the same instruction mix (no SIMD with three
// pair waves beside one with the twist wave), no barrier per block; with that LDS time
// freed, the (C,S) table is read as f32 pairs (one ds_read_b64, no unpack instructions):
// 3.83 -> 3.39 ms per 32-seed launch over 2^28 params (profiles/r03s_ab.log; the
// variants measured on the way are in profiles/r03k..r03s_ab.log).
// LDS: [R f32 x 256 | (C,S) f32 pairs x 256 | state half 0 | state half 1 | 2 twist flags |
// 6 half-0 progress words]; a
// half's state is 8 CHUNK arrays (planes 4q..4q+3 of all 624 rows, 16 B per row), so a
// row's chunk q is one ds_read_b128 / ds_write_b128.  The lane's first row is j+8 where
// (L >> 3) is odd, which makes every 16-lane group of a ds_read_b128 (8-lane group of a
// ds_write_b128) touch distinct rows mod 16: conflict free.
constexpr int kBsChunkBytes = kMtN * 16;               // 9,984
constexpr int kBsStateBytes = 8 * kBsChunkBytes;       // 79,872
constexpr int kBsTabBytes = 256 * 4 + 256 * 8;         // 3,072
constexpr uint32_t kBsFlagOff = kBsTabBytes + 2 * kBsStateBytes;  // u32 twisted-task count per half
constexpr uint32_t kBsProgOff = kBsFlagOff + 8;        // u32 per half-0 wave: its tasks < value are stored
constexpr uint32_t kBsProg1Off = kBsProgOff + 4 * 6;   // u32 per half-1 wave: its tasks < value are done
constexpr int kBsLdsBytes = (int)kBsProg1Off + 4 * 6;  // 162,872 <= 163,840
static_assert(kBsLdsBytes <= 163840, "slice kernel LDS");
constexpr int kBsWaves = kBsHalfThreads / 64;          // waves per half (6)
constexpr int kBsTaskWords = 128;                      // stream words per task

// the 32 planes of row i (row byte address ra = state base + 16 i)
__device__ __forceinline__ void bs_store_row(uint32_t ra, const uint32_t (&x)[32]) {
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const u32x4_t v = {x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]};
    lds_st4(ra + q * kBsChunkBytes, v);
  }
}

// The flag hand-off needs no memory fence: one wave's LDS operations are performed in
// order, so a wave that reads the new count issues its row loads after the writer's row
// stores were performed.  (A release fence would also wait for the writer's global
// stores.)  The lgkmcnt(0) keeps the count from running ahead of stores still queued;
// the asm barriers keep the compiler from moving LDS accesses across.
__device__ __forceinline__ uint32_t bs_flag_load(uint32_t off) {
  return *(volatile const lds_u32_t*)(size_t)off;
}
__device__ __forceinline__ void bs_flag_store(uint32_t off, uint32_t v) {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  *(volatile lds_u32_t*)(size_t)off = v;
}

// byte c of w times 2^S with a compile-time c (SDWA)
template <int S>
__device__ __forceinline__ uint32_t bs_index(uint32_t w, int c) {
  switch (c) {
    case 0: return bs::byte_x<0, S>(w);
    case 1: return bs::byte_x<1, S>(w);
    case 2: return bs::byte_x<2, S>(w);
    default: return bs::byte_x<3, S>(w);
  }
}

#if FKS_BS_WGTIME  // diagnostic build: per-workgroup start and per-wave end times (100 MHz)
__device__ uint64_t g_bs_wgtime[4096][16];
extern "C" int fks_debug_bs_wgtime(uint64_t* out, int nblocks) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bs_wgtime), sizeof(uint64_t) * 16 * (size_t)nblocks, 0,
                                  hipMemcpyDeviceToHost);
}
#endif

template <int MODE, bool FULL>
__global__ __launch_bounds__(kBsThreads, 1) void fks_apply_bs_kernel(ApplyBsArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds32[];
  if ((uint32_t)(size_t)(lds_u32_t*)lds32 != 0u) __builtin_trap();
  const int tid = threadIdx.x;
  const int lane = tid & 63;
#if FKS_BS_WGTIME
  if (tid == 0) g_bs_wgtime[blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();
  auto stamp = [&]() { if (lane == 0) g_bs_wgtime[blockIdx.x][1 + (tid >> 6)] = __builtin_amdgcn_s_memrealtime(); };
#else
  auto stamp = [&]() {};
#endif
  const int half = __builtin_amdgcn_readfirstlane(tid >= kBsHalfThreads ? 1 : 0);
  const int ht = tid - half * kBsHalfThreads;
  const int hw = __builtin_amdgcn_readfirstlane(ht >> 6);
  // slices (a pass of 33..64 seeds): both halves on plan chunks 2w, 2w+1, slice 0 with
  // seeds [0, nA), slice 1 with [nA, nseeds) applied after slice 0's; split (<= 32 seeds):
  // half h alone on plan chunk 2w+h with every seed
  const bool split = a.split != 0;  // FULL: 32 seeds in each half either way
  const int c = split ? 2 * (int)blockIdx.x + half : (int)blockIdx.x;  // index into the states
  const int nA = FULL ? kBsSeeds : split ? a.nseeds : (a.nseeds + 1) / 2;
  const int nseeds = FULL ? kBsSeeds : (half && !split ? a.nseeds - nA : nA);  // this half's seeds
  const int sfirst = half && !split ? nA : 0;
  const int64_t b0 = a.chunk_block[split ? c : 2 * c], b1 = a.chunk_block[split ? c + 1 : 2 * c + 2];
  const int nwords = (int)(kMtN * (b1 - b0));  // < 2^31 (the host's plan keeps chunks shorter)
  const int ntask = (nwords + kBsTaskWords - 1) / kBsTaskWords;
  const uint32_t sbase = kBsTabBytes + (uint32_t)half * kBsStateBytes;
  const uint32_t flag = kBsFlagOff + 4u * (uint32_t)half;

  for (int i = tid; i < 256; i += kBsThreads) {
    reinterpret_cast<float*>((uint8_t*)lds32)[i] = c_tab_bf16[i];
    reinterpret_cast<float2*>((uint8_t*)lds32 + 1024)[i] = make_float2(c_tab_bf16[256 + i], c_tab_bf16[512 + i]);
  }
  // prologue: the jump windows of this chunk (the state before block b0), as planes
  for (int i = ht; i < kMtN; i += kBsHalfThreads) {
    uint32_t w[32];
#pragma unroll
    for (int k = 0; k < 32; k++)
      w[k] = k < nseeds ? a.states[((size_t)(a.use_slot ? a.slot[sfirst + k] : (uint32_t)(sfirst + k)) * a.nchunks + c) *
                                       kMtN + i]
                        : 0u;
    bs::transpose32(w);
    bs_store_row(sbase + 16u * (uint32_t)i, w);
  }
  if (ht == 0) lds32[flag / 4] = 0u;
  if (ht < kBsWaves) lds32[(half ? kBsProg1Off : kBsProgOff) / 4 + ht] = 0u;
  __syncthreads();  // the only workgroup barrier
  if (nseeds == 0) return;  // a one-seed pass: slice 1 is empty

  const int toff = 16 * (lane >> 3) + (lane & 7);  // the lane's words toff, toff + 8 of a task
  const bool flip = ((lane >> 3) & 1) != 0;
  const bool odd = (lane & 1) != 0;

  float gk[kBsSeeds];
#pragma unroll
  for (int k = 0; k < kBsSeeds; k++) gk[k] = a.g[half ? k + sfirst : k];

  // the lane's current segment (positions only grow)
  const int64_t wbase = (int64_t)kMtN * b0;  // stream position of the chunk's first word
  int cur;
  {
    const int64_t s1 = wbase + (int64_t)kBsTaskWords * hw + toff;
    int lo = 0, hi = a.nsegs;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (a.segs[mid].start + a.segs[mid].numel <= s1) lo = mid + 1; else hi = mid;
    }
    cur = lo;
  }
  int64_t seg_start = INT64_MAX, seg_end = INT64_MAX;
  uint64_t seg_ptr = 0;
  float seg_lr = 0.0f, seg_wd = 0.0f;
  bool seg_wdf = false;
  auto load_seg = [&]() {
    if (cur < a.nsegs) {
      const DevSeg sg = a.segs[cur];
      seg_start = sg.start;
      seg_end = sg.start + sg.numel;
      seg_ptr = sg.ptr;
      seg_lr = sg.lr;
      seg_wd = sg.wd;
      seg_wdf = (sg.flags & FKS_HAS_WD) != 0;
    } else {
      seg_start = seg_end = INT64_MAX;
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): see fks_apply_kernel
  };
  load_seg();

  // The lane's parameters of task n: elements toff, toff + 8 of the task, loaded as the
  // aligned pairs (j, j+1) (even lane j) and (j+7, j+8) (odd lane j+1) and exchanged with
  // the neighbour lane (swap_adjacent).  Lanes past the chunk or off every fast segment
  // read and write the sink.
  using ST = Traits<MODE == kModeDelta ? FKS_F32 : FKS_BF16>;
  constexpr int kEs = MODE == kModeDelta ? 4 : 2;
  typedef typename ST::Pair Pair;
  struct Slot { uint64_t addr; float lr, wd; uint32_t wdf; Pair raw; };
  auto fetch = [&](int n) -> Slot {
    Slot sl;
    const int u1 = kBsTaskWords * n + toff;
    const int64_t s1 = wbase + u1;
    while (s1 >= seg_end) { cur++; load_seg(); }
    const bool on = u1 < nwords && s1 >= seg_start;
    sl.lr = seg_lr; sl.wd = seg_wd; sl.wdf = seg_wdf;
    sl.addr = on ? seg_ptr + (uint64_t)(s1 - seg_start + (odd ? 7 : 0)) * kEs : (uint64_t)(uintptr_t)a.sink;
    sl.raw = ST::load_pair(sl.addr);
    return sl;
  };

  // ---- the twist of task n: the lane's two rows in place; returns the tempered radius
  // bytes (row toff) and angle bytes (row toff + 8) as planes.  Streamed over the 8 chunk
  // arrays (planes 4q..4q+3): chunk q of every row of the task is loaded (V, M) before
  // any lane stores it -- through data dependence, since new plane 4q+3 needs V plane
  // 4q+4 of chunk q+1, loaded one step ahead; U31 and V plane 0 are loaded first.  M
  // rows lie 227 words back, outside the task, so the task never stores them.
  auto twist = [&](const int n, uint32_t (&oa)[8], uint32_t (&ob)[8]) {
    const int u1 = kBsTaskWords * n + toff;
    const bool valid = u1 < nwords;
    const int i1 = valid ? u1 % kMtN : 0;
    const int ia = flip ? i1 + 8 : i1, ib = flip ? i1 : i1 + 8;  // first / second row
    auto rows = [&](int i, uint32_t& av, uint32_t& am, uint32_t& au) {
      const int iv = i + 1 < kMtN ? i + 1 : 0;
      const int im = i < kMtN - kMtM ? i + kMtM : i - (kMtN - kMtM);
      av = sbase + 16u * (uint32_t)iv;
      am = sbase + 16u * (uint32_t)im;
      au = sbase + 7u * kBsChunkBytes + 16u * (uint32_t)i + 12u;
    };
    uint32_t av1, am1, au1, av2, am2, au2;
    rows(ia, av1, am1, au1);
    rows(ib, av2, am2, au2);
    uint32_t M1[32], M2[32];  // the new rows
    const uint32_t U1 = lds_u32((int)au1), U2 = lds_u32((int)au2);
    // (issuing all 34 loads of the task at once -- 164 VGPRs -- measured 5 % slower per
    // pass: profiles/r03v_ab.log)
    // (loads two or three chunk arrays ahead measured no faster: profiles/r03x_ab.log)
    u32x4_t va = lds_u4(av1), vb = lds_u4(av2), ma = lds_u4(am1), mb = lds_u4(am2);
    const uint32_t v0a = va.x, v0b = vb.x;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      u32x4_t va2 = va, vb2 = vb, ma2 = ma, mb2 = mb;
      if (q < 7) {
        va2 = lds_u4(av1 + (q + 1) * kBsChunkBytes);
        vb2 = lds_u4(av2 + (q + 1) * kBsChunkBytes);
        ma2 = lds_u4(am1 + (q + 1) * kBsChunkBytes);
        mb2 = lds_u4(am2 + (q + 1) * kBsChunkBytes);
      }
      const uint32_t Va[5] = {va.x, va.y, va.z, va.w, va2.x};
      const uint32_t Vb[5] = {vb.x, vb.y, vb.z, vb.w, vb2.x};
      const uint32_t Ma[4] = {ma.x, ma.y, ma.z, ma.w}, Mb[4] = {mb.x, mb.y, mb.z, mb.w};
#pragma unroll
      for (int t = 0; t < 4; t++) {
        // bs::twist_row plane by plane: plane b of y >> 1 is V plane b+1 (b < 30; t = 3
        // reads chunk q+1's plane 0), U31 (b = 30), none (b = 31)
        const int b = 4 * q + t;
        const bool am = ((bs::kMatrixA >> b) & 1u) != 0;
        uint32_t xa, xb;
        if (b < 30) { xa = Va[t + 1]; xb = Vb[t + 1]; }
        else if (b == 30) { xa = U1; xb = U2; }
        else { xa = 0u; xb = 0u; }
        M1[b] = am ? bs::xor3(Ma[t], xa, v0a) : (Ma[t] ^ xa);
        M2[b] = am ? bs::xor3(Mb[t], xb, v0b) : (Mb[t] ^ xb);
      }
      if (valid) {
        lds_st4(sbase + 16u * (uint32_t)ia + q * kBsChunkBytes, u32x4_t{M1[4 * q], M1[4 * q + 1], M1[4 * q + 2], M1[4 * q + 3]});
        lds_st4(sbase + 16u * (uint32_t)ib + q * kBsChunkBytes, u32x4_t{M2[4 * q], M2[4 * q + 1], M2[4 * q + 2], M2[4 * q + 3]});
      }
      va = va2; vb = vb2; ma = ma2; mb = mb2;
    }
    uint32_t o1[8], o2[8];
    bs::temper_low8(M1, o1);
    bs::temper_low8(M2, o2);
#pragma unroll
    for (int j = 0; j < 8; j++) {
      oa[j] = flip ? o2[j] : o1[j];  // row toff: the radius uniforms
      ob[j] = flip ? o1[j] : o2[j];  // row toff + 8: the angle uniforms
    }
  };

  // ---- the 32-seed chain of the lane's two parameters (slot sl), z from the bytes of
  // twist(): z = bf16(R[a] C[b]) + 0, bf16(R[a] S[b]) + 0 (normal_fill_16<BFloat16>: an
  // exact f32 product, one rounding; the fma's +0 turns -0 into +0 like "+ mean")
  auto chain = [&](const Slot& sl, uint32_t (&oa)[8], uint32_t (&ob)[8]) {
    bs::transpose8(oa);
    bs::transpose8(ob);
    f32x2_t p;
    {
      const uint32_t keep = odd ? ST::hi(sl.raw) : ST::lo(sl.raw);
      const uint32_t got = swap_adjacent(odd ? ST::lo(sl.raw) : ST::hi(sl.raw));
      p.x = ST::cvt(odd ? got : keep);
      p.y = ST::cvt(odd ? keep : got);
    }
    auto z_of = [&](const int k) __attribute__((always_inline)) -> f32x2_t {
      // (R read through the vector-memory path instead, an L1-resident 1 KB table off the
      // LDS: 13 % slower, profiles/r04rg_r_global_ab.log)
      const float r = lds_f32(bs_index<2>(oa[k & 7], k >> 3));
      const f32x2_t rr = {r, r}, zero = {0.0f, 0.0f};
      const f32x2_t cs = lds_f32x2(1024u + bs_index<3>(ob[k & 7], k >> 3));
      return rnd2<FKS_BF16>(__builtin_elementwise_fma(rr, cs, zero));
    };
    // (issuing seed k+1's lookups, z and g z ahead of seed k's p-dependent tail, which
    // removes the wait state between the tail's dependent packed ops, measured 1 % slower:
    // profiles/r04d_pipe_ab.log; dropping the wd0 tail's fma -- t = gz for wd = +0 and a
    // finite p, with the chain redone exactly for the lanes that end non-finite -- issues one
    // packed op per element pair and seed fewer but measured 1.5 % slower, its lr*gz waiting
    // on gz's conversions: profiles/r04o_wd0_nofma_ab.log)
    {
#pragma unroll
      for (int k = 0; k < kBsSeeds; k++) {
        if (FULL || k < nseeds) p = apply_pair<FKS_BF16, MODE>(p, z_of(k), gk[k], sl.lr, sl.wd, sl.wdf != 0, 0.0f);
        // the lookups of one byte column (8 seeds) at a time: hoisting all 64 table reads
        // ahead of the chain would spill
        if ((k % kBsFence) == kBsFence - 1) asm volatile("" ::: "memory");
      }
    }
    const uint32_t b1v = ST::bits(p.x), b2v = ST::bits(p.y);
    const uint32_t back = swap_adjacent(odd ? b1v : b2v);
    const Pair out = odd ? ST::pack(back, b2v) : ST::pack(b1v, back);
    ST::store_pair(sl.addr, out);
  };

  const bool ordered = !split;  // half 1 depends on half 0's stores
  // ---- half 0 publishes its task m's parameters as stored (the wave's global stores
  // done: vmcnt(0), the workgroup-scope release); half 1 waits for that before loading them
  const uint32_t prog = kBsProgOff + 4u * (uint32_t)hw;
  auto publish_stored = [&](const int m) {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    if (lane == 0) *(volatile lds_u32_t*)(size_t)prog = (uint32_t)m + 1u;
  };
  auto await_stored = [&](const int m) {
    if (m >= ntask) return;
    const uint32_t pm = kBsProgOff + 4u * (uint32_t)(m % kBsWaves);
    while (__builtin_amdgcn_readfirstlane(bs_flag_load(pm)) < (uint32_t)m + 1u) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
  };
  // The lag bound.  Nothing else keeps half 0 from running ahead of half 1 (it wins the
  // VALU arbitration by age), and with the longer weight-decay chain half 1 fell so far
  // behind that its loads of half 0's output came back from HBM (7.9 B/param per launch,
  // profiles/pmc_apply_r04_full.json).  Half 1 publishes each task as applied; half 0 waits
  // for task n - FKS_BS_LAG before twisting task n.  Half 1's task m needs half 0's task
  // m + 2 kBsWaves (publish_stored), so the bound must exceed 2 kBsWaves = 12.
  static_assert(FKS_BS_LAG == 0 || FKS_BS_LAG > 2 * kBsWaves, "FKS_BS_LAG: half 1 trails by 12 tasks");
  // only the weight-decay chains need it: the wd 0 / None chains keep half 1 within L2 reach
  // unaided (4.17 B/param), and there the bound measured 1.4 % slower (profiles/r05d_ab_lag.log)
  constexpr bool kLag = FKS_BS_LAG > 0 && (MODE == kModeUpdateWd || MODE == kModeUpdate);
  const uint32_t prog1 = kBsProg1Off + 4u * (uint32_t)hw;
  auto publish_applied = [&](const int m) {
    if (lane == 0) *(volatile lds_u32_t*)(size_t)prog1 = (uint32_t)m + 1u;
  };
  auto await_applied = [&](const int m) {
    if (m < 0) return;
    const uint32_t pm = kBsProg1Off + 4u * (uint32_t)(m % kBsWaves);
    while (__builtin_amdgcn_readfirstlane(bs_flag_load(pm)) < (uint32_t)m + 1u) __builtin_amdgcn_s_sleep(1);
  };

  // ---- task n: wait for task n-1's twist, twist, publish, chain; fetches task n + 6
  // into nx (past the last task: the sink)
  auto task = [&](const int n, const Slot& sl, Slot& nx) {
    uint32_t oa[8], ob[8];
    if (kLag && ordered && half == 0) await_applied(n - FKS_BS_LAG);
    __builtin_amdgcn_s_setprio(2);
#if !FKS_BS_DIAG_NOWAIT  // diagnostic (wrong values): no hand-off wait, the resource bound
    while (__builtin_amdgcn_readfirstlane(bs_flag_load(flag)) < (uint32_t)n) __builtin_amdgcn_s_sleep(0);
#endif
    asm volatile("" ::: "memory");
    twist(n, oa, ob);
    if (lane == 0) bs_flag_store(flag, (uint32_t)n + 1u);
    __builtin_amdgcn_s_setprio(0);
    if (ordered && half == 0) {
      if (n >= kBsWaves) publish_stored(n - kBsWaves);  // the store of the wave's previous task
    } else if (ordered) {
      await_stored(n + kBsWaves);
    }
    nx = fetch(n + kBsWaves);
#if FKS_BS_DIAG_NOCHAIN  // diagnostic (wrong values): the twist and its hand-offs alone
    if (__builtin_amdgcn_readfirstlane(oa[0] ^ ob[0]) == 0x12345u) chain(sl, oa, ob);
#else
    chain(sl, oa, ob);
#endif
    if (kLag && ordered && half) publish_applied(n);
  };

  // two named slots and a loop unrolled by two: a slot copy on the back edge would wait
  // for the load -- and the store before it -- at the top of every task
  if (hw >= ntask) { stamp(); return; }
  if (ordered && half) await_stored(hw);
  Slot s0 = fetch(hw), s1;
  int n = hw;
  for (;;) {
    task(n, s0, s1);
    if (n + kBsWaves >= ntask) break;
    n += kBsWaves;
    task(n, s1, s0);
    if (n + kBsWaves >= ntask) break;
    n += kBsWaves;
  }
  if (ordered && half == 0) publish_stored(n);  // the wave's last task
  stamp();
}

// ------------------------------------------------------------------ irregular kernel
// Everything the fast kernel does not take (DESIGN.md "Irregular layouts"):
//   * runs of whole 16-blocks at any stream phase (a tensor after a ragged one, a
//     ragged tensor's head with its overwritten elements masked, its 16-word tail
//     recompute, f16 tensors, parameters not 2-element aligned), and
//   * single elements of numel < 16 tensors (serial normal_distribution<double>,
//     DistributionsHelper.h:189-221, with the cached second sample).
// A work item is handled in the MT block holding its LAST word; its first words may
// lie up to 15 words back, in the previous block, so every seed window carries the
// previous block's last 16 raw words in front of it: [carry 16 | 624].
__constant__ float c_tab_f16[3 * 2048];  // R | C | S of the 11-bit f16 uniforms

constexpr int kIrrCarry = 16;
constexpr int kIrrWin = kIrrCarry + kMtN;  // words per seed window

__device__ __forceinline__ uint32_t win_word(const uint32_t* win, int k, int w) {  // w in [-16, 624)
  return win[k * kIrrWin + kIrrCarry + w];
}

// in-place twist of every window, phase PH of 3 (i in [0,227) / [227,454) / [454,624));
// phase 0 also saves the old words 608..623 as the next block's carry
template <int PH>
__device__ __forceinline__ void irr_twist_phase(uint32_t* win, int nseeds, int tid) {
  constexpr int lo = PH == 0 ? 0 : (PH == 1 ? 227 : 454);
  constexpr int hi = PH == 0 ? 227 : (PH == 1 ? 454 : kMtN);
  constexpr int len = hi - lo;
  constexpr int per = (kMaxSeedsPerPass * len + kApplyThreads - 1) / kApplyThreads;
  uint32_t v[per];
#pragma unroll
  for (int j = 0; j < per; j++) {
    const int idx = tid + j * kApplyThreads;
    if (idx < nseeds * len) {
      const int k = idx / len, i = lo + idx % len;
      const uint32_t* w = win + k * kIrrWin + kIrrCarry;
      const uint32_t nx = i == kMtN - 1 ? w[0] : w[i + 1];
      const uint32_t m = i < kMtN - kMtM ? w[i + kMtM] : w[i - (kMtN - kMtM)];
      v[j] = m ^ mt_twist(w[i], nx);
    }
  }
  uint32_t cv = 0;
  if (PH == 0 && tid < nseeds * kIrrCarry) cv = win[(tid / kIrrCarry) * kIrrWin + kIrrCarry + kMtN - kIrrCarry + tid % kIrrCarry];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < per; j++) {
    const int idx = tid + j * kApplyThreads;
    if (idx < nseeds * len) win[(idx / len) * kIrrWin + kIrrCarry + lo + idx % len] = v[j];
  }
  if (PH == 0 && tid < nseeds * kIrrCarry) win[(tid / kIrrCarry) * kIrrWin + tid % kIrrCarry] = cv;
  __syncthreads();
}

// z pair from two raw words, any dtype (f16 through its 11-bit tables in constant memory)
constexpr int kIrrLogfOff = kLdsTabBytes + 4 * (kIrrWin * kMaxSeedsPerPass + 16);  // after the wave counters
static_assert(kIrrLogfOff % 16 == 0, "logf table alignment");

template <int DT>
__device__ __forceinline__ void irr_z_pair(const uint8_t* lds, uint32_t r1, uint32_t r2, float& z1, float& z2) {
  if constexpr (DT == kDtF32Libm) {
    z_pair_f32_libm((uint32_t)kIrrLogfOff, r1, r2, z1, z2);
  } else if constexpr (DT == FKS_F16) {
    const uint32_t a = mt_temper(r1) & 0x7FFu, b = mt_temper(r2) & 0x7FFu;
    z1 = rhf(__fmaf_rn(c_tab_f16[a], c_tab_f16[2048 + b], 0.0f));
    z2 = rhf(__fmaf_rn(c_tab_f16[a], c_tab_f16[4096 + b], 0.0f));
  } else {
    z_pair<DT>(lds, r1, r2, z1, z2);
  }
}

template <int DT, int MODE>
__device__ __forceinline__ void irr_run_lane(const uint8_t* lds, const uint32_t* win, const IrrArgs& a, const DevRun& R,
                                             int64_t e1, int w1) {
  using TR = Traits<MODE == kModeDelta ? FKS_F32 : DT>;  // storage (kModeDelta: the f32 delta)
  const bool on1 = e1 < R.limit, on2 = e1 + 8 < R.limit;
  float p1 = 0.0f, p2 = 0.0f;
  if (MODE != kModeWriteZ) {
    if (on1) p1 = TR::load(R.ptr, e1);
    if (on2) p2 = TR::load(R.ptr, e1 + 8);
  }
  const bool has_wd = (R.flags & FKS_HAS_WD) != 0;
  const float* g = a.g[DT == kDtF32Libm ? FKS_F32 : DT];
  const bool dv = MODE == kModePerturbUpdate && a.gdev;
  const bool upd = dv ? dev_value_apply(a.gdev) : true;
  for (int k = 0; k < a.nseeds; k++) {
    float z1, z2;
    irr_z_pair<DT>(lds, win_word(win, k, w1), win_word(win, k, w1 + 8), z1, z2);
    const float gv = dv ? dev_value_g<DT>(a.gdev) : g[k];
    p1 = apply_one<DT>(p1, z1, gv, R.lr, R.wd, has_wd, MODE, R.ps, upd);
    p2 = apply_one<DT>(p2, z2, gv, R.lr, R.wd, has_wd, MODE, R.ps, upd);
  }
  if (on1) TR::store(R.ptr, e1, p1);
  if (on2) TR::store(R.ptr, e1 + 8, p2);
}

__device__ __forceinline__ double u53(uint32_t hi, uint32_t lo) {  // uniform_real_distribution<double>
  const uint64_t x = (((uint64_t)hi << 32) | lo) & ((1ull << 53) - 1);
  return (double)x * (1.0 / 9007199254740992.0);
}

template <int DT, int MODE>
__device__ __forceinline__ void irr_tiny_lane(const uint32_t* win, const IrrArgs& a, const DevTiny& T, int w) {
  using TR = Traits<MODE == kModeDelta ? FKS_F32 : DT>;  // storage (kModeDelta: the f32 delta)
  float p = MODE != kModeWriteZ ? TR::load(T.ptr, 0) : 0.0f;
  const bool has_wd = (T.flags & FKS_HAS_WD) != 0;
  const bool sin_half = (T.flags & kTinySin) != 0;
  const float* g = a.g[DT];
  const bool dv = MODE == kModePerturbUpdate && a.gdev;
  const bool upd = dv ? dev_value_apply(a.gdev) : true;
  for (int k = 0; k < a.nseeds; k++) {
    const double u1 = u53(mt_temper(win_word(win, k, w)), mt_temper(win_word(win, k, w + 1)));
    const double u2 = u53(mt_temper(win_word(win, k, w + 2)), mt_temper(win_word(win, k, w + 3)));
    // glibc's log1p and correctly rounded sin / cos (fks_libm.h): ocml's differ from the
    // host libm by an ulp often enough to flip fp32 midpoint cases
    const double r = sqrt(-2.0 * fks_libm::log1p(-u2));
    const double theta = 2.0 * 3.14159265358979323846 * u1;
    const double v = r * fks_libm::sin_or_cos(theta, sin_half) * 1.0 + 0.0;
    const float zf = (float)v;  // static_cast<scalar_t>(double): via float for bf16 / f16
    const float z = DT == FKS_F32 ? zf : Traits<DT>::rnd(zf);
    p = apply_one<DT>(p, z, dv ? dev_value_g<DT>(a.gdev) : g[k], T.lr, T.wd, has_wd, MODE, T.ps, upd);
  }
  TR::store(T.ptr, 0, p);
}

template <int MODE>
__global__ __launch_bounds__(kApplyThreads) void fks_irregular_kernel(IrrArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds32[];
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds32);
  uint32_t* win = reinterpret_cast<uint32_t*>(lds + kLdsTabBytes);
  uint32_t* cnt = win + kIrrWin * kMaxSeedsPerPass;  // per-wave counters
  if ((uint32_t)(size_t)(lds_u32_t*)lds32 != 0u) __builtin_trap();  // z_pair reads the tables at LDS 0
  const int tid = threadIdx.x;
  const int c = blockIdx.x;
  const int nseeds = a.nseeds;
  const int64_t b0 = a.chunk_lo[c], b1 = a.chunk_hi[c];
  {
    float2* tabCS = reinterpret_cast<float2*>(lds + kLdsCsOff);
    for (int i = tid; i < 256; i += kApplyThreads) {
      reinterpret_cast<float*>(lds)[i] = c_tab_bf16[i];
      tabCS[i] = make_float2(c_tab_bf16[256 + i], c_tab_bf16[512 + i]);
    }
  }
  if (a.libm) logf_tab_fill((uint32_t)kIrrLogfOff, tid, kApplyThreads);
  for (int idx = tid; idx < nseeds * kMtN; idx += kApplyThreads) {
    const int k = idx / kMtN, i = idx - k * kMtN;
    win[k * kIrrWin + kIrrCarry + i] = a.states[((size_t)k * a.nchunks + c) * kMtN + i];
  }
  // first run whose last word is in or after block b0; first single element likewise
  int ri, ti;
  {
    int lo = 0, hi = a.nruns;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (a.runs[mid].start + a.runs[mid].numel - 1 < (int64_t)kMtN * b0) lo = mid + 1; else hi = mid;
    }
    ri = lo;
    lo = 0, hi = a.ntiny;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (a.tiny[mid].word + 3 < (int64_t)kMtN * b0) lo = mid + 1; else hi = mid;
    }
    ti = lo;
  }
  __syncthreads();
  const int m = tid >> 3, r8 = tid & 7;
  for (int64_t b = b0; b < b1; b++) {
    irr_twist_phase<0>(win, nseeds, tid);
    irr_twist_phase<1>(win, nseeds, tid);
    irr_twist_phase<2>(win, nseeds, tid);
    const int64_t base = (int64_t)kMtN * b, end = base + kMtN;
    // runs with a 16-block ending in this block (disjoint, sorted: a contiguous range)
    while (ri < a.nruns && a.runs[ri].start + 15 < end) {
      const DevRun R = a.runs[ri];
      const int ph = (int)(R.start & 15);
      const int64_t s0 = base + 16 * m + (ph ? ph - 16 : 0);  // this lane's 16-block start
      if (tid < kMtN / 2 && s0 >= R.start && s0 < R.start + R.numel) {
        const int64_t e1 = s0 - R.start + r8;
        const int w1 = (int)(s0 - base) + r8;
        switch (R.dtype) {
          case FKS_F32:
            if (a.libm) irr_run_lane<kDtF32Libm, MODE>(lds, win, a, R, e1, w1);
            else irr_run_lane<FKS_F32, MODE>(lds, win, a, R, e1, w1);
            break;
          case FKS_BF16: irr_run_lane<FKS_BF16, MODE>(lds, win, a, R, e1, w1); break;
          default: irr_run_lane<FKS_F16, MODE>(lds, win, a, R, e1, w1); break;
        }
      }
      if (R.start + R.numel - 1 < end) ri++; else break;
    }
    // single elements whose draw pair ends in this block (sorted: a prefix from ti)
    for (;;) {
      const int idx = ti + tid;
      const bool mine = idx < a.ntiny && a.tiny[idx].word + 3 < end;
      if (mine) {
        const DevTiny T = a.tiny[idx];
        const int w = (int)(T.word - base);
        switch (T.dtype) {
          case FKS_F32: irr_tiny_lane<FKS_F32, MODE>(win, a, T, w); break;
          case FKS_BF16: irr_tiny_lane<FKS_BF16, MODE>(win, a, T, w); break;
          default: irr_tiny_lane<FKS_F16, MODE>(win, a, T, w); break;
        }
      }
      // block-wide count of `mine` through a few dynamic-LDS words (__syncthreads_count
      // would add static LDS and move the dynamic block off address 0)
      const uint64_t bal = __ballot(mine);
      if ((tid & 63) == 0) cnt[tid >> 6] = (uint32_t)__popcll(bal);
      __syncthreads();
      int n = 0;
#pragma unroll
      for (int w = 0; w < kApplyThreads / 64; w++) n += (int)cnt[w];
      __syncthreads();
      ti += n;
      if (n < kApplyThreads) break;
    }
  }
}

// ------------------------------------------------------------------ torch_rocm stream
// fks_philox_kernel<MODE>: the z stream torch.normal draws on a HIP device (FKS_STREAM_ROCM;
// PhxTensor in fks_internal.h has the mapping), then the same per-op-rounded update as the
// CPU stream.  One thread per work item (tensor, idx, j): for every seed in order one
// Philox4x32-10 call at counter (off4 + j, idx, 0) and key (seed), two rocrand Box-Muller
// pairs, four elements idx + stride (4 j + i).  Counter-mode: no generator state, no jump.
// Round 1 of Philox4x32-10 multiplies the COUNTER only (the key enters by xor), so an
// item computes it once for all the seeds of a pass.
struct PhxRound1 {
  uint32_t a0, a2;  // hi(M1 c2) ^ c1, hi(M0 c0) ^ c3: xored with the key halves
  uint32_t c1, c3;  // lo(M1 c2), lo(M0 c0)
};
__device__ __forceinline__ PhxRound1 philox_round1(uint64_t ctr, uint32_t idx) {
  const uint64_t m0 = (uint64_t)0xD2511F53u * (uint32_t)ctr, m1 = (uint64_t)0xCD9E8D57u * idx;
  return PhxRound1{(uint32_t)(m1 >> 32) ^ (uint32_t)(ctr >> 32), (uint32_t)(m0 >> 32), (uint32_t)m1, (uint32_t)m0};
}
__device__ __forceinline__ uint4 philox4x32_10(const PhxRound1& r1, uint64_t seed) {
  // Random123 Philox4x32-10 as rocrand_philox4x32_10.h:270-303 (counter (x, y, z, w) =
  // (ctr lo, ctr hi, subsequence lo, hi), key (seed lo, hi), bumped by the Weyl constants)
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  uint32_t c0 = r1.a0 ^ k0, c1 = r1.c1, c2 = r1.a2 ^ k1, c3 = r1.c3;
  k0 += 0x9E3779B9u;
  k1 += 0xBB67AE85u;
#pragma unroll
  for (int r = 1; r < 10; r++) {
    const uint64_t m0 = (uint64_t)0xD2511F53u * c0, m1 = (uint64_t)0xCD9E8D57u * c2;
    // one v_bitop3_b32 per three-input xor (two v_xor_b32 otherwise)
    const uint32_t n0 = bs::xor3((uint32_t)(m1 >> 32), c1, k0), n2 = bs::xor3((uint32_t)(m0 >> 32), c3, k1);
    c1 = (uint32_t)m1;
    c3 = (uint32_t)m0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return make_uint4(c0, c1, c2, c3);
}

// rocrand_normal.h:53-68 box_muller as torch's ROCm build compiles it (hipcc's default
// fp-contract: the uniforms' multiply-add is one fma): (sin * s, cos * s) -- then torch's
// transformation::normal, val * std + mean with std 1, mean 0 (one fma: -0 becomes +0).
__device__ __forceinline__ float2 rocrand_box_muller(uint32_t x, uint32_t y) {
  const float u = __fmaf_rn((float)x, 2.3283064e-10f, 2.3283064e-10f);
  const float v = __fmaf_rn((float)y, 1.46291807e-09f, 1.46291807e-09f);
  const float s = sqrtf(-2.0f * logf(u));
  float sn, cs;
  __sincosf(v, &sn, &cs);
  return make_float2(__fmaf_rn(sn * s, 1.0f, 0.0f), __fmaf_rn(cs * s, 1.0f, 0.0f));
}

template <int DT>
__device__ __forceinline__ float phx_cast(float v) {  // static_cast<scalar_t>(float)
  return DT == FKS_F32 ? v : Traits<DT>::rnd(v);
}

// Both Box-Muller pairs of one Philox output, (w.x, w.y) and (w.z, w.w), as the
// instructions rocrand_box_muller compiles to, restricted to the inputs Philox can give
// them and with the two pairs' float arithmetic packed (v_pk_*_f32):
//   u = fma(x, 2^-32, 2^-32) lies in [2^-32, 1]: ocml's logf takes its normal-input path
//     -- v_log_f32, then y ln2 in extended precision, r + e with r = RN(y ln2_hi),
//     e = fma(y, ln2_hi, -r) + y ln2_lo -- with no denormal rescaling and no infinity
//     select; the -2 (an exact scaling) is folded into ln2_hi / ln2_lo (RN(-2 a) = -2 RN(a)
//     without underflow; only the sign of a zero can change, and a zero radius becomes +0
//     in the final "+ 0" either way);
//   x = -2 log u is 0 or >= 1.19e-7: the correctly rounded sqrtf takes its unscaled path
//     -- v_sqrt_f32 and the +-1 ulp correction by two fma residuals (sqrt(+-0) = +-0
//     falls out of the correction unchanged, so the +-0 / inf class select is dead);
//   (sin(v) s, cos(v) s) + 0 as one fma with a +0 addend (no product underflows: |s| >=
//     3.4e-4 or s = 0, |sin|, |cos| >= 1e-9 or exactly 0).
// fks_device_selfcheck(FKS_CHECK_PHILOX_RADIUS) compares phx_radius2 with ocml's
// sqrtf(-2 logf(u)) on all 2^32 words; tests/test_gpu_torch_rocm.py the whole stream with
// torch.normal on the device.
// The bf16 fast path's radius: x = RN(log2(u) RN(-2 ln 2)) in ONE rounding instead of
// ocml's extended-precision r + e, then the raw v_sqrt_f32.  Within kPhxFastUlps ulps of
// the exact radius on every one of the 2^32 words (fks_device_selfcheck
// FKS_CHECK_PHILOX_BF16_RADIUS reports the largest distance; tests/test_gpu_selfcheck.py).
constexpr uint32_t kPhxFastUlps = 2;
__device__ __forceinline__ f32x2_t phx_radius2_fast(const f32x2_t u) {
  const f32x2_t y = {__builtin_amdgcn_logf(u.x), __builtin_amdgcn_logf(u.y)};
  const f32x2_t x = y * (f32x2_t){__uint_as_float(0xbfb17218u), __uint_as_float(0xbfb17218u)};  // RN(-2 ln 2)
  return (f32x2_t){__builtin_amdgcn_sqrtf(x.x), __builtin_amdgcn_sqrtf(x.y)};
}

template <bool kExact = true>
__device__ __forceinline__ f32x2_t phx_radius2(const f32x2_t u) {
  const f32x2_t y = {__builtin_amdgcn_logf(u.x), __builtin_amdgcn_logf(u.y)};
  const f32x2_t m2hi = {__uint_as_float(0xbfb17217u), __uint_as_float(0xbfb17217u)};  // -2 x 0x3f317217
  const f32x2_t m2lo = {__uint_as_float(0xb3f7d1cfu), __uint_as_float(0xb3f7d1cfu)};  // -2 x 0x3377d1cf
  const f32x2_t r = y * m2hi;
  f32x2_t e = __builtin_elementwise_fma(y, m2hi, -r);
  e = __builtin_elementwise_fma(m2lo, y, e);
  const f32x2_t x = r + e;
  f32x2_t sq = {__builtin_amdgcn_sqrtf(x.x), __builtin_amdgcn_sqrtf(x.y)};
  if (!kExact) return sq;  // within 1 ulp of the correctly rounded root (phx_z_bf16)
  const f32x2_t sm = {__int_as_float(__float_as_int(sq.x) - 1), __int_as_float(__float_as_int(sq.y) - 1)};
  const f32x2_t sp = {__int_as_float(__float_as_int(sq.x) + 1), __int_as_float(__float_as_int(sq.y) + 1)};
  const f32x2_t rm = __builtin_elementwise_fma(-sm, sq, x), rp = __builtin_elementwise_fma(-sp, sq, x);
  sq.x = rm.x <= 0.0f ? sm.x : sq.x;
  sq.y = rm.y <= 0.0f ? sm.y : sq.y;
  sq.x = rp.x > 0.0f ? sp.x : sq.x;
  sq.y = rp.y > 0.0f ? sp.y : sq.y;
  return sq;
}

template <bool kExact = true, bool kFast = false>
__device__ __forceinline__ void phx_box_muller2(const uint4 w, f32x2_t& zA, f32x2_t& zB) {
  const f32x2_t cu = {2.3283064e-10f, 2.3283064e-10f}, cv = {1.46291807e-09f, 1.46291807e-09f};
  const f32x2_t fx = {(float)w.x, (float)w.z}, fy = {(float)w.y, (float)w.w};
  const f32x2_t u = __builtin_elementwise_fma(fx, cu, cu);
  const f32x2_t sq = kFast ? phx_radius2_fast(u) : phx_radius2<kExact>(u);
  const f32x2_t v = __builtin_elementwise_fma(fy, cv, cv);
  const f32x2_t rev = v * (f32x2_t){__uint_as_float(0x3e22f983u), __uint_as_float(0x3e22f983u)};  // 1/(2 pi)
  const f32x2_t sc1 = {__builtin_amdgcn_sinf(rev.x), __builtin_amdgcn_cosf(rev.x)};
  const f32x2_t sc2 = {__builtin_amdgcn_sinf(rev.y), __builtin_amdgcn_cosf(rev.y)};
  const f32x2_t zero = {0.0f, 0.0f};
  zA = __builtin_elementwise_fma(sc1, (f32x2_t){sq.x, sq.x}, zero);
  zB = __builtin_elementwise_fma(sc2, (f32x2_t){sq.y, sq.y}, zero);
}

// The four z of one Philox output rounded to bf16.  Only the bf16 value matters here, so
// the radius's +-1 ulp correction (a third of phx_radius2's instructions) is skipped
// unless it could change it: with the root within 1 ulp, z = (sin or cos) s moves by at
// most 3 f32 ulps, which changes the bf16 rounding only for a product within 3 ulps of a
// rounding midpoint (low 16 bits 0x8000; across a binade both round to the power of two).
// Lanes with any of their four products within 4 ulps of one redo the pair exactly (about
// 3.5 % of the waves' iterations branch).
// Window half-width W in f32 ulps around a bf16 rounding midpoint: a radius within k ulps
// of the exact one moves z = RN(sc s) by at most 2k + 1 ulps (|sc| <= 1, the product's
// ulp at most twice sc's ulp times s's), so W = 2k + 2: k = 1 for the raw root of the
// exact x (W = 4), k = kPhxFastUlps for the one-rounding x (FKS_PHX_FAST_LOG).
#ifndef FKS_PHX_FAST_LOG
#define FKS_PHX_FAST_LOG 1
#endif
constexpr uint32_t kPhxMidW = FKS_PHX_FAST_LOG ? 2 * kPhxFastUlps + 2 : 4;
__device__ __forceinline__ bool phx_near_bf16_mid(float z) {
  return ((__float_as_uint(z) & 0xFFFFu) - (0x8000u - kPhxMidW)) <= 2 * kPhxMidW;
}
__device__ __forceinline__ void phx_z_bf16(const uint4 w, f32x2_t& zA, f32x2_t& zB) {
#if FKS_PHX_EXACT_RADIUS  // A/B: the corrected radius always
  phx_box_muller2<true>(w, zA, zB);
#else
  phx_box_muller2<false, FKS_PHX_FAST_LOG != 0>(w, zA, zB);
  const bool near = (int)phx_near_bf16_mid(zA.x) | (int)phx_near_bf16_mid(zA.y) | (int)phx_near_bf16_mid(zB.x) |
                    (int)phx_near_bf16_mid(zB.y);
  if (__builtin_expect(near, 0)) phx_box_muller2<true>(w, zA, zB);
#endif
  zA = rnd2<FKS_BF16>(zA);
  zB = rnd2<FKS_BF16>(zB);
}

// the radius of one word as ocml computes it (the reference's instructions), for the
// self check of phx_radius2
__device__ __forceinline__ float phx_radius_ocml(uint32_t x) {
  return sqrtf(-2.0f * logf(__fmaf_rn((float)x, 2.3283064e-10f, 2.3283064e-10f)));
}

// The item's four elements through every seed of the pass, in seed order, as two packed
// pairs (apply_pair: the values of apply_one); MODE may be a launch-wide weight-decay
// specialisation of kModeUpdate (kModeUpdateWd / NoWd / Wd0, as the CPU stream's kernels).
// (phx_seeds: the seed loop of work item (idx, j) on its four elements e[i], values p[i])
template <int DT, int MODE_>
__device__ __forceinline__ void phx_seeds(const PhiloxArgs& a, const PhxTensor& T, uint32_t idx, uint64_t j,
                                          const int64_t e[4], float p[4]) {
  // (the host gives kModeUpdateWdPos0 launches bf16 / f32 tensors only)
  constexpr int MODE = (MODE_ == kModeUpdateWdPos0 && DT == FKS_F16) ? (int)kModeUpdateWd0 : MODE_;
#pragma unroll
  for (int i = 0; i < 4; i++)  // kModeUpdateWdPos0: a +-inf parameter is NaN after the reference's first seed (wd p)
    if (MODE == kModeUpdateWdPos0 && __builtin_isinf(p[i])) p[i] = __builtin_nanf("");
  const bool has_wd = (T.flags & FKS_HAS_WD) != 0;
  const bool dv = MODE == kModePerturbUpdate && a.gdev;
  const bool upd = dv ? dev_value_apply(a.gdev) : true;
  const float gd = dv ? dev_value_g<DT>(a.gdev) : 0.0f;
  const PhxRound1 r1 = philox_round1(T.off4 + j, idx);
  f32x2_t pA = {p[0], p[1]}, pB = {p[2], p[3]};
  // f16: which elements torch's unrolled path (one rounding) takes (mul_f16_ref): the
  // partial last block of the launch, or every element of a launch whose fresh tensors do
  // not start 16-byte aligned (a later 32-bit piece of a tensor past 2^31 bytes)
  bool tail[4] = {false, false, false, false};
  const bool p16 = (T.flags & kPhxWdP16) != 0;  // the first wd * p's operand, in the reference
  if (DT == FKS_F16) {
    const bool fresh16 = (T.flags & kPhxFresh16) != 0;
#pragma unroll
    for (int i = 0; i < 4; i++) tail[i] = !fresh16 || e[i] >= T.numel - T.numel % kTorchHalfBlockWork;
  }
  for (int k = 0; k < a.nseeds; k++) {
    const uint64_t seed = a.seeds[k];  // wave-uniform: scalar loads
    const float g = dv ? gd : a.g[3 * k + DT];
    const uint4 w = philox4x32_10(r1, seed);
#if FKS_PHX_V1  // round-3 form (A/B): ocml's general logf / sqrtf and one pair at a time
    const float2 b1 = rocrand_box_muller(w.x, w.y), b2 = rocrand_box_muller(w.z, w.w);
    const f32x2_t zA = {phx_cast<DT>(b1.x), phx_cast<DT>(b1.y)}, zB = {phx_cast<DT>(b2.x), phx_cast<DT>(b2.y)};
#else
    f32x2_t zA, zB;
    if constexpr (DT == FKS_BF16) {
      phx_z_bf16(w, zA, zB);
    } else {
      phx_box_muller2(w, zA, zB);
      zA = (f32x2_t){phx_cast<DT>(zA.x), phx_cast<DT>(zA.y)};
      zB = (f32x2_t){phx_cast<DT>(zB.x), phx_cast<DT>(zB.y)};
    }
#endif
    if (MODE == kModeWriteZ) {
      pA = zA;
      pB = zB;
    } else if constexpr (DT == FKS_F16 && MODE != kModeDelta) {  // torch's device rounding of the products (mul_f16_ref)
      // wd p at the call's first seed reads the caller's parameter (its alignment); later
      // seeds read the reference's freshly allocated, aligned result.  (kModePerturbUpdate's
      // update follows the restore perturbation, whose result is fresh.)
      const bool first = a.call_first && k == 0 && MODE != kModePerturbUpdate;
      const bool wA[2] = {tail[0] || (first && !p16), tail[1] || (first && !p16)};
      const bool wB[2] = {tail[2] || (first && !p16), tail[3] || (first && !p16)};
      const bool oA[2] = {tail[0], tail[1]}, oB[2] = {tail[2], tail[3]};
      pA = apply_pair_f16dev<MODE>(pA, zA, g, T.lr, T.wd, has_wd, T.ps, upd, oA, wA);
      pB = apply_pair_f16dev<MODE>(pB, zB, g, T.lr, T.wd, has_wd, T.ps, upd, oB, wB);
    } else {
      pA = apply_pair<DT, MODE>(pA, zA, g, T.lr, T.wd, has_wd, T.ps, upd);
      pB = apply_pair<DT, MODE>(pB, zB, g, T.lr, T.wd, has_wd, T.ps, upd);
    }
  }
  p[0] = pA.x; p[1] = pA.y; p[2] = pB.x; p[3] = pB.y;
}

template <int DT, int MODE>
__device__ __forceinline__ void phx_item(const PhiloxArgs& a, const PhxTensor& T, int64_t r) {
  using TR = Traits<MODE == kModeDelta ? FKS_F32 : DT>;  // storage (kModeDelta: the f32 delta)
  const uint32_t S = T.stride;
  const uint32_t idx = (uint32_t)(r % S);
  const uint64_t j = (uint64_t)(r / S);
  int64_t e[4];
  bool on[4];
  float p[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    e[i] = (int64_t)idx + (int64_t)S * (int64_t)(4 * j + i);
    on[i] = e[i] < T.numel;
    p[i] = (MODE != kModeWriteZ && on[i]) ? TR::load(T.ptr, e[i]) : 0.0f;
  }
  phx_seeds<DT, MODE>(a, T, idx, j, e, p);
#pragma unroll
  for (int i = 0; i < 4; i++)
    if (on[i]) TR::store(T.ptr, e[i], p[i]);
}

// kPhxVec consecutive work items (idx0 .. idx0 + 7 of one row j; item boundaries of
// tensors and shards are multiples of 256): element i of each lies in the 8-element run
// idx0 + S (4 j + i) + [0, 8), so the eight items load and store as four 16-byte runs
// (bf16 / f16; two each for f32) instead of 32 single-element accesses.  A call of few
// seeds is bound by the memory accesses in flight, not by the VALU (the item loop above
// issues 2-byte loads, 128 bytes per wave instruction: a one-seed perturb of the 7B layout
// took 20.9 ms there, 7.2 ms here; profiles/r05h_smallk_rocm_maxk*.log).
#ifndef FKS_PHX_VEC_ITEMS
#define FKS_PHX_VEC_ITEMS 8
#endif
constexpr int kPhxVec = FKS_PHX_VEC_ITEMS;  // 8 (A/B: 4)
static_assert(kPhxVec == 4 || kPhxVec == 8, "16- or 8-byte runs of 2-byte elements");
typedef __attribute__((address_space(1))) u32x4_t gu128;

typedef __attribute__((address_space(1))) u32x2_t gu64v;

template <int DT>
__device__ __forceinline__ void phx_load8(uint64_t ptr, int64_t e, float v[kPhxVec]) {
  const gu128* q = reinterpret_cast<const gu128*>(ptr + (uint64_t)e * (DT == FKS_F32 ? 4 : 2));
  if constexpr (kPhxVec == 4) {
    if constexpr (DT == FKS_F32) {
      const u32x4_t x = q[0];
      v[0] = __uint_as_float(x.x); v[1] = __uint_as_float(x.y); v[2] = __uint_as_float(x.z); v[3] = __uint_as_float(x.w);
    } else {
      const u32x2_t x = *reinterpret_cast<const gu64v*>(q);
      v[0] = Traits<DT>::cvt(x.x & 0xffffu); v[1] = Traits<DT>::cvt(x.x >> 16);
      v[2] = Traits<DT>::cvt(x.y & 0xffffu); v[3] = Traits<DT>::cvt(x.y >> 16);
    }
  } else if constexpr (DT == FKS_F32) {
    const u32x4_t x = q[0], y = q[1];
    const uint32_t w[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = __uint_as_float(w[i]);
  } else {
    const u32x4_t x = q[0];
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
      v[2 * i] = Traits<DT>::cvt(w[i] & 0xffffu);
      v[2 * i + 1] = Traits<DT>::cvt(w[i] >> 16);
    }
  }
}

template <int DT>
__device__ __forceinline__ void phx_store8(uint64_t ptr, int64_t e, const float v[kPhxVec]) {
  gu128* q = reinterpret_cast<gu128*>(ptr + (uint64_t)e * (DT == FKS_F32 ? 4 : 2));
  if constexpr (kPhxVec == 4) {
    if constexpr (DT == FKS_F32) {
      q[0] = (u32x4_t){__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
    } else {
      *reinterpret_cast<gu64v*>(q) = (u32x2_t){Traits<DT>::pack(Traits<DT>::bits(v[0]), Traits<DT>::bits(v[1])),
                                               Traits<DT>::pack(Traits<DT>::bits(v[2]), Traits<DT>::bits(v[3]))};
    }
  } else if constexpr (DT == FKS_F32) {
    q[0] = (u32x4_t){__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
    q[1] = (u32x4_t){__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]), __float_as_uint(v[7])};
  } else {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; i++) w[i] = Traits<DT>::pack(Traits<DT>::bits(v[2 * i]), Traits<DT>::bits(v[2 * i + 1]));
    q[0] = (u32x4_t){w[0], w[1], w[2], w[3]};
  }
}

template <int DT, int MODE>
__device__ __forceinline__ void phx_vitem(const PhiloxArgs& a, const PhxTensor& T, int64_t r0) {
  constexpr int ST = MODE == kModeDelta ? FKS_F32 : DT;  // storage (kModeDelta: the f32 delta)
  const uint32_t S = T.stride;
  const uint32_t idx0 = (uint32_t)(r0 % S);
  const uint64_t j = (uint64_t)(r0 / S);
  const int64_t e0 = (int64_t)idx0 + (int64_t)S * (int64_t)(4 * j);
  // whole runs only: 16-byte aligned data (idx0 and S are multiples of 8) and every element
  // of the four runs inside the tensor; else (a tensor's last row, unaligned data) per item
  if (!(T.flags & kPhxP16) || e0 + 3 * (int64_t)S + kPhxVec > T.numel) {
    for (int q = 0; q < kPhxVec; q++) phx_item<DT, MODE>(a, T, r0 + q);
    return;
  }
  float v[4][kPhxVec];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (MODE == kModeWriteZ) {
#pragma unroll
      for (int q = 0; q < kPhxVec; q++) v[i][q] = 0.0f;
    } else {
      phx_load8<ST>(T.ptr, e0 + (int64_t)S * i, v[i]);
    }
  }
#pragma unroll
  for (int q = 0; q < kPhxVec; q++) {
    int64_t e[4];
    float p[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      e[i] = e0 + (int64_t)S * i + q;
      p[i] = v[i][q];
    }
    phx_seeds<DT, MODE>(a, T, idx0 + (uint32_t)q, j, e, p);
#pragma unroll
    for (int i = 0; i < 4; i++) v[i][q] = p[i];
  }
#pragma unroll
  for (int i = 0; i < 4; i++) phx_store8<ST>(T.ptr, e0 + (int64_t)S * i, v[i]);
}

template <int MODE>
__global__ __launch_bounds__(256) void fks_philox_kernel(PhiloxArgs a) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  int t0 = 0;  // items only grow: the search starts at the previous item's tensor
  for (int64_t it = a.item_lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; it < a.item_hi; it += step) {
    int lo = t0, hi = a.nt - 1;  // the last tensor whose first item is <= it
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (a.t[mid].item0 <= it) lo = mid; else hi = mid - 1;
    }
    t0 = lo;
    const PhxTensor T = a.t[lo];
    switch (T.dtype) {
      case FKS_F32: phx_item<FKS_F32, MODE>(a, T, it - T.item0); break;
      case FKS_BF16: phx_item<FKS_BF16, MODE>(a, T, it - T.item0); break;
      default: phx_item<FKS_F16, MODE>(a, T, it - T.item0); break;
    }
  }
}

// fks_philox_kernel over kPhxVec-item groups (phx_vitem): the launch form of calls of few
// seeds (the ZO step's perturb / restore + update, K-small reconstructs)
#if defined(FKS_PHX_VEC_WPE) && FKS_PHX_VEC_WPE > 0  // A/B: a waves-per-SIMD floor (caps the VGPRs)
#define FKS_PHX_VEC_ATTR __attribute__((amdgpu_waves_per_eu(FKS_PHX_VEC_WPE)))
#else
#define FKS_PHX_VEC_ATTR
#endif
// FKS_PHX_VEC_UNIFORM: the tensor of a wave's 64 groups is looked up once per wave, with
// wave-uniform indices, instead of a per-lane binary search whose dependent vector loads
// each wait for every load and store in flight (vmcnt is in order); 2 (default): from a
// copy of the tensor table in LDS (launches of at most kPhxLdsTensors tensors).  One-seed
// perturb of the 7B layout: 7.07 (0, per-lane search) / 6.86-7.30 (1) / 6.41-6.45 ms (2),
// 32-seed launches unchanged (profiles/r05k_phx_vec_uniform_ab.log)
#ifndef FKS_PHX_VEC_UNIFORM
#define FKS_PHX_VEC_UNIFORM 2
#endif
constexpr int kPhxLdsTensors = 512;
__device__ __forceinline__ int64_t rfl64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
template <class Tab>
__device__ __forceinline__ int phx_find_t(Tab tab, int nt, int64_t it, int lo, int probes) {
  // the last tensor whose first item is <= it, at or after lo (items only grow; a wave's
  // next groups lie mostly in the same or the next tensor: a few probes, then bisection)
  for (int p = 0; p < probes; p++) {
    if (lo + 1 >= nt || tab[lo + 1].item0 > it) return lo;
    ++lo;
  }
  int hi = nt - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].item0 <= it) lo = mid; else hi = mid - 1;
  }
  return lo;
}
template <int MODE, class Tab>
__device__ __forceinline__ void phx_vec_uniform(const PhiloxArgs& a, Tab tab, int64_t step) {
  const int lane = (int)(threadIdx.x & 63u);
  int64_t wb = rfl64(a.item_lo + ((int64_t)blockIdx.x * blockDim.x + (int64_t)(threadIdx.x & ~63u)) * kPhxVec);
  int ts = 0;
  // this lane's group of the wave's groups from wb, and its tensor (ts: the wave's first)
  auto lane_tensor = [&](int64_t w, int t, int64_t& it) {
    const int64_t wend = w + 64 * kPhxVec < a.item_hi ? w + 64 * kPhxVec : a.item_hi;
    const bool one = t + 1 >= a.nt || tab[t + 1].item0 >= wend;  // the whole wave in tensor t
    it = w + (int64_t)lane * kPhxVec;
    return one ? t : phx_find_t(tab, a.nt, it < a.item_hi ? it : a.item_hi - 1, t, 0);
  };
  for (; wb < a.item_hi; wb += step) {
    ts = __builtin_amdgcn_readfirstlane(phx_find_t(tab, a.nt, wb, ts, 2));
    int64_t it;
    const int ti = lane_tensor(wb, ts, it);
    if (it >= a.item_hi) continue;
    const PhxTensor T = tab[ti];
    switch (T.dtype) {
      case FKS_F32: phx_vitem<FKS_F32, MODE>(a, T, it - T.item0); break;
      case FKS_BF16: phx_vitem<FKS_BF16, MODE>(a, T, it - T.item0); break;
      default: phx_vitem<FKS_F16, MODE>(a, T, it - T.item0); break;
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(256) FKS_PHX_VEC_ATTR void fks_philox_vec_kernel(PhiloxArgs a) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x * kPhxVec;
#if FKS_PHX_VEC_UNIFORM
#if FKS_PHX_VEC_UNIFORM == 2
  extern __shared__ PhxTensor s_tab[];
  if (a.nt <= kPhxLdsTensors) {
    constexpr int W = (int)(sizeof(PhxTensor) / 4);
    for (int i = (int)threadIdx.x; i < a.nt * W; i += (int)blockDim.x)
      reinterpret_cast<uint32_t*>(s_tab)[i] = reinterpret_cast<const uint32_t*>(a.t)[i];
    __syncthreads();
    phx_vec_uniform<MODE>(a, s_tab, step);
    return;
  }
#endif
  phx_vec_uniform<MODE>(a, a.t, step);
#else
  int t0 = 0;
  for (int64_t it = a.item_lo + ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * kPhxVec; it < a.item_hi;
       it += step) {
    int lo = t0, hi = a.nt - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (a.t[mid].item0 <= it) lo = mid; else hi = mid - 1;
    }
    t0 = lo;
    const PhxTensor T = a.t[lo];
    switch (T.dtype) {
      case FKS_F32: phx_vitem<FKS_F32, MODE>(a, T, it - T.item0); break;
      case FKS_BF16: phx_vitem<FKS_BF16, MODE>(a, T, it - T.item0); break;
      default: phx_vitem<FKS_F16, MODE>(a, T, it - T.item0); break;
    }
  }
#endif
}

// ------------------------------------------------------------------ delta apply
// Seed-sharded variant, last step: p_K = a^K p_0 - delta (delta = sum_k lr g_k
// a^(K-1-k) z_k, a = 1 - lr wd, all-reduced over the ranks), one fma in f32 and one
// rounding to the parameter dtype.  grid (x, tensors): each row walks one tensor.
template <int DT>
__device__ __forceinline__ void delta_apply_one(const DeltaApplyDesc& D, const float* delta, int64_t e) {
  using TR = Traits<DT>;
  const float p = TR::load(D.ptr, e);
  TR::store(D.ptr, e, TR::rnd(__fmaf_rn(D.decay, p, -delta[D.delta_off + e])));
}

__global__ __launch_bounds__(256) void fks_delta_apply_kernel(const DeltaApplyDesc* d, const float* delta) {
  const DeltaApplyDesc D = d[blockIdx.y];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < D.numel; e += stride) {
    switch (D.dtype) {
      case FKS_F32: delta_apply_one<FKS_F32>(D, delta, e); break;
      case FKS_BF16: delta_apply_one<FKS_BF16>(D, delta, e); break;
      default: delta_apply_one<FKS_F16>(D, delta, e); break;
    }
  }
}

}  // namespace

// ------------------------------------------------------------------ launchers
int launch_delta_apply(const DeltaApplyDesc* d, int n, int64_t max_numel, const float* delta, void* stream) {
  const int64_t blocks = std::min<int64_t>(std::max<int64_t>(1, (max_numel + 255) / 256), 2048);
  hipLaunchKernelGGL(fks_delta_apply_kernel, dim3((unsigned)blocks, (unsigned)n), dim3(256), 0, (hipStream_t)stream,
                     d, delta);
  return (int)hipGetLastError();
}

static size_t apply_lds_bytes() { return (size_t)kLdsTabBytes + (size_t)kLdsStBytes; }

int device_cu_count() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) return 256;
  return n;
}

// Once-per-DEVICE host setup: __constant__ memory and function attributes belong to
// the device a call runs on, and one process may drive several GPUs (the plan cache
// keys on the device id), so every such flag is a bitmask over device ids.
class PerDevice {
 public:
  template <class F>
  int run(F&& f) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -FKS_EINVAL;
    const uint64_t bit = 1ull << dev;
    if (done_.load(std::memory_order_acquire) & bit) return 0;
    std::lock_guard<std::mutex> lk(mu_);
    if (done_.load(std::memory_order_relaxed) & bit) return 0;
    const int e = f();
    if (e == 0) done_.fetch_or(bit, std::memory_order_release);
    return e;
  }

 private:
  std::mutex mu_;
  std::atomic<uint64_t> done_{0};
};

static int ensure_tables() {
  static PerDevice once;
  return once.run([] {
    const Tables& t = tables();
    static float buf[3 * 2048];  // used under the PerDevice mutex only
    for (int i = 0; i < 256; i++) {
      buf[i] = t.r_bf16[i];
      buf[256 + i] = t.c_bf16[i];
      buf[512 + i] = t.s_bf16[i];
    }
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_tab_bf16), buf, sizeof(float) * 768, 0, hipMemcpyHostToDevice);
    if (e != hipSuccess) return (int)e;
    for (int i = 0; i < 2048; i++) {
      buf[i] = t.r_f16[i];
      buf[2048 + i] = t.c_f16[i];
      buf[4096 + i] = t.s_f16[i];
    }
    e = hipMemcpyToSymbol(HIP_SYMBOL(c_tab_f16), buf, sizeof(buf), 0, hipMemcpyHostToDevice);
    return (int)e;
  });
}

// hipFuncAttributeMaxDynamicSharedMemorySize for kernel `fn`, once per device
template <class K>
static int ensure_lds_attr(PerDevice& once, K* fn, int bytes) {
  return once.run([&] {
    return (int)hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    bytes);
  });
}

int launch_jump(const JumpArgs& a, int nseeds, void* stream) {
  const size_t lds = sizeof(uint32_t) * (size_t)kJumpLds2Words;
  static PerDevice attr;
  if (int e = ensure_lds_attr(attr, &fks_jump_kernel, (int)lds)) return e;
  dim3 grid((unsigned)nseeds, (unsigned)((a.nchunks + a.chunks_per_wg - 1) / a.chunks_per_wg));
  hipLaunchKernelGGL(fks_jump_kernel, grid, dim3(kJumpThreads), lds, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

template <int DT, int MODE, bool FULL, bool DB = false>
static int launch_apply_f(const ApplyArgs& a, void* stream) {
  // a partial pass allocates only its own windows (+1 spare: the twist's last-phase lanes
  // read past a window), so calls of few seeds fit more workgroups per CU
  const size_t lds = FULL ? apply_lds_bytes()
                          : (size_t)kLdsTabBytes + (size_t)((DB ? 2 : 1) * a.nseeds + 1) * kWinBytes;
  static PerDevice attr;
  if (int e = ensure_lds_attr(attr, &fks_apply_kernel<DT, MODE, FULL, DB>, (int)apply_lds_bytes())) return e;
  hipLaunchKernelGGL((fks_apply_kernel<DT, MODE, FULL, DB>), dim3((unsigned)a.nchunks),
                     dim3(DB ? kDbThreads : kApplyThreads), lds, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

template <int DT, int MODE, int ZM = 0>
static int launch_small2(const ApplyArgs& a, void* stream) {
  const size_t lds = (size_t)kLdsTabBytes + (size_t)(2 * a.nseeds + 1) * kWinBytes;
  static PerDevice attr;
  // the attribute is set once per device: for the largest pass this kernel takes
  constexpr int kMaxLds = kLdsTabBytes + (2 * kSmallK + 1) * kWinBytes;
  if (int e = ensure_lds_attr(attr, &fks_small2_kernel<DT, MODE, ZM>, kMaxLds)) return e;
  hipLaunchKernelGGL((fks_small2_kernel<DT, MODE, ZM>), dim3((unsigned)a.nchunks), dim3(kSm2Threads), lds,
                     (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

template <int DT, int MODE>
static int launch_apply_t(const ApplyArgs& a, void* stream) {
  if (a.nseeds == kMaxSeedsPerPass) return launch_apply_f<DT, MODE, true>(a, stream);
  if constexpr (DT == FKS_BF16) {
    // one-seed bf16 passes with a z-index buffer (fks_capi.cpp ZCache): store / replay
    if (a.zmode == 1 && a.nseeds == 1 && MODE == kModePerturb) return launch_small2<DT, MODE, 1>(a, stream);
    if (a.zmode == 2 && a.nseeds == 1 &&
        (MODE == kModePerturb || MODE == kModePerturbUpdate || MODE == kModeUpdate || MODE == kModeUpdateWd ||
         MODE == kModeUpdateNoWd || MODE == kModeUpdateWd0)) {
      hipLaunchKernelGGL((fks_zreplay_kernel<MODE>), dim3((unsigned)a.nchunks), dim3(kZrThreads), (size_t)3 * 1024,
                         (hipStream_t)stream, a);
      return (int)hipGetLastError();
    }
  }
  if (a.zmode == 2) return -FKS_ENOTSUP;  // replay without a replay kernel: a host bug
  if (a.nseeds <= kSmallK && DT != FKS_F16) return launch_small2<DT == FKS_F16 ? FKS_F32 : DT, MODE>(a, stream);
  if (a.nseeds <= kSmallK) return launch_apply_f<DT, MODE, false, true>(a, stream);  // f16
  return launch_apply_f<DT, MODE, false>(a, stream);
}

int launch_apply(int dtype, const ApplyArgs& a, void* stream) {
  if (a.nseeds < 1 || a.nseeds > kMaxSeedsPerPass || a.nchunks < 1) return -FKS_EINVAL;
  if (dtype == FKS_BF16) {
    int e = ensure_tables();
    if (e) return e;
  }
  switch (dtype * 8 + a.mode) {
    case FKS_F32 * 8 + kModeUpdate: return launch_apply_t<FKS_F32, kModeUpdate>(a, stream);
    case FKS_F32 * 8 + kModeUpdateWd: return launch_apply_t<FKS_F32, kModeUpdateWd>(a, stream);
    case FKS_F32 * 8 + kModeUpdateNoWd: return launch_apply_t<FKS_F32, kModeUpdateNoWd>(a, stream);
    case FKS_F32 * 8 + kModeUpdateWd0: return launch_apply_t<FKS_F32, kModeUpdateWd0>(a, stream);
    case FKS_F32 * 8 + kModePerturb: return launch_apply_t<FKS_F32, kModePerturb>(a, stream);
    case FKS_F32 * 8 + kModePerturbUpdate: return launch_apply_t<FKS_F32, kModePerturbUpdate>(a, stream);
    case FKS_F32 * 8 + kModeWriteZ: return launch_apply_t<FKS_F32, kModeWriteZ>(a, stream);
    case FKS_F32 * 8 + kModeDelta: return launch_apply_t<FKS_F32, kModeDelta>(a, stream);
    case kDtF32Libm * 8 + kModeUpdate: return launch_apply_t<kDtF32Libm, kModeUpdate>(a, stream);
    case kDtF32Libm * 8 + kModeUpdateWd: return launch_apply_t<kDtF32Libm, kModeUpdateWd>(a, stream);
    case kDtF32Libm * 8 + kModeUpdateNoWd: return launch_apply_t<kDtF32Libm, kModeUpdateNoWd>(a, stream);
    case kDtF32Libm * 8 + kModeUpdateWd0: return launch_apply_t<kDtF32Libm, kModeUpdateWd0>(a, stream);
    case kDtF32Libm * 8 + kModePerturb: return launch_apply_t<kDtF32Libm, kModePerturb>(a, stream);
    case kDtF32Libm * 8 + kModePerturbUpdate: return launch_apply_t<kDtF32Libm, kModePerturbUpdate>(a, stream);
    case kDtF32Libm * 8 + kModeWriteZ: return launch_apply_t<kDtF32Libm, kModeWriteZ>(a, stream);
    case kDtF32Libm * 8 + kModeDelta: return launch_apply_t<kDtF32Libm, kModeDelta>(a, stream);
    case FKS_BF16 * 8 + kModeUpdate: return launch_apply_t<FKS_BF16, kModeUpdate>(a, stream);
    case FKS_BF16 * 8 + kModeUpdateWd: return launch_apply_t<FKS_BF16, kModeUpdateWd>(a, stream);
    case FKS_BF16 * 8 + kModeUpdateNoWd: return launch_apply_t<FKS_BF16, kModeUpdateNoWd>(a, stream);
    case FKS_BF16 * 8 + kModeUpdateWd0: return launch_apply_t<FKS_BF16, kModeUpdateWd0>(a, stream);
    case FKS_BF16 * 8 + kModePerturb: return launch_apply_t<FKS_BF16, kModePerturb>(a, stream);
    case FKS_BF16 * 8 + kModePerturbUpdate: return launch_apply_t<FKS_BF16, kModePerturbUpdate>(a, stream);
    case FKS_BF16 * 8 + kModeWriteZ: return launch_apply_t<FKS_BF16, kModeWriteZ>(a, stream);
    case FKS_BF16 * 8 + kModeDelta: return launch_apply_t<FKS_BF16, kModeDelta>(a, stream);
    default: return -FKS_ENOTSUP;
  }
}

template <int MODE, bool FULL>
static int launch_apply_bs_m(const ApplyBsArgs& a, void* stream) {
  static PerDevice attr;
  if (int e = ensure_lds_attr(attr, &fks_apply_bs_kernel<MODE, FULL>, kBsLdsBytes)) return e;
  hipLaunchKernelGGL((fks_apply_bs_kernel<MODE, FULL>), dim3((unsigned)(a.split ? a.nchunks / 2 : a.nchunks)),
                     dim3(kBsThreads), kBsLdsBytes, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

template <int MODE>
static int launch_apply_bs_t(const ApplyBsArgs& a, void* stream) {
  // FULL: 32 seeds in each half (a split pass of 32, a two-slice pass of 64)
  const bool full = a.nseeds == (a.split ? kBsSeeds : kBsPassSeeds);
  return full ? launch_apply_bs_m<MODE, true>(a, stream) : launch_apply_bs_m<MODE, false>(a, stream);
}

int launch_apply_bs(const ApplyBsArgs& a, void* stream) {
  if (a.nseeds < 1 || a.nseeds > (a.split ? kBsSeeds : kBsPassSeeds) || a.nchunks < 1 ||
      (a.split && a.nchunks % 2))
    return -FKS_EINVAL;
  int e = ensure_tables();
  if (e) return e;
  switch (a.mode) {
    case kModeUpdate: return launch_apply_bs_t<kModeUpdate>(a, stream);
    case kModeUpdateWd: return launch_apply_bs_t<kModeUpdateWd>(a, stream);
    case kModeUpdateNoWd: return launch_apply_bs_t<kModeUpdateNoWd>(a, stream);
    case kModeUpdateWd0: return launch_apply_bs_t<kModeUpdateWd0>(a, stream);
    case kModeDelta: return launch_apply_bs_t<kModeDelta>(a, stream);
    default: return -FKS_ENOTSUP;
  }
}

template <int MODE>
static int launch_irregular_m(const IrrArgs& a, void* stream) {
  const size_t lds = (size_t)kIrrLogfOff + kLdsLogfBytes;  // tables | windows | wave counters | logf table
  static PerDevice attr;
  if (int e = ensure_lds_attr(attr, &fks_irregular_kernel<MODE>, (int)lds)) return e;
  hipLaunchKernelGGL((fks_irregular_kernel<MODE>), dim3((unsigned)a.nchunks), dim3(kApplyThreads), lds,
                     (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

// Device self check FKS_CHECK_SQRT_DOMAIN: for every u1 = 1 - k 2^-24 the fp32
// Box-Muller can draw, x = -2 cephes_logf(u1); counts the k where radius_sqrt(x) is not
// the correctly rounded square root.  The criterion is exact and uses no square root:
// s = RN(sqrt(x)) iff m_lo^2 < x < m_hi^2 for the midpoints m to s's neighbours (25-bit
// values, squared exactly in double; a 24-bit x never equals such a square).  One count
// per workgroup of 256.
__global__ __launch_bounds__(256) void fks_sqrt_domain_kernel(uint32_t* counts) {
  __shared__ uint32_t bad;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  const uint32_t k = blockIdx.x * 256u + threadIdx.x;
  const float x = -2.0f * cephes_logf(1.0f - (float)k * (1.0f / 16777216.0f));
  const float s = radius_sqrt(x);
  bool ok;
  if (x > 0.0f) {
    const double sd = (double)s;
    const double lo = 0.5 * (sd + (double)__int_as_float(__float_as_int(s) - 1));
    const double hi = 0.5 * (sd + (double)__int_as_float(__float_as_int(s) + 1));
    ok = lo * lo < (double)x && (double)x < hi * hi;
  } else {
    ok = __float_as_uint(s) == __float_as_uint(x);  // sqrt(+-0) = +-0
  }
  if (!ok) atomicAdd(&bad, 1u);
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = bad;
}

// Device self check FKS_CHECK_PHILOX_RADIUS: the torch_rocm stream's radius
// (phx_radius2, the trimmed logf + correctly rounded sqrtf) against ocml's general
// sqrtf(-2 logf(u)) -- the reference's instructions -- on every one of the 2^32 Philox
// words, bit for bit except the sign of a zero radius (the "+ 0" that follows erases
// it).  kSqrtDomainBlocks workgroups of 256, 256 words per thread, one count each.
__global__ __launch_bounds__(256) void fks_philox_radius_kernel(uint32_t* counts) {
  __shared__ uint32_t bad;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  uint32_t n = 0;
  const uint32_t base = (blockIdx.x * 256u + threadIdx.x) * 256u;
  for (uint32_t i = 0; i < 256u; i += 2) {
    const uint32_t x0 = base + i, x1 = base + i + 1;
    const f32x2_t u = {__fmaf_rn((float)x0, 2.3283064e-10f, 2.3283064e-10f),
                       __fmaf_rn((float)x1, 2.3283064e-10f, 2.3283064e-10f)};
    const f32x2_t s = phx_radius2(u);
    const float r0 = phx_radius_ocml(x0), r1 = phx_radius_ocml(x1);
    n += (__float_as_uint(s.x + 0.0f) != __float_as_uint(r0 + 0.0f)) ? 1u : 0u;
    n += (__float_as_uint(s.y + 0.0f) != __float_as_uint(r1 + 0.0f)) ? 1u : 0u;
  }
  if (n) atomicAdd(&bad, n);
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = bad;
}

// Device self check FKS_CHECK_PHILOX_BF16_RADIUS: the largest distance, in f32 ulps, of
// the bf16 fast path's radius (phx_radius2_fast) from ocml's sqrtf(-2 logf(u)) over all
// 2^32 words (both are >= +0, so the distance is the difference of the bit patterns);
// one maximum per workgroup.
__global__ __launch_bounds__(256) void fks_philox_fast_radius_kernel(uint32_t* counts) {
  __shared__ uint32_t worst;
  if (threadIdx.x == 0) worst = 0;
  __syncthreads();
  uint32_t m = 0;
  const uint32_t base = (blockIdx.x * 256u + threadIdx.x) * 256u;
  for (uint32_t i = 0; i < 256u; i += 2) {
    const uint32_t x0 = base + i, x1 = base + i + 1;
    const f32x2_t u = {__fmaf_rn((float)x0, 2.3283064e-10f, 2.3283064e-10f),
                       __fmaf_rn((float)x1, 2.3283064e-10f, 2.3283064e-10f)};
    const f32x2_t s = phx_radius2_fast(u);
    const uint32_t a0 = __float_as_uint(s.x + 0.0f), b0 = __float_as_uint(phx_radius_ocml(x0) + 0.0f);
    const uint32_t a1 = __float_as_uint(s.y + 0.0f), b1 = __float_as_uint(phx_radius_ocml(x1) + 0.0f);
    m = max(m, max(a0 > b0 ? a0 - b0 : b0 - a0, a1 > b1 ? a1 - b1 : b1 - a1));
  }
  atomicMax(&worst, m);
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = worst;
}

int launch_philox_fast_radius_check(uint32_t* counts, void* stream) {
  hipLaunchKernelGGL(fks_philox_fast_radius_kernel, dim3(kSqrtDomainBlocks), dim3(256), 0, (hipStream_t)stream, counts);
  return (int)hipGetLastError();
}

int launch_philox_radius_check(uint32_t* counts, void* stream) {
  hipLaunchKernelGGL(fks_philox_radius_kernel, dim3(kSqrtDomainBlocks), dim3(256), 0, (hipStream_t)stream, counts);
  return (int)hipGetLastError();
}

int launch_sqrt_domain_check(uint32_t* counts, void* stream) {
  hipLaunchKernelGGL(fks_sqrt_domain_kernel, dim3(kSqrtDomainBlocks), dim3(256), 0, (hipStream_t)stream, counts);
  return (int)hipGetLastError();
}

int device_max_threads_per_cu() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 2048;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMaxThreadsPerMultiProcessor, dev) != hipSuccess || n <= 0) return 2048;
  return n;
}

// launches of at most this many seeds take fks_philox_vec_kernel: every launch by default
// (7B bf16 wd 0, 32-seed launches: 4.39 against 4.57 ms per seed in the item loop;
// profiles/r05i_rocm_rate_vec_ab.log); FKS_PHX_VEC_MAXK=0 restores the item loop (A/B)
static int phx_vec_maxk() {
  static const int v = [] {
    const char* s = std::getenv("FKS_PHX_VEC_MAXK");
    return (s && *s) ? std::atoi(s) : kPhxSeeds;
  }();
  return v;
}

template <int MODE>
static int launch_philox_m(const PhiloxArgs& a, void* stream) {
  const int64_t items = a.item_hi - a.item_lo;
  if (items <= 0) return 0;
  if (a.nseeds <= phx_vec_maxk() && a.item_lo % kPhxVec == 0 && items % kPhxVec == 0) {
    const int64_t vitems = items / kPhxVec;
    const int64_t blocks = std::min<int64_t>((vitems + 255) / 256, (int64_t)device_cu_count() * 16);
    const size_t lds = (FKS_PHX_VEC_UNIFORM == 2 && a.nt <= kPhxLdsTensors) ? sizeof(PhxTensor) * (size_t)a.nt : 0;
    hipLaunchKernelGGL((fks_philox_vec_kernel<MODE>), dim3((unsigned)blocks), dim3(256), lds, (hipStream_t)stream, a);
    return (int)hipGetLastError();
  }
  const int64_t blocks = std::min<int64_t>((items + 255) / 256, (int64_t)device_cu_count() * 16);
  hipLaunchKernelGGL((fks_philox_kernel<MODE>), dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

int launch_philox(const PhiloxArgs& a, void* stream) {
  if (a.nseeds < 1 || a.nt < 1) return -FKS_EINVAL;
  switch (a.mode) {
    case kModeUpdate: return launch_philox_m<kModeUpdate>(a, stream);
    case kModeUpdateWd: return launch_philox_m<kModeUpdateWd>(a, stream);
    case kModeUpdateNoWd: return launch_philox_m<kModeUpdateNoWd>(a, stream);
    case kModeUpdateWd0: return launch_philox_m<kModeUpdateWd0>(a, stream);
    case kModeUpdateWdPos0: return launch_philox_m<kModeUpdateWdPos0>(a, stream);
    case kModePerturb: return launch_philox_m<kModePerturb>(a, stream);
    case kModePerturbUpdate: return launch_philox_m<kModePerturbUpdate>(a, stream);
    case kModeWriteZ: return launch_philox_m<kModeWriteZ>(a, stream);
    case kModeDelta: return launch_philox_m<kModeDelta>(a, stream);
    default: return -FKS_ENOTSUP;
  }
}

int launch_irregular(const IrrArgs& a, void* stream) {
  if (a.nseeds < 1 || a.nseeds > kMaxSeedsPerPass) return -FKS_EINVAL;
  int e = ensure_tables();
  if (e) return e;
  switch (a.mode) {
    case kModeUpdate: return launch_irregular_m<kModeUpdate>(a, stream);
    case kModePerturb: return launch_irregular_m<kModePerturb>(a, stream);
    case kModePerturbUpdate: return launch_irregular_m<kModePerturbUpdate>(a, stream);
    case kModeWriteZ: return launch_irregular_m<kModeWriteZ>(a, stream);
    case kModeDelta: return launch_irregular_m<kModeDelta>(a, stream);
    default: return -FKS_ENOTSUP;
  }
}

}  // namespace fks
