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

#include "fks_internal.h"

namespace fks {
namespace {

// ------------------------------------------------------------------ MT19937 pieces
__device__ __forceinline__ uint32_t mt_twist(uint32_t u, uint32_t v) {
  return (((u & 0x80000000u) | (v & 0x7fffffffu)) >> 1) ^ ((v & 1u) ? kMatrixA : 0u);
}

// v_bitop3_b32 truth tables (LOP3 convention: f(0xF0, 0xCC, 0xAA))
constexpr unsigned kXorAnd = 0x78;  // a ^ (b & c)
constexpr unsigned kXorMask = 0x28; // (a ^ b) & c

// tempering, MT19937RNGEngine.h:141-145; each "y ^= (y << s) & M" is one shift + one bitop3
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y = __builtin_amdgcn_bitop3_b32(y, y << 7, 0x9d2c5680u, kXorAnd);
  y = __builtin_amdgcn_bitop3_b32(y, y << 15, 0xefc60000u, kXorAnd);
  y ^= (y >> 18);
  return y;
}

// low 8 bits of the tempered word (the bf16 uniform), times 4 (a byte offset into a
// 256-entry f32 table): ((y ^ (y >> 18)) & 0xFF) << 2 = ((y << 2) ^ (y >> 16)) & 0x3FC
__device__ __forceinline__ uint32_t mt_temper_u8x4(uint32_t y) {
  y ^= (y >> 11);
  y = __builtin_amdgcn_bitop3_b32(y, y << 7, 0x9d2c5680u, kXorAnd);
  y = __builtin_amdgcn_bitop3_b32(y, y << 15, 0xefc60000u, kXorAnd);
  return __builtin_amdgcn_bitop3_b32(y << 2, y >> 16, 0x3FCu, kXorMask);
}

// ------------------------------------------------------------------ rounding
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
// RNE to bf16, result kept as the f32 with the same value: ONE v_cvt_pk_bf16_f32 with
// a zero low half (hi = bf16(x), lo = bf16(0) = 0x0000).  NaN stays NaN.
__device__ __forceinline__ float rbf(float x) {
  const f32x2_t v = {0.0f, x};
  return __builtin_bit_cast(float, __builtin_convertvector(v, bf16x2_t));
}
__device__ __forceinline__ float rhf(float x) {  // RNE to f16 and back
  return static_cast<float>(static_cast<_Float16>(x));
}

// ------------------------------------------------------------------ fp32 Box-Muller
// normal_fill_16_AVX2 (DistributionTemplates.h:88-106) with log256_ps / sincos256_ps
// (avx_mathfun.h:90-160, 426-520) restated lane by lane; the fmaf()s are the
// contractions GCC applies in libtorch's AVX2/AVX512 build (pinned bit-exact by
// oracle/fks_oracle.c against the reference's golden streams).
__device__ __forceinline__ float cephes_logf(float x) {  // x in [2^-24, 1]
  int32_t imm0 = (int32_t)(__float_as_uint(x) >> 23);
  x = __uint_as_float((__float_as_uint(x) & ~0x7f800000u) | 0x3f000000u);
  imm0 -= 0x7f;
  float e = (float)imm0;
  e = e + 1.0f;
  const bool mask = x < 0.707106781186547524f;
  const float tmp = mask ? x : 0.0f;
  x = x - 1.0f;
  e = e - (mask ? 1.0f : 0.0f);
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

__device__ __forceinline__ void cephes_sincosf(float xin, float& s, float& c) {
  uint32_t sign_bit_sin = __float_as_uint(xin) & 0x80000000u;
  float x = __uint_as_float(__float_as_uint(xin) & 0x7fffffffu);
  float y = x * 1.27323954473516f;
  int32_t imm2 = (int32_t)y;  // cvttps: truncation
  imm2 = (imm2 + 1) & ~1;
  y = (float)imm2;
  const int32_t imm4 = imm2 - 2;
  const uint32_t swap_sign_bit_sin = ((uint32_t)(imm2 & 4)) << 29;
  const bool poly_mask = (imm2 & 2) == 0;
  x = __fmaf_rn(y, -0.78515625f, x);
  x = __fmaf_rn(y, -2.4187564849853515625e-4f, x);
  x = __fmaf_rn(y, -3.77489497744594108e-8f, x);
  const uint32_t sign_bit_cos = ((uint32_t)(~imm4 & 4)) << 29;
  sign_bit_sin ^= swap_sign_bit_sin;
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
  const float ysin2 = poly_mask ? ys : 0.0f;
  const float ysin1 = poly_mask ? 0.0f : yc;
  ys = ys - ysin2;
  yc = yc - ysin1;
  const float xmm1 = ysin1 + ysin2;
  const float xmm2 = yc + ys;
  s = __uint_as_float(__float_as_uint(xmm1) ^ sign_bit_sin);
  c = __uint_as_float(__float_as_uint(xmm2) ^ sign_bit_cos);
}

// z pair (element j, element j+8) from the two tempered words of a 16-block
__device__ __forceinline__ void z_pair_f32(uint32_t w1, uint32_t w2, float& z1, float& z2) {
  const float d1 = (float)(w1 & 0xFFFFFFu) * (1.0f / 16777216.0f);  // uniform_real<float>
  const float d2 = (float)(w2 & 0xFFFFFFu) * (1.0f / 16777216.0f);
  const float u1 = 1.0f - d1;
  const float radius = sqrtf(-2.0f * cephes_logf(u1));  // _mm256_sqrt_ps: correctly rounded
  const float theta = 6.28318548202514648438f * d2;      // (float)(2.0f * c10::pi<double>)
  float s, c;
  cephes_sincosf(theta, s, c);
  z1 = radius * c + 0.0f;  // _mm256_fmadd_ps(n1, std=1, mean=0)
  z2 = radius * s + 0.0f;
}

// ------------------------------------------------------------------ per-dtype traits
template <int DT>
struct Traits;

typedef __attribute__((address_space(1))) float gf32;
typedef __attribute__((address_space(1))) uint16_t gu16;
typedef __attribute__((address_space(1))) _Float16 gf16;

template <>
struct Traits<FKS_F32> {
  __device__ static float load(uint64_t p, int64_t i) { return reinterpret_cast<const gf32*>(p)[i]; }
  __device__ static void store(uint64_t p, int64_t i, float v) { reinterpret_cast<gf32*>(p)[i] = v; }
  __device__ static float rnd(float x) { return x; }
};

template <>
struct Traits<FKS_BF16> {
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
  __device__ static float load(uint64_t p, int64_t i) { return static_cast<float>(reinterpret_cast<const gf16*>(p)[i]); }
  __device__ static void store(uint64_t p, int64_t i, float v) { reinterpret_cast<gf16*>(p)[i] = static_cast<_Float16>(v); }
  __device__ static float rnd(float x) { return rhf(x); }
};

// One parameter through one seed.  zo_utils.py:49 (has_wd) / :52 ; optimizer.py:173.
// Each statement is one torch op rounded to the parameter dtype (fp32 opmath).
template <int DT>
__device__ __forceinline__ float apply_one(float p, float z, float g, float lr, float wd, bool has_wd, int mode) {
  using TR = Traits<DT>;
  if (mode == kModeUpdate) {
    const float gz = TR::rnd(g * z);                    // directional_derivative_value * z
    const float t2 = TR::rnd(gz + TR::rnd(wd * p));     // + weight_decay * param.data
    const float t = has_wd ? t2 : gz;                   // (select: keeps the seed loop branch-free)
    return TR::rnd(p - TR::rnd(lr * t));                // param.data - lr * (...)
  } else if (mode == kModePerturb) {           // lr carries f32(scaling_factor * eps) here
    return TR::rnd(p + TR::rnd(lr * z));      // param.data + scaling_factor * eps * z
  }
  return z;
}

// ------------------------------------------------------------------ jump kernel
// grid (nseeds, ceil(nchunks / chunks_per_wg)); block kJumpThreads (8 waves).
// LDS holds the seed's x[0..20560] (+ slack read by the last sliding window) at a
// 3-word offset, so that y = x + 1 is 16-byte aligned.  Each wave evaluates the jump
// of one chunk at a time: lane l < 52 owns window words w = 12l .. 12l+11 and sweeps
// the 19937 coefficients of c(t) = t^J mod phi four at a time, keeping
// y[i + 12l .. i + 12l + 15] in a 16-register sliding window fed by one ds_read_b128
// per step:  acc[j] ^= y[i + d + 12l + j] & -c[i + d]   (d = 0..3, j = 0..11).
constexpr int kJumpLanes = 52;          // 52 lanes x 12 words = 624
constexpr int kJumpXOff = 3;            // x at word 3 -> y = x + 1 at word 4 (16 B aligned)
constexpr int kJumpLdsWords = kJumpXOff + kJumpXLen + 64;  // + over-read slack of the last window

__device__ __forceinline__ uint4 lds_b128(const uint32_t* p) { return *reinterpret_cast<const uint4*>(p); }

__global__ __launch_bounds__(kJumpThreads) void fks_jump_kernel(JumpArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_j[];
  uint32_t* xs = lds_j + kJumpXOff;
  const int tid = threadIdx.x;
  const int k = blockIdx.x;
  const uint64_t seed = a.seeds[k];
  // mt19937::init_with_uint32 (MT19937RNGEngine.h:156-162): a serial recurrence
  if (tid == 0) {
    uint32_t s = (uint32_t)(seed & 0xffffffffu);
    xs[0] = s;
    for (int j = 1; j < kMtN; j++) {
      s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)j;
      xs[j] = s;
    }
  }
  for (int j = kJumpXLen + tid; j < kJumpLdsWords - kJumpXOff; j += kJumpThreads) xs[j] = 0u;
  __syncthreads();
  // x[n] = x[n-227] ^ twist(x[n-624], x[n-623]): 227 independent words per step
  for (int base = kMtN; base < kJumpXLen; base += kMtN - kMtM) {
    const int n = base + tid;
    if (tid < kMtN - kMtM && n < kJumpXLen) xs[n] = xs[n - (kMtN - kMtM)] ^ mt_twist(xs[n - kMtN], xs[n - kMtN + 1]);
    __syncthreads();
  }
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const uint32_t* yb = xs + 1 + 12 * lane;  // y[12 lane]
  const int c0 = blockIdx.y * a.chunks_per_wg;
  const int c1 = min(c0 + a.chunks_per_wg, a.nchunks);
  for (int c = c0 + wave; c < c1; c += kJumpThreads / 64) {
    const int64_t b = a.chunk_block[c];
    uint32_t acc[12];
#pragma unroll
    for (int j = 0; j < 12; j++) acc[j] = 0u;
    if (lane < kJumpLanes) {
      if (b == 0) {
#pragma unroll
        for (int j = 0; j < 12; j++) acc[j] = xs[12 * lane + j];
      } else {
        const uint64_t* poly = a.polys + (size_t)c * 312;  // wave-uniform: scalar loads
        uint32_t win[16];
        {
          const uint4 q0 = lds_b128(yb), q1 = lds_b128(yb + 4), q2 = lds_b128(yb + 8);
          win[0] = q0.x; win[1] = q0.y; win[2] = q0.z; win[3] = q0.w;
          win[4] = q1.x; win[5] = q1.y; win[6] = q1.z; win[7] = q1.w;
          win[8] = q2.x; win[9] = q2.y; win[10] = q2.z; win[11] = q2.w;
          const uint4 q3 = lds_b128(yb + 12);
          win[12] = q3.x; win[13] = q3.y; win[14] = q3.z; win[15] = q3.w;
        }
        uint64_t next = poly[0];
        for (int wd = 0; wd < 312; wd++) {
          const uint64_t bits = next;
          if (wd + 1 < 312) next = poly[wd + 1];  // prefetch the next 64 coefficients
          const uint32_t lo = (uint32_t)bits, hi = (uint32_t)(bits >> 32);
          const uint32_t* yw = yb + 64 * wd;
#pragma unroll
          for (int q = 0; q < 16; q++) {
            // window = y[64 wd + 4q + 12 lane + 0..15], stored rotated by 4q (mod 16)
            const uint4 nx = lds_b128(yw + 4 * q + 16);
            const int rot = (4 * q) & 15;
            const uint32_t word = q < 8 ? lo : hi;
#pragma unroll
            for (int d = 0; d < 4; d++) {
              // all-ones if coefficient 64 wd + 4q + d is set (scalar bit-field extract)
              const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)word, (4 * q + d) & 31, 1);
#pragma unroll
              for (int j = 0; j < 12; j++) acc[j] = __builtin_amdgcn_bitop3_b32(acc[j], win[(rot + j + d) & 15], m, kXorAnd);
            }
            win[(rot + 0) & 15] = nx.x;
            win[(rot + 1) & 15] = nx.y;
            win[(rot + 2) & 15] = nx.z;
            win[(rot + 3) & 15] = nx.w;
          }
        }
      }
      uint32_t* out = a.states + ((size_t)k * a.nchunks + c) * kMtN + 12 * lane;
#pragma unroll
      for (int j = 0; j < 12; j += 4) *reinterpret_cast<uint4*>(out + j) = make_uint4(acc[j], acc[j + 1], acc[j + 2], acc[j + 3]);
    }
  }
}

// ------------------------------------------------------------------ apply kernel
// In-place twist of nseeds windows (MT19937RNGEngine.h:164-175).  Word i of the new
// block needs OLD words i and i+1 plus word i+397 (old, i < 227) or i-227 (new), so
// the 624 words form 3 dependency phases [0,227) [227,454) [454,624); word 623 pairs
// with the NEW word 0 (MT19937RNGEngine.h:174).  Items are dealt round-robin over
// the 320 threads; every phase reads into registers, barriers, then writes (word i
// reads word i+1, which another thread writes in the same phase).  Item addresses
// depend only on (thread, nseeds), so they are computed once per kernel and the
// three reads use immediate offsets.
constexpr int kR12 = (227 * kMaxSeedsPerPass + kApplyThreads - 1) / kApplyThreads;  // items / thread, phases 1-2
constexpr int kR3 = (170 * kMaxSeedsPerPass + kApplyThreads - 1) / kApplyThreads;   // items / thread, phase 3

struct TwistPlan {
  int a12[kR12];   // byte offset of (window k, word i') for phases 1-2
  int a3[kR3];     // byte offset of (window k, word i'') for phase 3 (word 454 + i'')
  uint32_t last3;  // bit r: item r of phase 3 is word 623 (its partner is the NEW word 0)
};

// Items are dealt round-robin; an item past the last seed lands in a window that is
// either unused in this pass or the spare window kMaxSeedsPerPass, so every item runs
// unconditionally (no exec-masked branches, all LDS reads of a phase in flight at once).
__device__ __forceinline__ void twist_plan(TwistPlan& P, int tid, int st_base) {
#pragma unroll
  for (int r = 0; r < kR12; r++) {
    const int it = tid + r * kApplyThreads;
    const int k = it / 227, i = it - k * 227;
    P.a12[r] = st_base + 4 * (min(k, kMaxSeedsPerPass) * kMtN + i);  // overflow items: spare window
  }
  P.last3 = 0;
#pragma unroll
  for (int r = 0; r < kR3; r++) {
    const int it = tid + r * kApplyThreads;
    const int k = it / 170, i = it - k * 170;
    P.a3[r] = st_base + 4 * (min(k, kMaxSeedsPerPass) * kMtN + i);
    if (i == 169) P.last3 |= 1u << r;
  }
}

__device__ __forceinline__ uint32_t lds_u32(const uint8_t* base, int off) {
  return *reinterpret_cast<const uint32_t*>(base + off);
}
__device__ __forceinline__ void lds_st(uint8_t* base, int off, uint32_t v) {
  *reinterpret_cast<uint32_t*>(base + off) = v;
}

__device__ __forceinline__ void twist_all(uint8_t* lds, const TwistPlan& P) {
  uint32_t nv[kR12];
  // phase 1: words [0, 227): m = x[i + 397] (old)
#pragma unroll
  for (int r = 0; r < kR12; r++) {
    const int o = P.a12[r];
    nv[r] = lds_u32(lds, o + 4 * kMtM) ^ mt_twist(lds_u32(lds, o), lds_u32(lds, o + 4));
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kR12; r++) lds_st(lds, P.a12[r], nv[r]);
  __syncthreads();
  // phase 2: words [227, 454): m = x[i - 227] (new, phase 1)
#pragma unroll
  for (int r = 0; r < kR12; r++) {
    const int o = P.a12[r];
    nv[r] = lds_u32(lds, o) ^ mt_twist(lds_u32(lds, o + 4 * 227), lds_u32(lds, o + 4 * 228));
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kR12; r++) lds_st(lds, P.a12[r] + 4 * 227, nv[r]);
  __syncthreads();
  // phase 3: words [454, 624): m = x[i - 227] (new, phase 2); word 623 pairs with new x[0]
#pragma unroll
  for (int r = 0; r < kR3; r++) {
    const int o = P.a3[r];
    const int ov = ((P.last3 >> r) & 1u) ? o - 4 * 169 - 4 * 455 : o;  // ov + 4*455 -> x[0] of this window
    nv[r] = lds_u32(lds, o + 4 * 227) ^ mt_twist(lds_u32(lds, o + 4 * 454), lds_u32(lds, ov + 4 * 455));
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kR3; r++) lds_st(lds, P.a3[r] + 4 * 454, nv[r]);
  __syncthreads();
}

__constant__ float c_tab_bf16[3 * 256];  // R | C | S, set once from fks::tables()

// LDS: [R[256] f32 | (C,S)[256] f32x2 | windows (kMaxSeedsPerPass + 1) x 624 u32]
constexpr int kLdsTabBytes = 256 * 4 + 256 * 8;
constexpr int kLdsStBytes = (kMaxSeedsPerPass + 1) * kMtN * 4;

// z pair of seed k for this lane's 16-block slot: raw words j1, j1+8 -> (z_j, z_{j+8})
template <int DT>
__device__ __forceinline__ void z_pair(const uint8_t* lds, uint32_t r1, uint32_t r2, float& z1, float& z2) {
  if constexpr (DT == FKS_F32) {
    z_pair_f32(mt_temper(r1), mt_temper(r2), z1, z2);
  } else {
    // normal_fill_16<BFloat16>: z = bf16(R[a] * C[b]) * 1 + 0 (std, mean).  R*C is exact
    // in f32 (8-bit x 8-bit significands) and fma(R, C, +0) turns -0 into +0 like "+ mean".
    const uint32_t a4 = mt_temper_u8x4(r1), b4 = mt_temper_u8x4(r2);
    const float r = *reinterpret_cast<const float*>(lds + a4);
    const float2 cs = *reinterpret_cast<const float2*>(lds + 1024 + 2 * b4);
    z1 = rbf(__fmaf_rn(r, cs.x, 0.0f));
    z2 = rbf(__fmaf_rn(r, cs.y, 0.0f));
  }
}

// Seeds [k0, k0 + U): all LDS reads and z first (independent across seeds), then the
// sequential per-element update chain in seed order.
template <int DT, int MODE, int U>
__device__ __forceinline__ void pair_group(const uint8_t* lds, int st_off, int k0, const float* g, float lr,
                                           float wd, bool has_wd, float& p1, float& p2) {
  uint32_t r1[U], r2[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    r1[u] = lds_u32(lds, st_off + (k0 + u) * (kMtN * 4));
    r2[u] = lds_u32(lds, st_off + (k0 + u) * (kMtN * 4) + 32);
  }
  float z1[U], z2[U];
#pragma unroll
  for (int u = 0; u < U; u++) z_pair<DT>(lds, r1[u], r2[u], z1[u], z2[u]);
#pragma unroll
  for (int u = 0; u < U; u++) {
    p1 = apply_one<DT>(p1, z1[u], g[k0 + u], lr, wd, has_wd, MODE);
    p2 = apply_one<DT>(p2, z2[u], g[k0 + u], lr, wd, has_wd, MODE);
  }
}

template <int DT, int MODE, bool FULL>
__global__ __launch_bounds__(kApplyThreads, (kApplyWgPerCu * kApplyThreads + 255) / 256) void fks_apply_kernel(ApplyArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds32[];
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds32);
  const int tid = threadIdx.x;
  const int c = blockIdx.x;
  const int nseeds = FULL ? kMaxSeedsPerPass : a.nseeds;
  const int64_t b0 = a.chunk_block[c], b1 = a.chunk_block[c + 1];

  if constexpr (DT == FKS_BF16) {
    float* tabR = reinterpret_cast<float*>(lds);
    float2* tabCS = reinterpret_cast<float2*>(lds + 1024);
    for (int i = tid; i < 256; i += kApplyThreads) {
      tabR[i] = c_tab_bf16[i];
      tabCS[i] = make_float2(c_tab_bf16[256 + i], c_tab_bf16[512 + i]);
    }
  }
  uint32_t* st = reinterpret_cast<uint32_t*>(lds + kLdsTabBytes);
  for (int idx = tid; idx < nseeds * kMtN; idx += kApplyThreads) {
    const int k = idx / kMtN, i = idx - k * kMtN;
    st[k * kMtN + i] = a.states[((size_t)k * a.nchunks + c) * kMtN + i];
  }
  TwistPlan plan;
  twist_plan(plan, tid, kLdsTabBytes);
  // per-seed multipliers: wave-uniform, kept in SGPRs for the whole kernel
  float gk[kMaxSeedsPerPass];
#pragma unroll
  for (int k = 0; k < kMaxSeedsPerPass; k++)
    gk[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(k < nseeds ? a.g[k] : 0.0f)));
  __syncthreads();

  // Thread q < 312 owns Box-Muller pair q of every block: 16-block q/8, slot q%8,
  // i.e. block words j1 = 16*(q/8) + q%8 and j1 + 8 (DistributionTemplates.h:141-146).
  const bool lane_on = tid < kMtN / 2;
  const int j1 = 16 * (tid >> 3) + (tid & 7);
  const int st_off = kLdsTabBytes + 4 * j1;

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
  };
  load_seg();

  // software pipeline: block b+1's parameters are fetched before block b's Box-Muller
  struct Slot { uint64_t ptr; int64_t e1; float lr, wd; bool wdf, on; float p1, p2; };
  auto fetch = [&](int64_t b) {
    Slot sl;
    const int64_t s1 = (int64_t)kMtN * b + j1;
    while (s1 >= seg_end) { cur++; load_seg(); }
    sl.on = lane_on && s1 >= seg_start;
    sl.ptr = seg_ptr; sl.e1 = s1 - seg_start; sl.lr = seg_lr; sl.wd = seg_wd; sl.wdf = seg_wdf;
    sl.p1 = 0.0f; sl.p2 = 0.0f;
    if (MODE != kModeWriteZ && sl.on) {
      sl.p1 = Traits<DT>::load(sl.ptr, sl.e1);
      sl.p2 = Traits<DT>::load(sl.ptr, sl.e1 + 8);
    }
    return sl;
  };
  Slot nxt = fetch(b0);

#ifndef FKS_DIAG
#define FKS_DIAG 0  // diagnostic builds only: 1 = twist only, 2 = Box-Muller/update only
#endif
  for (int64_t b = b0; b < b1; b++) {
    Slot sl = nxt;
    if (FKS_DIAG != 2) twist_all(lds, plan);  // the raw words of stream block b (sl's loads in flight meanwhile)
    if (FKS_DIAG == 2) __syncthreads();
    if (b + 1 < b1) nxt = fetch(b + 1);
    if (sl.on && FKS_DIAG != 1) {
      float p1 = sl.p1, p2 = sl.p2;
      if constexpr (FULL) {
#pragma unroll
        for (int k0 = 0; k0 + 4 <= kMaxSeedsPerPass; k0 += 4)
          pair_group<DT, MODE, 4>(lds, st_off, k0, gk, sl.lr, sl.wd, sl.wdf, p1, p2);
        constexpr int kTail = kMaxSeedsPerPass % 4;
        if constexpr (kTail > 0)
          pair_group<DT, MODE, kTail>(lds, st_off, kMaxSeedsPerPass - kTail, gk, sl.lr, sl.wd, sl.wdf, p1, p2);
      } else {
        for (int k = 0; k < nseeds; k++) pair_group<DT, MODE, 1>(lds, st_off, k, gk, sl.lr, sl.wd, sl.wdf, p1, p2);
      }
      Traits<DT>::store(sl.ptr, sl.e1, p1);
      Traits<DT>::store(sl.ptr, sl.e1 + 8, p2);
    }
    // no barrier here: the next twist's first barrier orders these LDS reads before
    // its first write
  }
}

}  // namespace

// ------------------------------------------------------------------ launchers
static size_t apply_lds_bytes() { return (size_t)kLdsTabBytes + (size_t)kLdsStBytes; }

int device_cu_count() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) return 256;
  return n;
}

static int ensure_tables() {
  static int done = 0;  // per process; the constant symbol lives in this code object
  if (done) return 0;
  const Tables& t = tables();
  float buf[768];
  for (int i = 0; i < 256; i++) {
    buf[i] = t.r_bf16[i];
    buf[256 + i] = t.c_bf16[i];
    buf[512 + i] = t.s_bf16[i];
  }
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_tab_bf16), buf, sizeof(buf), 0, hipMemcpyHostToDevice);
  if (e != hipSuccess) return (int)e;
  done = 1;
  return 0;
}

int launch_jump(const JumpArgs& a, int nseeds, void* stream) {
  const size_t lds = sizeof(uint32_t) * (size_t)kJumpLdsWords;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&fks_jump_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  dim3 grid((unsigned)nseeds, (unsigned)((a.nchunks + a.chunks_per_wg - 1) / a.chunks_per_wg));
  hipLaunchKernelGGL(fks_jump_kernel, grid, dim3(kJumpThreads), lds, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

template <int DT, int MODE, bool FULL>
static int launch_apply_f(const ApplyArgs& a, void* stream) {
  const size_t lds = apply_lds_bytes();
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&fks_apply_kernel<DT, MODE, FULL>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  hipLaunchKernelGGL((fks_apply_kernel<DT, MODE, FULL>), dim3((unsigned)a.nchunks), dim3(kApplyThreads), lds,
                     (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

template <int DT, int MODE>
static int launch_apply_t(const ApplyArgs& a, void* stream) {
  return a.nseeds == kMaxSeedsPerPass ? launch_apply_f<DT, MODE, true>(a, stream)
                                      : launch_apply_f<DT, MODE, false>(a, stream);
}

int launch_apply(int dtype, const ApplyArgs& a, void* stream) {
  if (dtype == FKS_BF16) {
    int e = ensure_tables();
    if (e) return e;
  }
  switch (dtype * 4 + a.mode) {
    case FKS_F32 * 4 + kModeUpdate: return launch_apply_t<FKS_F32, kModeUpdate>(a, stream);
    case FKS_F32 * 4 + kModePerturb: return launch_apply_t<FKS_F32, kModePerturb>(a, stream);
    case FKS_F32 * 4 + kModeWriteZ: return launch_apply_t<FKS_F32, kModeWriteZ>(a, stream);
    case FKS_BF16 * 4 + kModeUpdate: return launch_apply_t<FKS_BF16, kModeUpdate>(a, stream);
    case FKS_BF16 * 4 + kModePerturb: return launch_apply_t<FKS_BF16, kModePerturb>(a, stream);
    case FKS_BF16 * 4 + kModeWriteZ: return launch_apply_t<FKS_BF16, kModeWriteZ>(a, stream);
    default: return -FKS_ENOTSUP;
  }
}

}  // namespace fks
