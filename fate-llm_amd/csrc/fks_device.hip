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

// tempering, MT19937RNGEngine.h:141-145
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

// LDS word swizzle: flips bit 3 when bit 5 is set, so the 32 words a half-wave
// reads in the pair phase ({16b + r}, b in 0..3, r in 0..7) hit 32 distinct banks.
__device__ __forceinline__ int swz(int i) { return i ^ (((i >> 5) & 1) << 3); }

// ------------------------------------------------------------------ rounding
__device__ __forceinline__ float rbf(float x) {  // RNE to bf16 and back (v_cvt_pk_bf16_f32)
  return static_cast<float>(static_cast<__bf16>(x));
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

template <>
struct Traits<FKS_F32> {
  using T = float;
  __device__ static float load(const void* p, int64_t i) { return reinterpret_cast<const float*>(p)[i]; }
  __device__ static void store(void* p, int64_t i, float v) { reinterpret_cast<float*>(p)[i] = v; }
  __device__ static float rnd(float x) { return x; }
};

template <>
struct Traits<FKS_BF16> {
  __device__ static float load(const void* p, int64_t i) {
    return __uint_as_float((uint32_t)reinterpret_cast<const uint16_t*>(p)[i] << 16);
  }
  __device__ static void store(void* p, int64_t i, float v) {  // v is bf16-exact
    reinterpret_cast<uint16_t*>(p)[i] = (uint16_t)(__float_as_uint(v) >> 16);
  }
  __device__ static float rnd(float x) { return rbf(x); }
};

template <>
struct Traits<FKS_F16> {
  __device__ static float load(const void* p, int64_t i) {
    return static_cast<float>(reinterpret_cast<const _Float16*>(p)[i]);
  }
  __device__ static void store(void* p, int64_t i, float v) {
    reinterpret_cast<_Float16*>(p)[i] = static_cast<_Float16>(v);
  }
  __device__ static float rnd(float x) { return rhf(x); }
};

// One parameter through one seed.  zo_utils.py:49 (has_wd) / :52 ; optimizer.py:173.
// Each statement is one torch op rounded to the parameter dtype (fp32 opmath).
template <int DT>
__device__ __forceinline__ float apply_one(float p, float z, float g, float lr, float wd, bool has_wd, int mode) {
  using TR = Traits<DT>;
  if (mode == kModeUpdate) {
    float t = TR::rnd(g * z);                 // directional_derivative_value * z
    if (has_wd) t = TR::rnd(t + TR::rnd(wd * p));  // + weight_decay * param.data
    return TR::rnd(p - TR::rnd(lr * t));      // param.data - lr * (...)
  } else if (mode == kModePerturb) {           // lr carries f32(scaling_factor * eps) here
    return TR::rnd(p + TR::rnd(lr * z));      // param.data + scaling_factor * eps * z
  }
  return z;
}

// ------------------------------------------------------------------ jump kernel
// grid (ceil(nchunks / chunks_per_wg), nseeds); block kJumpThreads; LDS kJumpXLen words.
__global__ __launch_bounds__(kJumpThreads) void fks_jump_kernel(JumpArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t xs[];
  const int tid = threadIdx.x;
  const int k = blockIdx.y;
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
  __syncthreads();
  // x[n] = x[n-227] ^ twist(x[n-624], x[n-623]): 227 independent words per step
  for (int base = kMtN; base < kJumpXLen; base += kMtN - kMtM) {
    const int n = base + tid;
    if (tid < kMtN - kMtM && n < kJumpXLen) xs[n] = xs[n - (kMtN - kMtM)] ^ mt_twist(xs[n - kMtN], xs[n - kMtN + 1]);
    __syncthreads();
  }
  const int c0 = blockIdx.x * a.chunks_per_wg;
  const int c1 = min(c0 + a.chunks_per_wg, a.nchunks);
  const int w = tid;
  for (int c = c0; c < c1; c++) {
    const int64_t b = a.chunk_block[c];
    uint32_t acc = 0;
    if (b == 0) {
      if (w < kMtN) acc = xs[w];
    } else {
      const uint64_t* poly = a.polys + (size_t)c * 312;
      const uint32_t* yb = xs + 1 + w;  // y[i + w] = x[i + w + 1]
      for (int wd = 0; wd < 312; wd++) {
        uint64_t bits = poly[wd];
        const int i0 = wd * 64;
        while (bits) {
          const int i = i0 + __builtin_ctzll(bits);
          bits &= bits - 1;
          if (w < kMtN) acc ^= yb[i];
        }
      }
    }
    if (w < kMtN) a.states[((size_t)k * a.nchunks + c) * kMtN + w] = acc;
  }
}

// ------------------------------------------------------------------ apply kernel
// In-place twist of nseeds windows (MT19937RNGEngine.h:164-175).  Word i of the new
// block needs OLD words i and i+1 plus word i+397 (old, i < 227) or i-227 (new), so
// the 624 words form 3 dependency phases [0,227) [227,454) [454,624).  Within a
// phase thread T walks a contiguous run of L items in ascending order (L odd, so
// the 64 lanes hit distinct LDS banks): it reads old word i+1 before writing word
// i+1 itself, and only the old word just past its run -- written by thread T+1 --
// is read up front; a barrier then separates those reads (and every lane's reads
// of the previous block) from the first write.  Word 623 pairs with the NEW word 0
// (MT19937RNGEngine.h:174).
__device__ __forceinline__ void twist_all(uint32_t* st, int nseeds, int tid) {
  int a[3], b[3], L[3];
  uint32_t pre[3];
#pragma unroll
  for (int ph = 0; ph < 3; ph++) {
    const int lo = ph == 0 ? 0 : (ph == 1 ? 227 : 454);
    const int len = ph == 2 ? 170 : 227;
    const int total = len * nseeds;
    L[ph] = ((total + kApplyThreads - 1) / kApplyThreads) | 1;
    a[ph] = tid * L[ph];
    b[ph] = min(a[ph] + L[ph], total);
    pre[ph] = 0;
    if (a[ph] < b[ph]) {
      const int last = b[ph] - 1;
      const int k = last / len;
      const int i = lo + (last - k * len);
      if (i + 1 < kMtN) pre[ph] = st[k * kMtN + swz(i + 1)];
    }
  }
  __syncthreads();
#pragma unroll
  for (int ph = 0; ph < 3; ph++) {
    const int lo = ph == 0 ? 0 : (ph == 1 ? 227 : 454);
    const int len = ph == 2 ? 170 : 227;
    if (a[ph] < b[ph]) {
      int k = a[ph] / len;
      int i = lo + (a[ph] - k * len);
      uint32_t* s = st + k * kMtN;
      uint32_t u = s[swz(i)];
      for (int it = a[ph]; it < b[ph]; it++) {
        uint32_t v;
        if (i == kMtN - 1) v = s[swz(0)];
        else if (it == b[ph] - 1) v = pre[ph];
        else v = s[swz(i + 1)];
        const uint32_t m = s[swz(i < kMtN - kMtM ? i + kMtM : i - (kMtN - kMtM))];
        s[swz(i)] = m ^ mt_twist(u, v);
        i++;
        if (i == lo + len) {
          k++;
          i = lo;
          s = st + k * kMtN;
          if (it + 1 < b[ph]) u = s[swz(i)];
        } else {
          u = v;
        }
      }
    }
    __syncthreads();
  }
}

__constant__ float c_tab_bf16[3 * 256];  // R | C | S, set once from fks::tables()

template <int DT, int MODE>
__global__ __launch_bounds__(kApplyThreads, 2) void fks_apply_kernel(ApplyArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* st = lds;                                                     // [nseeds][624], swizzled
  float* gs = reinterpret_cast<float*>(lds + kMaxSeedsPerPass * kMtN);    // [kMaxSeedsPerPass]
  float* tabR = gs + kMaxSeedsPerPass;                                    // bf16 radius R[a]
  float2* tabCS = reinterpret_cast<float2*>(tabR + 256);                  // bf16 (C[b], S[b])
  const int tid = threadIdx.x;
  const int c = blockIdx.x;
  const int nseeds = a.nseeds;
  const int64_t b0 = a.chunk_block[c], b1 = a.chunk_block[c + 1];

  if constexpr (DT == FKS_BF16) {
    for (int i = tid; i < 256; i += kApplyThreads) {
      tabR[i] = c_tab_bf16[i];
      tabCS[i] = make_float2(c_tab_bf16[256 + i], c_tab_bf16[512 + i]);
    }
  }
  if (tid < nseeds) gs[tid] = a.g[tid];
  for (int idx = tid; idx < nseeds * kMtN; idx += kApplyThreads) {
    const int k = idx / kMtN, i = idx - k * kMtN;
    st[k * kMtN + swz(i)] = a.states[((size_t)k * a.nchunks + c) * kMtN + i];
  }
  __syncthreads();

  // Thread q < 312 owns Box-Muller pair q of every block: 16-block q/8, slot q%8,
  // i.e. block words j1 = 16*(q/8) + q%8 and j1 + 8 (DistributionTemplates.h:141-146).
  const bool lane_on = tid < kMtN / 2;
  const int j1 = 16 * (tid >> 3) + (tid & 7);
  const int sj1 = swz(j1), sj2 = swz(j1 + 8);

  // first segment that ends after this lane's first position
  int cur = 0;
  {
    const int64_t s1 = (int64_t)kMtN * b0 + j1;
    int lo = 0, hi = a.nsegs;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (a.segs[mid].start + a.segs[mid].numel <= s1) lo = mid + 1; else hi = mid;
    }
    cur = lo;
  }

  for (int64_t b = b0; b < b1; b++) {
    twist_all(st, nseeds, tid);  // the words of stream block b, raw (untempered)
    const int64_t s1 = (int64_t)kMtN * b + j1;
    while (cur < a.nsegs && s1 >= a.segs[cur].start + a.segs[cur].numel) cur++;
    if (lane_on && cur < a.nsegs && s1 >= a.segs[cur].start) {
      const DevSeg* sg = a.segs + cur;
      void* ptr = reinterpret_cast<void*>(sg->ptr);
      const int64_t e1 = s1 - sg->start;
      const float lr = sg->lr, wd = sg->wd;
      const bool has_wd = (sg->flags & FKS_HAS_WD) != 0;
      float p1 = 0.0f, p2 = 0.0f;
      if (MODE != kModeWriteZ) {
        p1 = Traits<DT>::load(ptr, e1);
        p2 = Traits<DT>::load(ptr, e1 + 8);
      }
#pragma unroll 2
      for (int k = 0; k < nseeds; k++) {
        const uint32_t w1 = mt_temper(st[k * kMtN + sj1]);
        const uint32_t w2 = mt_temper(st[k * kMtN + sj2]);
        float z1, z2;
        if constexpr (DT == FKS_F32) {
          z_pair_f32(w1, w2, z1, z2);
        } else {
          // normal_fill_16<BFloat16>: z = bf16(R[a] * C[b]) * 1 + 0 (std, mean)
          const float r = tabR[w1 & 0xFFu];
          const float2 cs = tabCS[w2 & 0xFFu];
          z1 = rbf(r * cs.x) + 0.0f;
          z2 = rbf(r * cs.y) + 0.0f;
        }
        const float g = gs[k];
        p1 = apply_one<DT>(p1, z1, g, lr, wd, has_wd, MODE);
        p2 = apply_one<DT>(p2, z2, g, lr, wd, has_wd, MODE);
      }
      Traits<DT>::store(ptr, e1, p1);
      Traits<DT>::store(ptr, e1 + 8, p2);
    }
    // no barrier here: the next twist_all's first barrier orders these LDS reads
    // before its first write
  }
}

}  // namespace

// ------------------------------------------------------------------ launchers
static size_t apply_lds_bytes() {
  return sizeof(uint32_t) * (size_t)kMaxSeedsPerPass * kMtN + sizeof(float) * kMaxSeedsPerPass +
         sizeof(float) * 256 + sizeof(float2) * 256;
}

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
  const size_t lds = sizeof(uint32_t) * (size_t)kJumpXLen;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&fks_jump_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  dim3 grid((unsigned)((a.nchunks + a.chunks_per_wg - 1) / a.chunks_per_wg), (unsigned)nseeds);
  hipLaunchKernelGGL(fks_jump_kernel, grid, dim3(kJumpThreads), lds, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

template <int DT, int MODE>
static int launch_apply_t(const ApplyArgs& a, void* stream) {
  const size_t lds = apply_lds_bytes();
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&fks_apply_kernel<DT, MODE>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  hipLaunchKernelGGL((fks_apply_kernel<DT, MODE>), dim3((unsigned)a.nchunks), dim3(kApplyThreads), lds,
                     (hipStream_t)stream, a);
  return (int)hipGetLastError();
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
