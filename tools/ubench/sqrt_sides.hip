// Which side does v_sqrt_f32 miss the correctly rounded square root on, over the two
// radius domains the codec draws: the torch_rocm stream's x = -2 log(u) for all 2^32
// Philox words (u = fma(w, 2^-32, 2^-32), the trimmed logf of phx_radius2) and the CPU
// stream's x = -2 cephes_logf(1 - k 2^-24) for all 2^24 k.  Counts the inputs where the
// +-1 ulp correction steps down (rm <= 0: v_sqrt_f32 above) and up (rp > 0: below).  If
// one side never occurs on a domain, its half of the correction is dead there.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__device__ float phx_x(uint32_t w) {
  const float u = __fmaf_rn((float)w, 2.3283064e-10f, 2.3283064e-10f);
  const float y = __builtin_amdgcn_logf(u);
  const float m2hi = __uint_as_float(0xbfb17217u), m2lo = __uint_as_float(0xb3f7d1cfu);
  const float r = y * m2hi;
  float e = __fmaf_rn(y, m2hi, -r);
  e = __fmaf_rn(m2lo, y, e);
  return r + e;
}

__device__ float cephes_logf(float x) {  // as fks_device.hip (x in [2^-24, 1])
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

__device__ void sides(float x, unsigned long long* c) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sm = __int_as_float(__float_as_int(s) - 1), sp = __int_as_float(__float_as_int(s) + 1);
  const float rm = __fmaf_rn(-sm, s, x), rp = __fmaf_rn(-sp, s, x);
  if (rm <= 0.0f) atomicAdd(&c[0], 1ull);
  if (rp > 0.0f) atomicAdd(&c[1], 1ull);
}

__global__ void phx(unsigned long long* c) {
  const uint32_t base = (blockIdx.x * 256u + threadIdx.x) * 256u;
  for (uint32_t i = 0; i < 256u; i++) sides(phx_x(base + i), c);
}
__global__ void cpu(unsigned long long* c) {
  const uint32_t k = blockIdx.x * 256u + threadIdx.x;
  sides(-2.0f * cephes_logf(1.0f - (float)k * (1.0f / 16777216.0f)), c + 2);
}

int main() {
  unsigned long long* c;
  (void)hipMalloc(&c, 4 * sizeof(unsigned long long));
  (void)hipMemset(c, 0, 4 * sizeof(unsigned long long));
  hipLaunchKernelGGL(phx, dim3(1 << 16), dim3(256), 0, 0, c);
  hipLaunchKernelGGL(cpu, dim3(1 << 16), dim3(256), 0, 0, c);
  unsigned long long h[4];
  (void)hipMemcpy(h, c, sizeof h, hipMemcpyDeviceToHost);
  printf("philox words (2^32): v_sqrt_f32 above %llu, below %llu\n", h[0], h[1]);
  printf("cpu fp32 radius (2^24): v_sqrt_f32 above %llu, below %llu\n", h[2], h[3]);
  return 0;
}
