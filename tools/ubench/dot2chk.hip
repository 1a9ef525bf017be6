// Is v_dot2_f32_bf16(x, (1,1), 0) the IEEE f32 sum of the two bf16 halves of x (one RNE
// rounding), over random bf16 pairs of every exponent gap?  Counts mismatches vs v_add_f32.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
__global__ void k(uint32_t* bad, uint32_t* ex, uint64_t n) {
  uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h = i * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 32;
    uint32_t lo = (uint32_t)h & 0xffffu, hi = (uint32_t)(h >> 16) & 0xffffu;
    // restrict exponents to a window so sums are neither inf nor nan often
    lo = (lo & 0x807fu) | ((uint32_t)(0x30 + ((h >> 40) & 0x1f)) << 7);
    hi = (hi & 0x807fu) | ((uint32_t)(0x30 + ((h >> 48) & 0x1f)) << 7);
    if (((h >> 56) & 15) == 0) lo = 0x8000u & lo;  // some signed zeros
    const uint32_t x = lo | (hi << 16), ones = 0x3f803f80u;
    float d;
    asm volatile("v_dot2_f32_bf16 %0, %1, %2, 0" : "=v"(d) : "v"(x), "v"(ones));
    float r;
    const float a = __uint_as_float(lo << 16), b = __uint_as_float(hi << 16);
    asm volatile("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    if (__float_as_uint(d) != __float_as_uint(r)) {
      const uint32_t c = atomicAdd(bad, 1u);
      if (c < 8) { ex[3 * c] = x; ex[3 * c + 1] = __float_as_uint(d); ex[3 * c + 2] = __float_as_uint(r); }
    }
  }
}
int main() {
  uint32_t *bad, *ex;
  (void)hipMalloc(&bad, 4); (void)hipMalloc(&ex, 96);
  (void)hipMemset(bad, 0, 4);
  const uint64_t n = 1ull << 30;
  hipLaunchKernelGGL(k, dim3(4096), dim3(256), 0, 0, bad, ex, n);
  uint32_t hb = 0, he[24] = {0};
  (void)hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(he, ex, 96, hipMemcpyDeviceToHost);
  printf("dot2 vs add: %u mismatches of %llu\n", hb, (unsigned long long)n);
  for (int c = 0; c < 8 && c < (int)hb; c++) printf("  x=%08x dot2=%08x add=%08x\n", he[3 * c], he[3 * c + 1], he[3 * c + 2]);
  return 0;
}
