// Which SIMD does each wave of a 12-wave (768-thread) workgroup land on?  One workgroup per
// CU (160 KB of dynamic LDS, like the slice kernel); prints wave -> SIMD for a few
// workgroups from HW_REG_HW_ID (SIMD_ID bits [5:4], CU_ID bits [11:8]).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
__global__ __launch_bounds__(768, 1) void k(uint32_t* out) {
  extern __shared__ uint32_t lds[];
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 12 + threadIdx.x / 64] = hw;
  lds[threadIdx.x] = hw;
  __syncthreads();
  if (lds[(threadIdx.x + 64) % 768] == 0xdeadbeef) out[0] = 1;
}
int main() {
  uint32_t* d;
  const int wgs = 256;
  (void)hipMalloc(&d, wgs * 12 * 4);
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL(k, dim3(wgs), dim3(768), 160 * 1024, 0, d);
  (void)hipDeviceSynchronize();
  uint32_t h[wgs * 12];
  (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  int pattern_count[4][4] = {{0}};  // [wave % 4][simd] histogram over all workgroups, waves 0..11
  for (int b = 0; b < wgs; b++) {
    if (b < 6) {
      printf("wg %3d cu/se %2u/%u simd:", b, (h[b * 12] >> 8) & 15, (h[b * 12] >> 13) & 7);
      for (int w = 0; w < 12; w++) printf(" %u", (h[b * 12 + w] >> 4) & 3);
      printf("\n");
    }
  }
  // same-SIMD classes: for each workgroup, group waves by SIMD
  int same_mod4 = 0, seq3 = 0;
  for (int b = 0; b < wgs; b++) {
    bool m4 = true, s3 = true;
    for (int w = 0; w < 12; w++) {
      if (((h[b * 12 + w] >> 4) & 3) != ((h[b * 12 + (w % 4)] >> 4) & 3)) m4 = false;
      if (((h[b * 12 + w] >> 4) & 3) != ((h[b * 12 + 3 * (w / 3)] >> 4) & 3)) s3 = false;
    }
    same_mod4 += m4;
    seq3 += s3;
  }
  printf("workgroups where waves w, w+4, w+8 share a SIMD: %d / %d; where waves 3i..3i+2 share one: %d / %d\n",
         same_mod4, wgs, seq3, wgs);
  return 0;
}
