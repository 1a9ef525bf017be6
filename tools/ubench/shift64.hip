// Issue-rate probe on gfx950: v_lshrrev_b64 vs v_lshrrev_b32 vs v_bitop3_b32 vs v_pk_fma_f32
// (independent chains, 8 per wave, many waves).  Prints ns per wave-instruction per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int OP>
__global__ void probe(uint64_t* out, int iters) {
  uint64_t a[8];
  for (int j = 0; j < 8; j++) a[j] = (uint64_t)(threadIdx.x * 7 + j) * 0x9E3779B97F4A7C15ull;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (OP == 0) asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(a[j]));
      if (OP == 1) {
        uint32_t lo = (uint32_t)a[j];
        asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(lo));
        a[j] = (a[j] & 0xffffffff00000000ull) | lo;
      }
      if (OP == 2) {
        uint32_t lo = (uint32_t)a[j], hi = (uint32_t)(a[j] >> 32);
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x78" : "+v"(lo) : "v"(hi), "s"(0x1fffffu));
        a[j] = ((uint64_t)hi << 32) | lo;
      }
      if (OP == 3) asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(a[j]));
      if (OP == 4) asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(a[j]));
      if (OP == 5) {
        uint32_t lo = (uint32_t)a[j];
        asm volatile("v_cvt_pk_bf16_f32 %0, %0, 0" : "+v"(lo));
        a[j] = (a[j] & 0xffffffff00000000ull) | lo;
      }
    }
  }
  uint64_t s = 0;
  for (int j = 0; j < 8; j++) s ^= a[j];
  if (s == 0x1234) out[threadIdx.x] = s;
}

int main() {
  uint64_t* out;
  (void)hipMalloc(&out, 1 << 20);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int iters = 20000, blocks = cus * 8, threads = 256;  // 32 waves per CU
  const char* names[] = {"v_lshrrev_b64", "v_lshrrev_b32", "v_bitop3_b32", "v_pk_fma_f32", "v_lshlrev_b64",
                         "v_cvt_pk_bf16_f32"};
  for (int op = 0; op < 6; op++) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int rep = 0; rep < 2; rep++) {
      (void)hipEventRecord(a);
      switch (op) {
        case 0: hipLaunchKernelGGL(probe<0>, dim3(blocks), dim3(threads), 0, 0, out, iters); break;
        case 1: hipLaunchKernelGGL(probe<1>, dim3(blocks), dim3(threads), 0, 0, out, iters); break;
        case 2: hipLaunchKernelGGL(probe<2>, dim3(blocks), dim3(threads), 0, 0, out, iters); break;
        case 3: hipLaunchKernelGGL(probe<3>, dim3(blocks), dim3(threads), 0, 0, out, iters); break;
        case 4: hipLaunchKernelGGL(probe<4>, dim3(blocks), dim3(threads), 0, 0, out, iters); break;
        case 5: hipLaunchKernelGGL(probe<5>, dim3(blocks), dim3(threads), 0, 0, out, iters); break;
      }
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
    }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double wave_instr_per_cu = (double)iters * 8 * (blocks * threads / 64) / cus;
    printf("%-20s %8.3f ms  %.3f cycles@2.4GHz per wave-instr per SIMD\n", names[op], ms,
           ms * 1e-3 * 2.4e9 / (wave_instr_per_cu / 4));
  }
  return 0;
}
