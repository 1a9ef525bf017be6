// VALU issue-cost probe on gfx950: independent chains (8 per wave), 32 or 8 waves per CU.
// Reports SIMD cycles per wave-instruction assuming 2.4 GHz.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define BODY(ASM) \
  template <int W> __global__ void k_##ASM(uint32_t* out, int iters) { \
    uint32_t a[8]; uint32_t s1 = out[1024], s2 = out[1025]; \
    for (int j = 0; j < 8; j++) a[j] = threadIdx.x * 7 + j; \
    for (int it = 0; it < iters; it++) { _Pragma("unroll") for (int j = 0; j < 8; j++) ASM(a[j], s1, s2); } \
    uint32_t s = 0; for (int j = 0; j < 8; j++) s ^= a[j]; if (s == 0x1234) out[threadIdx.x] = s; }

#define XOR32(x, s1, s2) asm volatile("v_xor_b32_e32 %0, %1, %0" : "+v"(x) : "s"(s1))
#define XOR64(x, s1, s2) asm volatile("v_xor_b32_e64 %0, %1, %0" : "+v"(x) : "s"(s1))
#define ANDLIT(x, s1, s2) asm volatile("v_and_b32_e32 %0, 0x9d2c5680, %0" : "+v"(x))
#define BITOP3(x, s1, s2) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x78" : "+v"(x) : "s"(s1), "v"(s2))
#define MULF(x, s1, s2) asm volatile("v_mul_f32_e32 %0, %1, %0" : "+v"(x) : "s"(s1))
#define FMAF(x, s1, s2) asm volatile("v_fma_f32 %0, %1, %0, %2" : "+v"(x) : "s"(s1), "v"(s2))
#define CVTPK(x, s1, s2) asm volatile("v_cvt_pk_bf16_f32 %0, %1, %0" : "+v"(x) : "s"(s1))
#define SHR32(x, s1, s2) asm volatile("v_lshrrev_b32_e32 %0, 7, %0" : "+v"(x))
#define SHR64E(x, s1, s2) asm volatile("v_lshrrev_b32_e64 %0, 7, %0" : "+v"(x))
#define BFEI(x, s1, s2) asm volatile("v_bfe_i32 %0, %0, 0, 1" : "+v"(x))
#define DPP(x, s1, s2) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x))
BODY(XOR32) BODY(XOR64) BODY(ANDLIT) BODY(BITOP3) BODY(MULF) BODY(FMAF) BODY(CVTPK) BODY(SHR32) BODY(SHR64E) BODY(BFEI) BODY(DPP)

typedef void (*K)(uint32_t*, int);
int main() {
  uint32_t* out;
  (void)hipMalloc(&out, 1 << 20);
  (void)hipMemset(out, 0, 1 << 20);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  struct { const char* n; K k; } ks[] = {{"v_xor_b32_e32", k_XOR32<0>}, {"v_xor_b32_e64", k_XOR64<0>},
    {"v_and_b32_e32 lit", k_ANDLIT<0>}, {"v_bitop3_b32", k_BITOP3<0>}, {"v_mul_f32_e32", k_MULF<0>},
    {"v_fma_f32", k_FMAF<0>}, {"v_cvt_pk_bf16_f32", k_CVTPK<0>}, {"v_lshrrev_b32_e32", k_SHR32<0>},
    {"v_lshrrev_b32_e64", k_SHR64E<0>}, {"v_bfe_i32", k_BFEI<0>}, {"v_mov_b32_dpp", k_DPP<0>}};
  const int iters = 20000;
  for (int wpc : {8, 32}) {
    for (auto& e : ks) {
      hipEvent_t a, b;
      (void)hipEventCreate(&a);
      (void)hipEventCreate(&b);
      const int threads = 256, blocks = cus * wpc / 4;
      for (int rep = 0; rep < 2; rep++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(e.k, dim3(blocks), dim3(threads), 0, 0, out, iters);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
      }
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, b);
      const double per_simd = (double)iters * 8 * (blocks * threads / 64) / cus / 4;
      printf("waves/CU %2d  %-20s %7.3f ms  %.3f cyc/wave-instr/SIMD @2.4GHz\n", wpc, e.n, ms, ms * 1e-3 * 2.4e9 / per_simd);
    }
  }
  return 0;
}
