// gfx950 VALU issue-cost table (round 2): for each instruction form, 8 independent
// chains per wave, 12 or 32 waves per CU; prints SIMD cycles per wave-instruction at the
// clock the run holds (GRBM-free: ms -> cycles at 2.4 GHz; compare rows, and read the
// dual-issue share from SQ_ACTIVE_INST_VALU2 under rocprofv3).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define BODY(NAME, ASM)                                                                   \
  __global__ void k_##NAME(uint32_t* out, int iters) {                                   \
    uint32_t a[8], b[8];                                                                 \
    const uint32_t s = out[1024];                                                        \
    for (int j = 0; j < 8; j++) { a[j] = threadIdx.x * 7 + j; b[j] = threadIdx.x ^ (j * 977); } \
    for (int it = 0; it < iters; it++) {                                                 \
      _Pragma("unroll") for (int j = 0; j < 8; j++) { ASM; }                              \
    }                                                                                    \
    uint32_t r = 0;                                                                      \
    for (int j = 0; j < 8; j++) r ^= a[j] ^ b[j];                                        \
    if (r == 0x1234) out[threadIdx.x] = r;                                               \
  }

#define A0 "+v"(a[j])
BODY(mul_f32, asm volatile("v_mul_f32 %0, %1, %0" : A0 : "v"(b[j])))
BODY(add_f32, asm volatile("v_add_f32 %0, %1, %0" : A0 : "v"(b[j])))
BODY(fma_f32, asm volatile("v_fma_f32 %0, %1, %0, %1" : A0 : "v"(b[j])))
BODY(and_sgpr, asm volatile("v_and_b32 %0, %1, %0" : A0 : "s"(s)))
BODY(and_lit, asm volatile("v_and_b32 %0, 0xffff0000, %0" : A0))
BODY(lshl16, asm volatile("v_lshlrev_b32 %0, 16, %0" : A0))
BODY(xor_v, asm volatile("v_xor_b32 %0, %1, %0" : A0 : "v"(b[j])))
BODY(add_u32, asm volatile("v_add_u32 %0, %1, %0" : A0 : "v"(b[j])))
BODY(bitop3, asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : A0 : "v"(b[j]), "s"(s)))
BODY(bfe_u32, asm volatile("v_bfe_u32 %0, %0, 8, 8" : A0))
BODY(perm_b32, asm volatile("v_perm_b32 %0, %0, %1, %2" : A0 : "v"(b[j]), "s"(s)))
BODY(cndmask, asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : A0 : "v"(b[j])))
BODY(lshl_or, asm volatile("v_lshl_or_b32 %0, %0, 2, %1" : A0 : "v"(b[j])))
BODY(cvt_pk0, asm volatile("v_cvt_pk_bf16_f32 %0, 0, %0" : A0))
BODY(cvt_pk2, asm volatile("v_cvt_pk_bf16_f32 %0, %1, %0" : A0 : "v"(b[j])))
BODY(sdwa_sh, asm volatile("v_lshlrev_b32_sdwa %0, 2, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : A0))
BODY(dpp_mov, asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : A0))
BODY(cvt_f32_bf16, asm volatile("v_cvt_f32_bf16 %0, %0" : A0))
BODY(cvt_f32_bf16_sdwa, asm volatile("v_cvt_f32_bf16_sdwa %0, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1" : A0))
BODY(pk_mul_f32, asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(*(uint64_t*)&a[j & 6]) : "v"(*(uint64_t*)&b[j & 6])))
BODY(mix_mul_cvt, asm volatile("v_mul_f32 %0, %1, %0\n v_cvt_pk_bf16_f32 %1, 0, %1" : A0, "+v"(b[j])))
BODY(mix_and_cvt, asm volatile("v_and_b32 %0, %2, %0\n v_cvt_pk_bf16_f32 %1, 0, %1" : A0, "+v"(b[j]) : "s"(s)))
BODY(mix_mul_pk, asm volatile("v_mul_f32 %0, %1, %0\n v_pk_mul_f32 %2, %2, %2" : A0, "+v"(b[j]), "+v"(*(uint64_t*)&a[(j + 2) & 6])))

typedef void (*K)(uint32_t*, int);
int main() {
  uint32_t* out;
  (void)hipMalloc(&out, 1 << 20);
  (void)hipMemset(out, 0, 1 << 20);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
#define E(n, i) {#n, k_##n, i}
  struct { const char* n; K k; int instrs; } ks[] = {
      E(mul_f32, 1), E(add_f32, 1), E(fma_f32, 1), E(and_sgpr, 1), E(and_lit, 1), E(lshl16, 1), E(xor_v, 1),
      E(add_u32, 1), E(bitop3, 1), E(bfe_u32, 1), E(perm_b32, 1), E(cndmask, 1), E(lshl_or, 1), E(cvt_pk0, 1),
      E(cvt_pk2, 1), E(sdwa_sh, 1), E(dpp_mov, 1), E(cvt_f32_bf16, 1), E(cvt_f32_bf16_sdwa, 1), E(pk_mul_f32, 1),
      E(mix_mul_cvt, 2), E(mix_and_cvt, 2), E(mix_mul_pk, 2)};
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int iters = 20000;
  for (int wpc : {12, 32}) {
    for (auto& e : ks) {
      const int threads = 256, blocks = cus * wpc / 4;
      float ms = 0;
      for (int rep = 0; rep < 2; rep++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(e.k, dim3(blocks), dim3(threads), 0, 0, out, iters);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
      }
      const double per_simd = (double)iters * 8 * e.instrs * (blocks * threads / 64) / cus / 4;
      printf("waves/CU %2d  %-20s %8.3f ms  %.3f cyc/wave-instr/SIMD @2.4GHz\n", wpc, e.n, ms,
             ms * 1e-3 * 2.4e9 / per_simd);
    }
  }
  return 0;
}
