// gfx950 VALU issue cost, round 2b: FMA-class forms against the mul/add/cvt forms the
// slice kernel's update chain uses, on NORMAL f32 operands (issue3 fed raw integers,
// i.e. denormal floats).  8 independent chains per wave, 12 or 32 waves per CU; prints
// SIMD cycles per wave-instruction at 2.4 GHz.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

#define BODY(NAME, ASM)                                                                   \
  __global__ void k_##NAME(float* out, int iters) {                                     \
    float a[8], b[8];                                                                    \
    f2 pa[8], pb[8];                                                                     \
    const float s = out[1024], s1 = out[1025];                                           \
    for (int j = 0; j < 8; j++) {                                                        \
      a[j] = 1.0f + 1e-6f * (threadIdx.x * 8 + j);                                       \
      b[j] = (j & 1) ? 0.99999994f : 1.0000001f;                                         \
      pa[j] = f2{a[j], a[j] + 1e-6f};                                                    \
      pb[j] = f2{b[j], b[j]};                                                            \
    }                                                                                    \
    for (int it = 0; it < iters; it++) {                                                 \
      _Pragma("unroll") for (int j = 0; j < 8; j++) { ASM; }                              \
    }                                                                                    \
    float r = 0;                                                                         \
    for (int j = 0; j < 8; j++) r += a[j] + b[j] + pa[j].x + pa[j].y + pb[j].x;                                        \
    if (r == 1234.5f) out[threadIdx.x] = r;                                              \
  }

#define A0 "+v"(a[j])
#define P0 "+v"(pa[j])
#define PB "v"(pb[j])
BODY(mul_f32, asm volatile("v_mul_f32 %0, %1, %0" : A0 : "v"(b[j])))
BODY(mul_f32_s, asm volatile("v_mul_f32 %0, %1, %0" : A0 : "s"(s)))
BODY(add_f32, asm volatile("v_add_f32 %0, %1, %0" : A0 : "v"(b[j])))
BODY(fma_f32, asm volatile("v_fma_f32 %0, %1, %0, %1" : A0 : "v"(b[j])))
BODY(fma_f32_mz, asm volatile("v_fma_f32 %0, %1, %0, %2" : A0 : "v"(b[j]), "s"(s1)))
BODY(fma_f32_s, asm volatile("v_fma_f32 %0, %1, %0, %0" : A0 : "s"(s)))
BODY(fmac_f32, asm volatile("v_fmac_f32 %0, %1, %1" : A0 : "v"(b[j])))
BODY(pk_mul_f32, asm volatile("v_pk_mul_f32 %0, %0, %1" : P0 : PB))
BODY(pk_add_f32, asm volatile("v_pk_add_f32 %0, %0, %1" : P0 : PB))
BODY(pk_fma_f32, asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : P0 : PB))
BODY(pk_fma_f32_s, asm volatile("v_pk_fma_f32 %0, %0, %1, %0 op_sel_hi:[1,0,1]" : P0 : "s"(f2{s, s})))
BODY(cvt_pk0, asm volatile("v_cvt_pk_bf16_f32 %0, 0, %0" : A0))
BODY(cvt_pk2, asm volatile("v_cvt_pk_bf16_f32 %0, %1, %0" : A0 : "v"(b[j])))
BODY(mix_fma_cvt, asm volatile("v_fma_f32 %0, %1, %0, %1\n v_cvt_pk_bf16_f32 %1, 0, %1" : A0, "+v"(b[j])))
BODY(mix_pkfma_cvt, asm volatile("v_pk_fma_f32 %0, %0, %2, %2\n v_cvt_pk_bf16_f32 %1, 0, %1" : P0, "+v"(b[j]) : PB))
BODY(mix_pkmul_cvt, asm volatile("v_pk_mul_f32 %0, %0, %2\n v_cvt_pk_bf16_f32 %1, 0, %1" : P0, "+v"(b[j]) : PB))

typedef void (*K)(float*, int);
int main() {
  float* out;
  (void)hipMalloc(&out, 1 << 20);
  (void)hipMemset(out, 0, 1 << 20);
  const float host[2] = {1.0000001f, -0.0f};
  (void)hipMemcpy(out + 1024, host, sizeof host, hipMemcpyHostToDevice);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
#define E(n, i) {#n, k_##n, i}
  struct { const char* n; K k; int instrs; } ks[] = {
      E(mul_f32, 1), E(mul_f32_s, 1), E(add_f32, 1), E(fma_f32, 1), E(fma_f32_mz, 1), E(fma_f32_s, 1),
      E(fmac_f32, 1), E(pk_mul_f32, 1), E(pk_add_f32, 1), E(pk_fma_f32, 1), E(pk_fma_f32_s, 1), E(cvt_pk0, 1),
      E(cvt_pk2, 1), E(mix_fma_cvt, 2), E(mix_pkfma_cvt, 2), E(mix_pkmul_cvt, 2)};
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
      printf("waves/CU %2d  %-16s %8.3f ms  %.3f cyc/wave-instr/SIMD @2.4GHz\n", wpc, e.n, ms,
             ms * 1e-3 * 2.4e9 / per_simd);
    }
  }
  return 0;
}
