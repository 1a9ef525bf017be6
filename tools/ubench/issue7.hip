// gfx950 issue cost of the torch_rocm (Philox + Box-Muller) kernel's instruction forms:
// 32x32->64 multiplies (v_mad_u64_u32 against an SGPR constant, v_mul_hi/lo_u32), 24-bit
// multiplies, a 3-input xor (v_bitop3_b32 0x96) against two v_xor_b32, the transcendentals
// the Box-Muller pair uses, and a mix of one v_mad_u64_u32 with N plain VALU ops (does a
// long-latency multiply block its SIMD or only its wave?).  8 independent chains per wave,
// 64 instructions per loop iteration; prints SIMD cycles per wave-instruction at 2.4 GHz.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

template <int C, int OP>
__global__ void k(float* out, int iters, uint32_t m) {
  uint32_t a[C];
  uint64_t w[C];
  float f[C], g[C];
  const float fb = out[1024];
  const uint32_t ub = __float_as_uint(out[1025]);
  for (int j = 0; j < C; j++) {
    a[j] = threadIdx.x * C + j + 0x12345u;
    w[j] = a[j];
    f[j] = 0.5f + 1e-6f * (threadIdx.x * C + j);
    g[j] = f[j];
  }
  const int n = iters / 4;
  for (int it = 0; it < n; it++) {
#pragma unroll
    for (int jj = 0; jj < 64; jj++) {
      const int j = jj % C;
      if (OP == 0) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(w[j]) : "v"((uint32_t)w[j]), "s"(m) : "vcc");
      if (OP == 1) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[j]) : "s"(m));
      if (OP == 2) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[j]) : "s"(m));
      if (OP == 3) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[j]) : "v"(ub));
      if (OP == 4) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[j]) : "v"(ub));
      if (OP == 5) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[j]) : "v"(ub), "s"(m));
      if (OP == 6) asm volatile("v_xor_b32 %0, %1, %0\n v_xor_b32 %0, %0, %2" : "+v"(a[j]) : "s"(m), "v"(ub));
      if (OP == 7) asm volatile("v_log_f32 %0, %0" : "+v"(f[j]));
      if (OP == 8) asm volatile("v_sqrt_f32 %0, %0" : "+v"(f[j]));
      if (OP == 9) asm volatile("v_sin_f32 %0, %0" : "+v"(f[j]));
      if (OP == 10) asm volatile("v_cvt_f32_u32 %0, %1" : "=v"(f[j]) : "v"(a[j]));
      if (OP == 11) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[j]) : "v"(fb));
      if (OP == 12)  // one 64-bit multiply + 4 independent xors of another chain
        asm volatile("v_mad_u64_u32 %[w], vcc, %[lo], %[m], 0\n v_xor_b32 %[a], %[a], %[u]\n v_xor_b32 %[a], %[a], %[u]\n"
                     " v_xor_b32 %[a], %[a], %[u]\n v_xor_b32 %[a], %[a], %[u]"
                     : [w] "=v"(w[j]), [a] "+v"(a[j]) : [lo] "v"((uint32_t)w[j]), [m] "s"(m), [u] "v"(ub) : "vcc");
      if (OP == 13)  // one 64-bit multiply + 4 independent fmas
        asm volatile("v_mad_u64_u32 %[w], vcc, %[lo], %[m], 0\n v_fma_f32 %[f], %[f], %[b], %[b]\n"
                     " v_fma_f32 %[f], %[f], %[b], %[b]\n v_fma_f32 %[f], %[f], %[b], %[b]\n v_fma_f32 %[f], %[f], %[b], %[b]"
                     : [w] "=v"(w[j]), [f] "+v"(f[j]) : [lo] "v"((uint32_t)w[j]), [m] "s"(m), [b] "v"(fb) : "vcc");
      if (OP == 14)  // one transcendental + 4 independent fmas
        asm volatile("v_log_f32 %[g], %[g]\n v_fma_f32 %[f], %[f], %[b], %[b]\n v_fma_f32 %[f], %[f], %[b], %[b]\n"
                     " v_fma_f32 %[f], %[f], %[b], %[b]\n v_fma_f32 %[f], %[f], %[b], %[b]"
                     : [g] "+v"(g[j]), [f] "+v"(f[j]) : [b] "v"(fb));
    }
  }
  float r = 0;
  for (int j = 0; j < C; j++) r += (float)a[j] + (float)(uint32_t)w[j] + (float)(w[j] >> 32) + f[j] + g[j];
  if (r == 1234.5f) out[threadIdx.x] = r;
}

typedef void (*K)(float*, int, uint32_t);
int main() {
  float* out;
  (void)hipMalloc(&out, 1 << 20);
  (void)hipMemset(out, 0, 1 << 20);
  const float host[2] = {1.0000001f, 3.0f};
  (void)hipMemcpy(out + 1024, host, sizeof host, hipMemcpyHostToDevice);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  struct { const char* n; K k; int instrs; } ks[] = {
      {"mad_u64_u32", k<8, 0>, 1}, {"mul_hi_u32", k<8, 1>, 1}, {"mul_lo_u32", k<8, 2>, 1},
      {"mul_u32_u24", k<8, 3>, 1}, {"mul_hi_u32_u24", k<8, 4>, 1}, {"bitop3(xor3)", k<8, 5>, 1},
      {"2x xor_b32", k<8, 6>, 2}, {"log_f32", k<8, 7>, 1}, {"sqrt_f32", k<8, 8>, 1}, {"sin_f32", k<8, 9>, 1},
      {"cvt_f32_u32", k<8, 10>, 1}, {"fma_f32", k<8, 11>, 1}, {"mad64+4xor", k<8, 12>, 5},
      {"mad64+4fma", k<8, 13>, 5}, {"log+4fma", k<8, 14>, 5}};
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int iters = 10000;
  for (int wpc : {8, 16, 32}) {
    for (auto& e : ks) {
      const int threads = 256, blocks = cus * wpc / 4;
      float ms = 0;
      for (int rep = 0; rep < 2; rep++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(e.k, dim3(blocks), dim3(threads), 0, 0, out, iters, 0xD2511F53u);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
      }
      const double per_simd = (double)(iters / 4) * 64 * e.instrs * (blocks * threads / 64) / cus / 4;
      printf("waves/SIMD %2d  %-16s %8.3f ms  %.3f cyc/wave-instr/SIMD @2.4GHz  (%.3f per asm statement)\n", wpc / 4,
             e.n, ms, ms * 1e-3 * 2.4e9 / per_simd, ms * 1e-3 * 2.4e9 / per_simd * e.instrs);
    }
  }
  return 0;
}
