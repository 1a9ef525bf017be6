// gfx950 VALU issue cost vs independent chains per wave (ILP), round 2b: v_cvt_pk_bf16_f32
// and v_pk_mul_f32 on normal operands, C independent chains per wave, 12 / 20 / 32 waves
// per CU, 64 instructions per loop iteration; prints SIMD cycles per wave-instruction at 2.4 GHz.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int C, int OP>
__global__ void k(float* out, int iters) {
  float a[C];
  f2 pa[C];
  const f2 pb = {out[1024], out[1024]};
  for (int j = 0; j < C; j++) {
    a[j] = 1.0f + 1e-6f * (threadIdx.x * C + j);
    pa[j] = f2{a[j], a[j] + 1e-6f};
  }
  const int n = iters / 4;
  for (int it = 0; it < n; it++) {
#pragma unroll
    for (int jj = 0; jj < 64; jj++) {
      const int j = jj % C;
      if (OP == 0) asm volatile("v_cvt_pk_bf16_f32 %0, 0, %0" : "+v"(a[j]));
      if (OP == 1) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(pa[j]) : "v"(pb));
      if (OP == 3) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(pb.x));
      if (OP == 4) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[j]) : "v"(pb.x));
      if (OP == 5) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[j]) : "v"(pb.x));
      if (OP == 6) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[j]) : "v"(pb.x));
      if (OP == 7) asm volatile("v_dot2_f32_bf16 %0, %1, %1, %0" : "+v"(a[j]) : "v"(pb.x));
      if (OP == 8) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(pa[j]) : "v"(pb));
      if (OP == 2) asm volatile("v_pk_mul_f32 %0, %0, %2\n v_cvt_pk_bf16_f32 %1, 0, %1" : "+v"(pa[j]), "+v"(a[j]) : "v"(pb));
    }
  }
  float r = 0;
  for (int j = 0; j < C; j++) r += a[j] + pa[j].x + pa[j].y;
  if (r == 1234.5f) out[threadIdx.x] = r;
}

typedef void (*K)(float*, int);
int main() {
  float* out;
  (void)hipMalloc(&out, 1 << 20);
  (void)hipMemset(out, 0, 1 << 20);
  const float host[1] = {1.0000001f};
  (void)hipMemcpy(out + 1024, host, sizeof host, hipMemcpyHostToDevice);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  struct { const char* n; K k; int chains, instrs; } ks[] = {
      {"cvt", k<1, 0>, 1, 1},   {"cvt", k<2, 0>, 2, 1},   {"cvt", k<4, 0>, 4, 1},   {"cvt", k<8, 0>, 8, 1},
      {"cvt", k<16, 0>, 16, 1}, {"pkmul", k<1, 1>, 1, 1}, {"pkmul", k<2, 1>, 2, 1}, {"pkmul", k<4, 1>, 4, 1},
      {"pkmul", k<8, 1>, 8, 1}, {"pkmul", k<16, 1>, 16, 1}, {"mix", k<2, 2>, 2, 2}, {"mix", k<4, 2>, 4, 2},
      {"mix", k<8, 2>, 8, 2}, {"mix", k<16, 2>, 16, 2}, {"fma", k<8, 3>, 8, 1}, {"mul", k<8, 4>, 8, 1},
      {"add", k<8, 5>, 8, 1}, {"xor", k<8, 6>, 8, 1}, {"dot2", k<8, 7>, 8, 1}, {"pkfma", k<8, 8>, 8, 1},
      {"fma", k<16, 3>, 16, 1}, {"mul", k<16, 4>, 16, 1}, {"xor", k<16, 6>, 16, 1}};
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int iters = 10000;
  for (int wpc : {4, 8, 12, 16, 20, 32}) {
    for (auto& e : ks) {
      const int threads = 64 * (wpc >= 4 ? 4 : wpc), blocks = cus * wpc / 4;
      float ms = 0;
      for (int rep = 0; rep < 2; rep++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(e.k, dim3(blocks), dim3(threads), 0, 0, out, iters);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
      }
      const double per_simd = (double)(iters / 4) * 64 * e.instrs * (blocks * threads / 64) / cus / 4;
      printf("waves/SIMD %2d  %-6s chains %2d  %8.3f ms  %.3f cyc/wave-instr/SIMD @2.4GHz\n", wpc / 4, e.n, e.chains,
             ms, ms * 1e-3 * 2.4e9 / per_simd);
    }
  }
  return 0;
}
