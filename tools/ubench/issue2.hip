// Issue-cost and LDS-lookup probe on gfx950 (round 2): what the slice kernel's op mix
// costs at 2-3 waves per SIMD.
//   VALU: 8 independent chains per wave of one instruction (packed f32, cvt, sdwa, ...),
//         reported as SIMD cycles per wave-instruction at the measured clock-free rate
//         (ms -> cycles at 2.4 GHz; compare ratios, not absolutes).
//   LDS:  random 8-bit-indexed lookups into a 256-entry table (ds_read_b32 / _b64) in the
//         plain layout and in a per-lane-bank replicated layout; ds_bpermute_b32.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

#define BODY(NAME, ASM)                                                                  \
  __global__ void k_##NAME(uint32_t* out, int iters) {                                  \
    f2 a[8];                                                                            \
    const f2 s = {__uint_as_float(out[1024]), __uint_as_float(out[1025])};               \
    for (int j = 0; j < 8; j++) a[j] = f2{(float)threadIdx.x + j, (float)j};             \
    for (int it = 0; it < iters; it++) {                                                \
      _Pragma("unroll") for (int j = 0; j < 8; j++) ASM(a[j], s);                        \
    }                                                                                   \
    uint32_t r = 0;                                                                     \
    for (int j = 0; j < 8; j++) r ^= __float_as_uint(a[j].x) ^ __float_as_uint(a[j].y); \
    if (r == 0x1234) out[threadIdx.x] = r;                                              \
  }

#define PKMUL(x, s) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(x) : "v"(s))
#define PKADD(x, s) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(x) : "v"(s))
#define PKFMA(x, s) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(s))
#define MUL2(q, t) asm volatile("v_mul_f32 %0, %0, %2\n v_mul_f32 %1, %1, %3" : "+v"(q.x), "+v"(q.y) : "v"(t.x), "v"(t.y))
#define CVT2(q, t) asm volatile("v_cvt_pk_bf16_f32 %0, %0, 0\n v_cvt_pk_bf16_f32 %1, %1, 0" : "+v"(q.x), "+v"(q.y))
#define SDWA2(q, t) asm volatile("v_lshlrev_b32_sdwa %0, 2, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n v_lshlrev_b32_sdwa %1, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(q.x), "+v"(q.y))
#define AND2(q, t) asm volatile("v_and_b32 %0, 0xffff0000, %0\n v_lshlrev_b32 %1, 16, %1" : "+v"(q.x), "+v"(q.y))
BODY(pkmul, PKMUL) BODY(pkadd, PKADD) BODY(pkfma, PKFMA) BODY(mul2, MUL2) BODY(cvt2, CVT2) BODY(sdwa2, SDWA2)
BODY(and2, AND2)

// LDS lookups: each lane does `iters` x 8 lookups with indices from an xorshift stream;
// mode 0: ds_read_b32 of a 256 x 4 B table; 1: ds_read_b64 of a 256 x 8 B table;
// 2: ds_read_b32 replicated per lane bank (entry e of lane L at (e*32 + L%32)*4);
// 3: ds_read_b64 replicated (entry e of lane L at (e*32 + L%32)*8); 4: ds_bpermute_b32.
template <int MODE>
__global__ void k_lds(uint32_t* out, int iters) {
  extern __shared__ uint32_t tab[];
  const int n = MODE == 2 ? 256 * 32 : MODE == 3 ? 256 * 64 : 512;
  for (int i = threadIdx.x; i < n; i += blockDim.x) tab[i] = i * 2654435761u;
  __syncthreads();
  uint32_t xs[8], acc = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    uint32_t x = (threadIdx.x * 8 + j + 1) * 2654435761u + blockIdx.x * 40503u;
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    xs[j] = x;
  }
  const uint32_t L = threadIdx.x & 31;
  for (int it = 0; it < iters; it++) {
    uint32_t v[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      xs[j] += 0x9E3779B9u;  // one add per lookup: the bank pattern is random per lane
      const uint32_t e = xs[j] >> 24;
      if (MODE == 0) v[j] = tab[e];
      if (MODE == 1) { const uint2 w = reinterpret_cast<const uint2*>(tab)[e]; v[j] = w.x + w.y; }
      if (MODE == 2) v[j] = tab[e * 32 + L];
      if (MODE == 3) { const uint2 w = reinterpret_cast<const uint2*>(tab)[e * 32 + L]; v[j] = w.x + w.y; }
      if (MODE == 4) v[j] = __builtin_amdgcn_ds_bpermute((int)((e & 63) << 2), (int)xs[j]);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) acc += v[j];
  }
  if (acc == 0x1234567) out[threadIdx.x] = acc;
}

typedef void (*K)(uint32_t*, int);
int main() {
  uint32_t* out;
  (void)hipMalloc(&out, 1 << 20);
  (void)hipMemset(out, 0, 1 << 20);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  struct { const char* n; K k; int instrs; } ks[] = {
      {"v_pk_mul_f32", k_pkmul, 1}, {"v_pk_add_f32", k_pkadd, 1}, {"v_pk_fma_f32", k_pkfma, 1},
      {"v_mul_f32", k_mul2, 2}, {"v_cvt_pk_bf16_f32(x,0)", k_cvt2, 2}, {"v_lshlrev_b32_sdwa", k_sdwa2, 2},
      {"v_and/v_lshl", k_and2, 2}};
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int iters = 20000;
  for (int wpc : {8, 12, 16, 32}) {
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
      const double per_simd = (double)iters * 8 * e.instrs * (blocks * threads / 64) / cus / 4;
      printf("VALU waves/CU %2d  %-26s %8.3f ms  %.3f cyc/wave-instr/SIMD @2.4GHz\n", wpc, e.n, ms,
             ms * 1e-3 * 2.4e9 / per_simd);
    }
  }
  struct { const char* n; K k; size_t lds; } ls[] = {
      {"ds_read_b32 random 1KB", k_lds<0>, 2048}, {"ds_read_b64 random 2KB", k_lds<1>, 2048},
      {"ds_read_b32 per-lane-bank 32KB", k_lds<2>, 32768}, {"ds_read_b64 per-lane-bank 64KB", k_lds<3>, 65536},
      {"ds_bpermute_b32", k_lds<4>, 2048}};
  for (int wpc : {8, 16}) {
    for (auto& e : ls) {
      const int threads = 256, blocks = cus * wpc / 4;
      float ms = 0;
      for (int rep = 0; rep < 2; rep++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(e.k, dim3(blocks), dim3(threads), e.lds, 0, out, iters / 4);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
      }
      // blocks/CU resident at once: LDS-limited for the 64 KB table
      const double per_cu = (double)(iters / 4) * 8 * (blocks * threads / 64) / cus;
      printf("LDS  waves/CU %2d  %-32s %8.3f ms  %.3f CU-cycles per wave-instr @2.4GHz\n", wpc, e.n, ms,
             ms * 1e-3 * 2.4e9 / per_cu);
    }
  }
  return 0;
}
