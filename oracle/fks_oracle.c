/*
 * fks_oracle.c -- CPU restatement of FATE-LLM's FedKSeed codec arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker, never the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * liboracle.so.  The product path (fate-llm_amd/csrc, libfks.so) never links it.
 *
 * What it restates (the reference's hot path is pure Python over torch, so the
 * arithmetic lives in the pinned third-party dependency torch; installed
 * 2.10.0+rocm7.0, reference pins torch==2.3.1 at python/setup.py:34):
 *
 *   zo_utils.directional_derivative_step   python/fate_llm/algo/fedkseed/zo_utils.py:23-54
 *   ZerothOrderOptimizer.random_perturb_parameters
 *                                          python/fate_llm/algo/fedkseed/optimizer.py:152-173
 *   torch.manual_seed -> at::mt19937       torch/include/ATen/core/MT19937RNGEngine.h:115-175
 *   torch.normal (CPU) -> normal_kernel    torch/include/ATen/native/cpu/DistributionTemplates.h:88-256
 *   log256_ps / sincos256_ps               torch/include/ATen/native/cpu/avx_mathfun.h:90-160,426-520
 *   uniform_real / normal_distribution     torch/include/ATen/core/TransformationHelper.h:84-90,
 *                                          torch/include/ATen/core/DistributionsHelper.h:99-221
 *
 * Pinned against golden vectors captured by importing the reference
 * (tests/golden/make_golden.py); see tests/test_oracle_golden.py.
 *
 * Build: oracle/Makefile (gcc, -ffp-contract=off; every fused multiply-add is an
 * explicit fmaf() mirroring the contraction GCC performs in libtorch's AVX2 build).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* MT19937 exactly as at::mt19937 (MT19937RNGEngine.h:115-175)                */
/* ------------------------------------------------------------------------- */
#define MT_N 624
#define MT_M 397
#define MT_MATRIX_A 0x9908b0dfu
#define MT_UMASK 0x80000000u
#define MT_LMASK 0x7fffffffu

typedef struct {
    uint32_t state[MT_N];
    int32_t left;
    int32_t next;
    /* CPUGeneratorImpl's cached second Box-Muller sample of
     * normal_distribution<double> (DistributionsHelper.h:189-221);
     * reset by torch.manual_seed. */
    int32_t has_cached_double;
    int32_t pad_;
    double cached_double;
} fko_gen;

void fko_seed(fko_gen *g, uint64_t seed) {
    g->state[0] = (uint32_t)(seed & 0xffffffffu);
    for (int j = 1; j < MT_N; j++)
        g->state[j] = 1812433253u * (g->state[j - 1] ^ (g->state[j - 1] >> 30)) + (uint32_t)j;
    g->left = 1;
    g->next = 0;
    g->has_cached_double = 0;
    g->cached_double = 0.0;
}

static inline uint32_t mt_twist(uint32_t u, uint32_t v) {
    return (((u & MT_UMASK) | (v & MT_LMASK)) >> 1) ^ ((v & 1u) ? MT_MATRIX_A : 0u);
}

static void mt_next_state(fko_gen *g) {
    uint32_t *p = g->state;
    g->left = MT_N;
    g->next = 0;
    for (int j = MT_N - MT_M + 1; --j; p++) *p = p[MT_M] ^ mt_twist(p[0], p[1]);
    for (int j = MT_M; --j; p++) *p = p[MT_M - MT_N] ^ mt_twist(p[0], p[1]);
    *p = p[MT_M - MT_N] ^ mt_twist(p[0], g->state[0]);
}

uint32_t fko_random(fko_gen *g) {
    if (--(g->left) == 0) mt_next_state(g);
    uint32_t y = g->state[g->next++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

/* CPUGeneratorImpl::random64: two consecutive 32-bit draws, first draw in the
 * high word (pinned by tests/golden/mt.npz's int64 random_() stream). */
uint64_t fko_random64(fko_gen *g) {
    uint32_t hi = fko_random(g);
    uint32_t lo = fko_random(g);
    return ((uint64_t)hi << 32) | lo;
}

void fko_fill_u32(fko_gen *g, uint32_t *out, int64_t n) {
    for (int64_t i = 0; i < n; i++) out[i] = fko_random(g);
}

/* ------------------------------------------------------------------------- */
/* bf16 / f16 scalar helpers (c10::BFloat16 RNE, c10::Half)                   */
/* ------------------------------------------------------------------------- */
static inline float f_from_u(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t u_from_f(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* c10::detail::round_to_nearest_even (torch/headeronly/util/BFloat16.h:100-114) */
static inline uint16_t bf16_from_f(float f) {
    if (f != f) return 0x7FC0;
    uint32_t u = u_from_f(f);
    return (uint16_t)((u + (((u >> 16) & 1u) + 0x7FFFu)) >> 16);
}
static inline float f_from_bf16(uint16_t b) { return f_from_u((uint32_t)b << 16); }
static inline float bf(float f) { return f_from_bf16(bf16_from_f(f)); } /* round through bf16 */

/* IEEE binary16 <-> float with RNE (c10::Half uses the same conversion). */
static inline uint16_t h_from_f(float f) {
    uint32_t x = u_from_f(f);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t ax = x & 0x7fffffffu;
    if (ax > 0x7f800000u) return (uint16_t)(sign | 0x7e00u);           /* NaN */
    if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);          /* overflow -> inf */
    if (ax < 0x38800000u) {                                             /* subnormal half */
        float a = f_from_u(ax);
        /* a * 2^24 rounded to integer (RNE) */
        float s = a * 16777216.0f;
        uint32_t m = (uint32_t)nearbyintf(s);
        return (uint16_t)(sign | m);
    }
    uint32_t mant = ax & 0x7fffffu;
    uint32_t exp = (ax >> 23) - 127 + 15;
    uint32_t h = (exp << 10) | (mant >> 13);
    uint32_t rem = mant & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return (uint16_t)(sign | h);
}
static inline float f_from_h(uint16_t h) {
    uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1fu, mant = h & 0x3ffu;
    if (exp == 0) {
        float v = (float)mant * (1.0f / 16777216.0f);
        return sign ? -v : v;
    }
    if (exp == 31) return f_from_u(sign | 0x7f800000u | (mant << 13));
    return f_from_u(sign | ((exp - 15 + 127) << 23) | (mant << 13));
}
static inline float hf(float f) { return f_from_h(h_from_f(f)); }

/* ------------------------------------------------------------------------- */
/* fp32 Box-Muller, AVX2 flavour: normal_fill_16_AVX2 (DistributionTemplates.h:88-106)
 * with log256_ps / sincos256_ps restated lane by lane.  fmaf() marks exactly the
 * mul+add pairs GCC contracts in libtorch's AVX2/AVX512 kernels (GCC's
 * widening_mul pass fuses a product into its single PLUS/MINUS use, first
 * product in program order first).                                           */
/* ------------------------------------------------------------------------- */
static const float c_SQRTHF = 0.707106781186547524;
static const float c_log_p0 = 7.0376836292E-2, c_log_p1 = -1.1514610310E-1,
                   c_log_p2 = 1.1676998740E-1, c_log_p3 = -1.2420140846E-1,
                   c_log_p4 = +1.4249322787E-1, c_log_p5 = -1.6668057665E-1,
                   c_log_p6 = +2.0000714765E-1, c_log_p7 = -2.4999993993E-1,
                   c_log_p8 = +3.3333331174E-1, c_log_q1 = -2.12194440e-4,
                   c_log_q2 = 0.693359375;
static const float c_mDP1 = -0.78515625, c_mDP2 = -2.4187564849853515625e-4,
                   c_mDP3 = -3.77489497744594108e-8;
static const float c_sin_p0 = -1.9515295891E-4, c_sin_p1 = 8.3321608736E-3,
                   c_sin_p2 = -1.6666654611E-1;
static const float c_cos_p0 = 2.443315711809948E-005, c_cos_p1 = -1.388731625493765E-003,
                   c_cos_p2 = 4.166664568298827E-002;
static const float c_FOPI = 1.27323954473516;

/* contraction variant bits, for tests/test_oracle_golden.py's search; the
 * default (FKO_CONTRACT_DEFAULT) is the pattern pinned by the golden z stream. */
static int g_contract = -1;
#define FKO_CONTRACT_DEFAULT 0
void fko_set_contract(int bits) { g_contract = bits; }
static inline int cbit(int b) { return ((g_contract < 0 ? FKO_CONTRACT_DEFAULT : g_contract) >> b) & 1; }

static float cephes_logf(float x) {
    /* invalid (x <= 0) lanes are NaN; never reached: u1 in [2^-24, 1] */
    int invalid = !(x > 0.0f);
    if (x < f_from_u(0x00800000u)) x = f_from_u(0x00800000u); /* _mm256_max_ps(x, min_norm_pos) */
    int32_t imm0 = (int32_t)(u_from_f(x) >> 23);
    x = f_from_u((u_from_f(x) & ~0x7f800000u) | u_from_f(0.5f));
    imm0 -= 0x7f;
    float e = (float)imm0;
    e = e + 1.0f;
    int mask = x < c_SQRTHF;
    float tmp = mask ? x : 0.0f;
    x = x - 1.0f;
    e = e - (mask ? 1.0f : 0.0f);
    x = x + tmp;
    float z = x * x;
    float y = c_log_p0;
    y = fmaf(y, x, c_log_p1);
    y = fmaf(y, x, c_log_p2);
    y = fmaf(y, x, c_log_p3);
    y = fmaf(y, x, c_log_p4);
    y = fmaf(y, x, c_log_p5);
    y = fmaf(y, x, c_log_p6);
    y = fmaf(y, x, c_log_p7);
    y = fmaf(y, x, c_log_p8);
    y = y * x;
    /* y = y*z; y = y + e*q1 */
    if (cbit(0)) {
        y = fmaf(e, c_log_q1, y * z);
    } else {
        y = fmaf(y, z, e * c_log_q1);
    }
    /* y = y - z*0.5 */
    y = cbit(1) ? (y - z * 0.5f) : fmaf(-z, 0.5f, y);
    /* x = (x + y) + e*q2 */
    x = x + y;
    x = cbit(2) ? (x + e * c_log_q2) : fmaf(e, c_log_q2, x);
    if (invalid) x = f_from_u(0xffffffffu);
    return x;
}

static void cephes_sincosf(float xin, float *s, float *c) {
    uint32_t sign_bit_sin = u_from_f(xin) & 0x80000000u;
    float x = f_from_u(u_from_f(xin) & 0x7fffffffu);
    float y = x * c_FOPI;
    int32_t imm2 = (int32_t)y; /* _mm256_cvttps_epi32 (truncation) */
    imm2 = (imm2 + 1) & ~1;
    y = (float)imm2;
    int32_t imm4 = imm2;
    uint32_t swap_sign_bit_sin = ((uint32_t)(imm2 & 4)) << 29;
    int poly_mask = ((imm2 & 2) == 0);
    if (cbit(3)) {
        x = x + y * c_mDP1;
        x = x + y * c_mDP2;
        x = x + y * c_mDP3;
    } else {
        x = fmaf(y, c_mDP1, x);
        x = fmaf(y, c_mDP2, x);
        x = fmaf(y, c_mDP3, x);
    }
    imm4 = imm4 - 2;
    uint32_t sign_bit_cos = ((uint32_t)(~imm4 & 4)) << 29;
    sign_bit_sin ^= swap_sign_bit_sin;
    float z = x * x;
    float yc = c_cos_p0;
    yc = fmaf(yc, z, c_cos_p1);
    yc = fmaf(yc, z, c_cos_p2);
    yc = yc * z;
    /* y = y*z; y = y - z*0.5 */
    if (cbit(4)) {
        yc = fmaf(-z, 0.5f, yc * z);
    } else {
        yc = fmaf(yc, z, -(z * 0.5f));
    }
    yc = yc + 1.0f;
    float ys = c_sin_p0;
    ys = fmaf(ys, z, c_sin_p1);
    ys = fmaf(ys, z, c_sin_p2);
    ys = ys * z;
    ys = cbit(5) ? (ys * x + x) : fmaf(ys, x, x);
    float ysin2 = poly_mask ? ys : 0.0f;
    float ysin1 = poly_mask ? 0.0f : yc;
    ys = ys - ysin2;
    yc = yc - ysin1;
    float xmm1 = ysin1 + ysin2;
    float xmm2 = yc + ys;
    *s = f_from_u(u_from_f(xmm1) ^ sign_bit_sin);
    *c = f_from_u(u_from_f(xmm2) ^ sign_bit_cos);
}

static void normal_fill_16_f32_avx(float *d) {
    const float two_pi = (float)(2.0f * 3.14159265358979323846); /* 2.0f * c10::pi<double> */
    for (int j = 0; j < 8; j++) {
        float u1 = 1.0f - d[j];
        float u2 = d[j + 8];
        float radius = sqrtf(-2.0f * cephes_logf(u1));
        float theta = two_pi * u2;
        float s, c;
        cephes_sincosf(theta, &s, &c);
        float n1 = radius * c;
        float n2 = radius * s;
        d[j] = fmaf(n1, 1.0f, 0.0f);      /* _mm256_fmadd_ps(n1, std, mean) */
        d[j + 8] = fmaf(n2, 1.0f, 0.0f);
    }
}

/* fp32 Box-Muller, libm flavour: normal_fill_16<float> (DistributionTemplates.h:139-149),
 * used under ATEN_CPU_CAPABILITY=default. */
static void normal_fill_16_f32_libm(float *d) {
    for (int j = 0; j < 8; j++) {
        const float u1 = 1 - d[j];
        const float u2 = d[j + 8];
        const float radius = sqrtf(-2 * logf(u1));
        const float theta = (float)(2.0f * 3.14159265358979323846 * u2);
        d[j] = radius * cosf(theta) * 1.0f + 0.0f;
        d[j + 8] = radius * sinf(theta) * 1.0f + 0.0f;
    }
}

/* bf16 Box-Muller: normal_fill_16<BFloat16>; every c10::BFloat16 op is a float op
 * rounded to bf16, theta goes double -> float -> bf16 (BFloat16.h:306, ctor :125). */
static void normal_fill_16_bf16(uint16_t *d) {
    for (int j = 0; j < 8; j++) {
        const float u1 = bf(1.0f - f_from_bf16(d[j]));
        const float u2 = f_from_bf16(d[j + 8]);
        const float radius = bf(sqrtf(bf(-2.0f * bf(logf(u1)))));
        const float theta = bf((float)(2.0f * 3.14159265358979323846 * (double)u2));
        const float c = bf(cosf(theta)), s = bf(sinf(theta));
        d[j] = bf16_from_f(bf(bf(bf(radius * c) * 1.0f) + 0.0f));
        d[j + 8] = bf16_from_f(bf(bf(bf(radius * s) * 1.0f) + 0.0f));
    }
}

/* f16: same template, c10::Half ops. */
static void normal_fill_16_f16(uint16_t *d) {
    for (int j = 0; j < 8; j++) {
        const float u1 = hf(1.0f - f_from_h(d[j]));
        const float u2 = f_from_h(d[j + 8]);
        const float radius = hf(sqrtf(hf(-2.0f * hf(logf(u1)))));
        const float theta = hf((float)(2.0f * 3.14159265358979323846 * (double)u2));
        const float c = hf(cosf(theta)), s = hf(sinf(theta));
        d[j] = h_from_f(hf(hf(hf(radius * c) * 1.0f) + 0.0f));
        d[j + 8] = h_from_f(hf(hf(hf(radius * s) * 1.0f) + 0.0f));
    }
}

static void normal_fill_16_f64(double *d) {
    for (int j = 0; j < 8; j++) {
        const double u1 = 1 - d[j];
        const double u2 = d[j + 8];
        const double radius = sqrt(-2 * log(u1));
        const double theta = 2.0f * 3.14159265358979323846 * u2;
        d[j] = fma(radius * cos(theta), 1.0, 0.0);
        d[j + 8] = fma(radius * sin(theta), 1.0, 0.0);
    }
}

/* at::normal_distribution<double> (DistributionsHelper.h:189-221), numel < 16 path. */
static double normal_double(fko_gen *g) {
    if (g->has_cached_double) {
        g->has_cached_double = 0;
        return g->cached_double * 1.0 + 0.0;
    }
    const double u1 = (double)(fko_random64(g) & ((1ULL << 53) - 1)) * (1.0 / 9007199254740992.0);
    const double u2 = (double)(fko_random64(g) & ((1ULL << 53) - 1)) * (1.0 / 9007199254740992.0);
    const double r = sqrt(-2.0 * log1p(-u2));
    const double theta = 2.0 * 3.14159265358979323846 * u1;
    g->cached_double = r * sin(theta);
    g->has_cached_double = 1;
    return r * cos(theta) * 1.0 + 0.0;
}

/* dtype codes shared with include/fks.h */
enum { FKO_F32 = 0, FKO_BF16 = 1, FKO_F16 = 2, FKO_F64 = 3 };
/* capability: 0 = AVX2/AVX512 dispatch (any x86-64 host with AVX2), 1 = default */

/* torch.normal(mean=0, std=1, size=(n,), dtype) on the CPU generator
 * (normal_kernel, DistributionTemplates.h:231-256). */
void fko_normal(fko_gen *g, void *out, int64_t n, int dtype, int capability) {
    if (n <= 0) return;
    if (n < 16) {
        for (int64_t i = 0; i < n; i++) {
            double v = normal_double(g);
            switch (dtype) {
            case FKO_F32: ((float *)out)[i] = (float)v; break;
            case FKO_BF16: ((uint16_t *)out)[i] = bf16_from_f((float)v); break;
            case FKO_F16: ((uint16_t *)out)[i] = h_from_f((float)v); break;
            default: ((double *)out)[i] = v; break;
            }
        }
        return;
    }
    switch (dtype) {
    case FKO_F32: {
        float *d = (float *)out;
        for (int64_t i = 0; i < n; i++) d[i] = (float)(fko_random(g) & 0xFFFFFFu) * (1.0f / 16777216.0f);
        void (*fill)(float *) = capability == 0 ? normal_fill_16_f32_avx : normal_fill_16_f32_libm;
        for (int64_t i = 0; i < n - 15; i += 16) fill(d + i);
        if (n % 16 != 0) {
            d = d + n - 16;
            for (int i = 0; i < 16; i++) d[i] = (float)(fko_random(g) & 0xFFFFFFu) * (1.0f / 16777216.0f);
            fill(d);
        }
        break;
    }
    case FKO_BF16: {
        uint16_t *d = (uint16_t *)out;
        for (int64_t i = 0; i < n; i++) d[i] = bf16_from_f((float)(fko_random(g) & 0xFFu) * (1.0f / 256.0f));
        for (int64_t i = 0; i < n - 15; i += 16) normal_fill_16_bf16(d + i);
        if (n % 16 != 0) {
            d = d + n - 16;
            for (int i = 0; i < 16; i++) d[i] = bf16_from_f((float)(fko_random(g) & 0xFFu) * (1.0f / 256.0f));
            normal_fill_16_bf16(d);
        }
        break;
    }
    case FKO_F16: {
        uint16_t *d = (uint16_t *)out;
        for (int64_t i = 0; i < n; i++) d[i] = h_from_f((float)(fko_random(g) & 0x7FFu) * (1.0f / 2048.0f));
        for (int64_t i = 0; i < n - 15; i += 16) normal_fill_16_f16(d + i);
        if (n % 16 != 0) {
            d = d + n - 16;
            for (int i = 0; i < 16; i++) d[i] = h_from_f((float)(fko_random(g) & 0x7FFu) * (1.0f / 2048.0f));
            normal_fill_16_f16(d);
        }
        break;
    }
    default: {
        double *d = (double *)out;
        for (int64_t i = 0; i < n; i++)
            d[i] = (double)(fko_random64(g) & ((1ULL << 53) - 1)) * (1.0 / 9007199254740992.0);
        for (int64_t i = 0; i < n - 15; i += 16) normal_fill_16_f64(d + i);
        if (n % 16 != 0) {
            d = d + n - 16;
            for (int i = 0; i < 16; i++)
                d[i] = (double)(fko_random64(g) & ((1ULL << 53) - 1)) * (1.0 / 9007199254740992.0);
            normal_fill_16_f64(d);
        }
        break;
    }
    }
}

/* ------------------------------------------------------------------------- */
/* Parameter updates: one torch op per line, each rounded to the param dtype.  */
/* ------------------------------------------------------------------------- */

/* zo_utils.py:49  param.data - lr * (g * z + wd * param.data)    (has_wd)
 * zo_utils.py:52  param.data - lr * (g * z)                      (!has_wd)
 * Scalars enter as fp32 (opmath of fp32/bf16/f16) or fp64 (f64 params). */
void fko_update(void *p, const void *z, int64_t n, int dtype, double g, double lr, double wd, int has_wd) {
    const float gf = (float)g, lrf = (float)lr, wdf = (float)wd;
    switch (dtype) {
    case FKO_F32: {
        float *x = (float *)p;
        const float *zz = (const float *)z;
        for (int64_t i = 0; i < n; i++) {
            float t = gf * zz[i];
            if (has_wd) t = t + wdf * x[i];
            x[i] = x[i] - lrf * t;
        }
        break;
    }
    case FKO_BF16: {
        uint16_t *x = (uint16_t *)p;
        const uint16_t *zz = (const uint16_t *)z;
        for (int64_t i = 0; i < n; i++) {
            float xv = f_from_bf16(x[i]);
            float t = bf(gf * f_from_bf16(zz[i]));
            if (has_wd) t = bf(t + bf(wdf * xv));
            x[i] = bf16_from_f(xv - bf(lrf * t));
        }
        break;
    }
    case FKO_F16: {
        uint16_t *x = (uint16_t *)p;
        const uint16_t *zz = (const uint16_t *)z;
        for (int64_t i = 0; i < n; i++) {
            float xv = f_from_h(x[i]);
            float t = hf(gf * f_from_h(zz[i]));
            if (has_wd) t = hf(t + hf(wdf * xv));
            x[i] = h_from_f(xv - hf(lrf * t));
        }
        break;
    }
    default: {
        double *x = (double *)p;
        const double *zz = (const double *)z;
        for (int64_t i = 0; i < n; i++) {
            double t = g * zz[i];
            if (has_wd) t = t + wd * x[i];
            x[i] = x[i] - lr * t;
        }
        break;
    }
    }
}

/* optimizer.py:173  param.data + scaling_factor * eps * z ; `scale` is the python
 * double product scaling_factor*eps, cast to the opmath type at the multiply. */
void fko_perturb(void *p, const void *z, int64_t n, int dtype, double scale) {
    const float sf = (float)scale;
    switch (dtype) {
    case FKO_F32: {
        float *x = (float *)p;
        const float *zz = (const float *)z;
        for (int64_t i = 0; i < n; i++) x[i] = x[i] + sf * zz[i];
        break;
    }
    case FKO_BF16: {
        uint16_t *x = (uint16_t *)p;
        const uint16_t *zz = (const uint16_t *)z;
        for (int64_t i = 0; i < n; i++) x[i] = bf16_from_f(f_from_bf16(x[i]) + bf(sf * f_from_bf16(zz[i])));
        break;
    }
    case FKO_F16: {
        uint16_t *x = (uint16_t *)p;
        const uint16_t *zz = (const uint16_t *)z;
        for (int64_t i = 0; i < n; i++) x[i] = h_from_f(f_from_h(x[i]) + hf(sf * f_from_h(zz[i])));
        break;
    }
    default: {
        double *x = (double *)p;
        const double *zz = (const double *)z;
        for (int64_t i = 0; i < n; i++) x[i] = x[i] + scale * zz[i];
        break;
    }
    }
}

/* ------------------------------------------------------------------------- */
/* Whole reconstruct, for the CPU baseline: fedkseed.py:136-141 over a tensor  */
/* list already resolved to per-tensor (lr, wd, has_wd) by the sticky rule.    */
/* ------------------------------------------------------------------------- */
typedef struct {
    void *data;
    int64_t numel;
    int32_t dtype;
    int32_t has_wd;
    double lr;
    double wd;
} fko_tensor;

static size_t dsize(int dtype) { return dtype == FKO_F32 ? 4 : dtype == FKO_F64 ? 8 : 2; }

int fko_reconstruct(const fko_tensor *t, int32_t nt, const uint64_t *seeds, const double *g, int32_t k,
                    int32_t capability) {
    int64_t maxn = 16;
    for (int i = 0; i < nt; i++) if (t[i].numel > maxn) maxn = t[i].numel;
    void *z = malloc((size_t)maxn * 8);
    if (!z) return -12;
    fko_gen gen;
    for (int s = 0; s < k; s++) {
        if (g[s] == 0.0) continue; /* fedkseed.py:137 skips exact zeros only; NaN is applied */
        fko_seed(&gen, seeds[s]);
        for (int i = 0; i < nt; i++) {
            fko_normal(&gen, z, t[i].numel, t[i].dtype, capability);
            fko_update(t[i].data, z, t[i].numel, t[i].dtype, g[s], t[i].lr, t[i].wd, t[i].has_wd);
        }
    }
    free(z);
    (void)dsize;
    return 0;
}

/* random_perturb_parameters over a tensor list (requires_grad already filtered). */
int fko_perturb_params(const fko_tensor *t, int32_t nt, uint64_t seed, double scale, int32_t capability) {
    int64_t maxn = 16;
    for (int i = 0; i < nt; i++) if (t[i].numel > maxn) maxn = t[i].numel;
    void *z = malloc((size_t)maxn * 8);
    if (!z) return -12;
    fko_gen gen;
    fko_seed(&gen, seed);
    for (int i = 0; i < nt; i++) {
        fko_normal(&gen, z, t[i].numel, t[i].dtype, capability);
        fko_perturb(t[i].data, z, t[i].numel, t[i].dtype, scale);
    }
    free(z);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* Seed-sharded variant (include/fks.h fks_delta_accumulate / fks_delta_apply): */
/* NOT a reference routine -- the restated sum p_K = a^K p_0 - sum_k c_k z_k of */
/* the reference's K sequential steps (zo_utils.py:49 with a = 1 - lr*wd), with */
/* the device's exact f32 operation order, so its kernels can be checked bit    */
/* for bit.  z is the reference's stream (fedkseed.py:138 -> zo_utils.py:47).   */
/* ------------------------------------------------------------------------- */
static float z_as_float(const void *z, int64_t e, int dtype) {
    if (dtype == FKO_F32) return ((const float *)z)[e];
    if (dtype == FKO_BF16) return f_from_bf16(((const uint16_t *)z)[e]);
    return f_from_h(((const uint16_t *)z)[e]);
}

/* delta[cum_i + e] = fmaf(f32(coefs[s]), z_s(i, e), delta[cum_i + e]) for s in order;
 * frozen[i] != 0: the tensor draws its z but its delta is not written */
int fko_delta_accumulate(const fko_tensor *t, int32_t nt, const int32_t *frozen, const uint64_t *seeds,
                         const double *coefs, int32_t k, float *delta, int32_t capability) {
    int64_t maxn = 16;
    for (int i = 0; i < nt; i++) if (t[i].numel > maxn) maxn = t[i].numel;
    void *z = malloc((size_t)maxn * 8);
    if (!z) return -12;
    fko_gen gen;
    for (int s = 0; s < k; s++) {
        const float c = (float)coefs[s];
        fko_seed(&gen, seeds[s]);
        int64_t cum = 0;
        for (int i = 0; i < nt; i++) {
            fko_normal(&gen, z, t[i].numel, t[i].dtype, capability);
            if (!(frozen && frozen[i]))
                for (int64_t e = 0; e < t[i].numel; e++)
                    delta[cum + e] = fmaf(c, z_as_float(z, e, t[i].dtype), delta[cum + e]);
            cum += t[i].numel;
        }
    }
    free(z);
    return 0;
}

/* p = dtype(fmaf(f32(decay[i]), p, -delta[cum_i + e])) */
void fko_delta_apply(const fko_tensor *t, int32_t nt, const int32_t *frozen, const float *delta, const double *decay) {
    int64_t cum = 0;
    for (int i = 0; i < nt; i++) {
        if (!(frozen && frozen[i])) {
            const float d = (float)decay[i];
            for (int64_t e = 0; e < t[i].numel; e++) {
                if (t[i].dtype == FKO_F32) {
                    float *p = (float *)t[i].data;
                    p[e] = fmaf(d, p[e], -delta[cum + e]);
                } else if (t[i].dtype == FKO_BF16) {
                    uint16_t *p = (uint16_t *)t[i].data;
                    p[e] = bf16_from_f(fmaf(d, f_from_bf16(p[e]), -delta[cum + e]));
                } else {
                    uint16_t *p = (uint16_t *)t[i].data;
                    p[e] = h_from_f(fmaf(d, f_from_h(p[e]), -delta[cum + e]));
                }
            }
        }
        cum += t[i].numel;
    }
}

int fko_sizeof_gen(void) { return (int)sizeof(fko_gen); }
int fko_sizeof_tensor(void) { return (int)sizeof(fko_tensor); }
