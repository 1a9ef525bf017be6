// fks_internal.h -- shared declarations of libfks.so (host + device).
#pragma once

#include <cerrno>
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "fks.h"

namespace fks {

// Exceptions never cross the C ABI: fks_capi.cpp converts them to codes.
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// ---- MT19937 constants (MT19937RNGEngine.h:21-25) ----
constexpr int kMtN = 624;
constexpr int kMtM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu;

// ---- jump-ahead (fks_gf2.cpp) ----
int jump_poly_words();  // 312
void jump_polys_for_blocks(const std::vector<int64_t>& blocks, std::vector<uint64_t>& out);
void host_jump_window(uint64_t seed, int64_t block, uint32_t* out624);
void host_x_words(uint64_t seed, int64_t first, int n, uint32_t* out);  // untempered x[first, first + n)

// ---- Box-Muller tables for the 8-bit (bf16) and 11-bit (f16) uniforms (fks_tables.cpp) ----
// radius[a], cos[b], sin[b] as float values of the reduced type, exactly as
// normal_fill_16<scalar_t> (DistributionTemplates.h:139-149) computes them.
struct Tables {
  float r_bf16[256], c_bf16[256], s_bf16[256];
  float r_f16[2048], c_f16[2048], s_f16[2048];
};
const Tables& tables();

// ---- device-side descriptors ----
// A regular segment: a tensor (or the part of it) whose 16-element Box-Muller
// blocks sit on 16-aligned stream positions, so each 16-block lies inside one
// 624-word MT block.
struct DevSeg {
  int64_t start;   // stream position of element 0
  int64_t numel;   // multiple of 16
  uint64_t ptr;    // device address of element 0
  float lr;
  float wd;
  uint32_t flags;  // FKS_HAS_WD
  int32_t dtype;
  float ps;        // perturbation scale f32(scaling_factor * eps) (perturb modes)
  uint32_t pad;
};
static_assert(sizeof(DevSeg) == 48, "DevSeg layout");

// Irregular work (fks_irregular_kernel): a run of whole 16-blocks at any stream phase ...
struct DevRun {
  int64_t start;   // stream word of the run's first 16-block
  int64_t numel;   // 16 * (16-blocks in the run)
  uint64_t ptr;    // device address of the run's element 0
  int64_t limit;   // elements [limit, numel) are not written (a ragged head, see make_layout)
  float lr;
  float wd;
  uint32_t flags;  // FKS_HAS_WD
  int32_t dtype;
  float ps;        // perturbation scale (perturb modes)
  uint32_t pad;
};
static_assert(sizeof(DevRun) == 56, "DevRun layout");

// ... and one element of a numel < 16 tensor (serial normal_distribution<double>)
constexpr uint32_t kTinySin = 1u << 8;  // the element takes the pair's cached r*sin value
struct DevTiny {
  int64_t word;    // stream word of its Box-Muller pair (two random64 draws = 4 words)
  uint64_t ptr;    // device address of the element
  float lr;
  float wd;
  uint32_t flags;  // FKS_HAS_WD | kTinySin
  int32_t dtype;
  float ps;        // perturbation scale (perturb modes)
  uint32_t pad;
};
static_assert(sizeof(DevTiny) == 40, "DevTiny layout");

constexpr int kApplyThreads = 320;  // 312 Box-Muller pairs per 624-word block + 8 idle lanes
constexpr int kApplyWgPerCu = 3;  // resident apply workgroups per CU (LDS-limited)
// MT windows resident in LDS per workgroup: (seeds + 1 spare) x 2496 B + 4 KB tables <= 160 KB / WGs
constexpr int kMaxSeedsPerPass = (160 * 1024 / kApplyWgPerCu - 4096) / 2496 - 1;  // tables: <= 4 KB
// calls of at most kSmallK seeds run one pass over kSmallWgPerCu workgroups per CU
constexpr int kSmallK = 4;
// fks_small2_kernel (two Box-Muller pairs per lane): 56 VGPRs, 8 workgroups of 4 waves
// (8 waves/SIMD; K = 1, 2 fit 8 in LDS, K = 4 six): perturb 7.2 ms at 8 WGs, 7.8 ms at 6
// (profiles/r02_smallk_ab.log; the round-1 kernel of one pair per lane: 9.1 ms)
constexpr int kSmallWgPerCu = 8;
// one-seed bf16 z indices (fks_small2_kernel ZM 1 / 2): one u32 per pair lane and block
constexpr int kSm2ZidxPerBlock = 156;
constexpr int kSm2ZidxBytesPerBlock = 4 * kSm2ZidxPerBlock;
constexpr int kJumpThreads = 1024;  // 16 waves, one chunk's jump per wave at a time
constexpr int kJumpMaxCpw = 32;  // most chunks one jump workgroup takes (fks_capi.cpp jump_chunks_per_wg)
constexpr int kJumpXLen = 19937 + 624;  // x[0..20560]: y[i + w] = x[i + w + 1], i < 19937, w < 624

// kModeUpdateWd / kModeUpdateNoWd: kModeUpdate specialised for a launch whose segments
// all have / all lack the weight-decay term (fast kernel only; chosen by the host)
// kModeUpdateWd0: every segment has the term with wd = +-0.0 (the HF default the reference's
// ClientTrainer passes, fedkseed.py:140): wd*p is exactly +-0 or NaN and gz + wd*p is
// exactly gz, +-0 or NaN, so both roundings are identities and t = fma(wd, p, gz) gives
// the same bits (signed zeros and NaNs included) with one instruction instead of six
// per element pair
// kModeUpdateWdPos0 (torch_rocm stream only): every tensor has wd = +0.0 exactly, is bf16
// or f32, and the host has bounded |lr g z| <= 1e30 for every seed of the call; then for a
// finite p the fma above is exactly gz (wd*p is +0 for p >= +0, -0 for p <= -0, and the
// only sum that differs from gz, -0 + +0 = +0, is followed by lr*t and p - that, whose
// result for p >= +0 does not depend on that zero's sign), p - lr*t cannot overflow, and a
// +-inf p -- which the reference turns into NaN at the first seed (0 * inf) -- is set to
// NaN at load: t = gz, one packed op per element pair and seed fewer
enum ApplyModeExt : int { kModeUpdateWdPos0 = 8 };

// Device-side dtype of fp32 tensors drawn under FKS_LIBM (ATen's DEFAULT CPU capability):
// fp32 storage and arithmetic, z from normal_fill_16<float> with glibc's logf / sinf / cosf
// (fks_libm.h) instead of the AVX2 kernel's Cephes functions.  launch_apply takes it as its
// dtype; nothing outside the kernels sees it.
constexpr int kDtF32Libm = 3;

// kModePerturbUpdate: p + ps*z, then the update with the same z (the restore
// perturbation of zeroth_order_step fused with its directional step)
// kModeDelta: the seed-sharded variant; z is accumulated into an f32 delta buffer,
// delta += c_k * z (one fma), instead of updating the parameters
enum ApplyMode : int {
  kModeUpdate = 0, kModePerturb = 1, kModeWriteZ = 2, kModeUpdateWd = 3, kModeUpdateNoWd = 4, kModePerturbUpdate = 5,
  kModeDelta = 6, kModeUpdateWd0 = 7
};

// Per-pass seeds and multipliers travel BY VALUE in the kernel arguments: a call
// uploads nothing per pass, and the static header (chunk table, jump polynomials,
// descriptors) is cached on the device across calls (fks_capi.cpp, PlanCache).
struct ApplyArgs {
  const uint32_t* states;       // [nseeds][nchunks][624] generator windows at chunk starts
  float g[kMaxSeedsPerPass];    // update multiplier per seed (mode 0) / delta coefficient
  const DevSeg* segs;           // regular segments of this launch's dtype, sorted by start
  const int64_t* chunk_block;   // [nchunks + 1] first MT block of each chunk
  uint64_t* sink;               // 4 KB of workspace: loads/stores of idle lanes (>= one block of f32 pairs)
  const float* gdev;            // kModePerturbUpdate from device memory: {g, apply} (nullptr: g[] above)
  uint32_t* zidx;               // bf16 one-seed z indices: 156 u32 per block from block zlo (zmode 1 / 2)
  int64_t zlo;
  int32_t zmode;                // 0, 1 = store the indices while generating, 2 = replay them (no generator)
  int32_t nsegs;
  int32_t nchunks;
  int32_t nseeds;
  int32_t mode;
};

struct IrrArgs {
  const uint32_t* states;       // [nseeds][nchunks][624]
  float g[3][kMaxSeedsPerPass]; // per-dtype multipliers of this pass's seeds
  const DevRun* runs;           // sorted by start (disjoint)
  const DevTiny* tiny;          // sorted by word
  const int64_t* chunk_lo;      // [nchunks] chunk c twists MT blocks [chunk_lo[c], chunk_hi[c])
  const int64_t* chunk_hi;
  const float* gdev;            // kModePerturbUpdate from device memory: {g, apply} (nullptr: g[][] above)
  int32_t nruns;
  int32_t ntiny;
  int32_t nchunks;
  int32_t nseeds;
  int32_t mode;
  int32_t libm;                 // fp32 runs draw the libm flavour (FKS_LIBM: kDtF32Libm)
};

// bf16 slice kernel (fks_apply_bs_kernel): up to 64 seeds per pass; one workgroup per CU
// with two bit-sliced 32-seed states (one plane word per 32 seeds) in two 384-thread
// halves of six waves, each wave twisting and updating 128-word tasks; LDS = 3 KB of
// tables + 2 x 79,872 B of state + task flags.  The plan cuts the stream into 2 x (one per
// CU) chunks; a pass of 33..64 seeds runs two SLICES on one chunk PAIR (half 1 applies
// seeds [ceil(n/2), n) after half 0 applied [0, ceil(n/2))), a pass of <= 32 seeds runs
// one slice on each chunk of the pair (split).
constexpr int kBsSeeds = 32;                  // seeds per slice (bits of a plane word)
constexpr int kBsPassSeeds = 2 * kBsSeeds;    // seeds per launch
constexpr int kBsHalfThreads = 384;
constexpr int kBsThreads = 2 * kBsHalfThreads;
constexpr int kBsChunksPerWg = 2;  // plan chunks per workgroup
// reconstructs of more seeds than one 19-seed pass take the slice kernel for their
// bf16 fast segments
constexpr int kBsMinSeeds = kMaxSeedsPerPass + 1;
constexpr int kJumpMaxSeeds = kBsPassSeeds > kMaxSeedsPerPass ? kBsPassSeeds : kMaxSeedsPerPass;

struct ApplyBsArgs {
  const uint32_t* states;       // [nseeds][nchunks][624] generator windows at chunk starts
  float g[kBsPassSeeds];        // update multiplier per seed / delta coefficient
  const DevSeg* segs;           // bf16 fast segments, sorted by start
  const int64_t* chunk_block;   // [2 x workgroups + 1] plan chunks
  uint64_t* sink;               // workspace sink for idle lanes' loads/stores
  int32_t nsegs;
  int32_t nchunks;              // chunks of the states array: workgroups (slices) or 2 x workgroups (split)
  int32_t nseeds;               // slices: 1..64, slice 0 takes seeds [0, ceil(n/2)), slice 1 the rest; split: 1..32
  int32_t mode;
  int32_t split;                // 1: one slice per plan chunk; 0: two slices on a chunk pair
  int32_t use_slot;             // 1: seed k's windows are window set slot[k] of states (the
                                // reconstruct window cache); 0: window set k
  uint32_t slot[kBsPassSeeds];
};

struct JumpArgs {
  uint64_t seeds[kJumpMaxSeeds];
  const uint64_t* polys;        // [nchunks][312] t^(624*b-1) mod phi (unused for b == 0)
  const int64_t* chunk_block;   // [nchunks + 1]
  uint32_t* states;             // [nseeds][nchunks][624]
  int32_t nchunks;
  int32_t chunks_per_wg;
  int32_t stride;               // chunk c starts at chunk_block[c * stride] (polys likewise); 0 = 1
  int32_t use_slot;             // 1: seed k's windows go to window set slot[k] of states; 0: set k
  uint32_t slot[kJumpMaxSeeds];
};

// ---- torch_rocm stream (FKS_STREAM_ROCM): torch.normal on a HIP device ----
// torch's normal_kernel (ATen/native/cuda/DistributionTemplates.h:444-471) draws through
// distribution_nullary_kernel (:97-160): a grid-stride loop of `stride` = 256 x grid
// threads (calc_execution_policy :50-62: grid = min(ceil(numel / 256), CUs x
// maxThreadsPerCU / 256)), thread idx drawing curand_normal4 (Philox4x32-10 at
// subsequence idx, offset `philox offset`; Box-Muller of rocrand) once per loop
// iteration j for the elements idx + stride (4 j + i), i < 4.  Each tensor's draw
// advances the generator's offset by ((numel - 1) / (4 stride) + 1) * 4.
// A work ITEM is one (tensor, idx, j): one Philox call, four elements.
struct PhxTensor {
  uint64_t ptr;     // device address of element 0
  int64_t numel;
  int64_t item0;    // the tensor's first work item (items of all tensors laid end to end)
  uint64_t off4;    // philox offset / 4 of this tensor's draw (the counter's 64-bit low half)
  uint32_t stride;  // 256 x grid of torch's launch
  int32_t dtype;
  float lr;
  float wd;
  uint32_t flags;   // FKS_HAS_WD | kPhxP16
  float ps;         // perturbation scale (perturb modes)
};
static_assert(sizeof(PhxTensor) == 56, "PhxTensor layout");
// PhxTensor::flags: the parameter's data is 16-byte aligned (an f16 tensor then takes torch's
// 8-wide vectorized elementwise path; fks_device.hip mul_f16_ref)
constexpr uint32_t kPhxP16 = 1u << 8;
// ... and the entry's first element sits 16-byte aligned in a freshly allocated tensor of the
// parameter's size (z, g z, the update's temporaries): false only for the later pieces of a
// tensor past 2^31 bytes, whose 32-bit-indexed launches start mid-tensor
constexpr uint32_t kPhxFresh16 = 1u << 9;
// ... and the p the call's first `wd * p` reads in the reference is 16-byte aligned (the
// buffer itself, or with FKS_FRESH the fresh tensor an earlier reference step rebound
// param.data to)
constexpr uint32_t kPhxWdP16 = 1u << 10;
// torch's elementwise kernels on ROCm (ATen/native/cuda/CUDALoops.cuh): a 2-byte tensor is
// processed in blocks of 256 threads x 8 elements; a partial last block takes the unrolled path
constexpr int64_t kTorchHalfBlockWork = 2048;

constexpr int kPhxSeeds = 32;  // seeds per launch (by value in the arguments)
struct PhiloxArgs {
  uint64_t seeds[kPhxSeeds];
  float g[kPhxSeeds * 3];  // the multiplier per seed, per dtype
  const PhxTensor* t;   // sorted by item0
  const float* gdev;    // kModePerturbUpdate from device memory: {g, apply} (nullptr: g[] above)
  int64_t item_lo;      // this launch's items [item_lo, item_hi) (element shards)
  int64_t item_hi;
  int32_t nt;
  int32_t nseeds;
  int32_t mode;
  int32_t call_first;   // seed 0 of this launch is the first seed of the call
};
int launch_philox(const PhiloxArgs& a, void* stream);
int device_max_threads_per_cu();

// fks_delta_apply: p = dtype(f32(decay) * p - delta[delta_off + e]) over one tensor
struct DeltaApplyDesc {
  uint64_t ptr;       // the tensor's parameters
  int64_t numel;
  int64_t delta_off;  // its first element in the delta buffer
  int32_t dtype;
  float decay;        // (1 - lr*wd)^K, or 1 without the weight-decay term
};
static_assert(sizeof(DeltaApplyDesc) == 32, "DeltaApplyDesc layout");

// launchers (fks_device.hip); return hipError_t as int
int launch_jump(const JumpArgs& a, int nseeds, void* stream);
int launch_apply(int dtype, const ApplyArgs& a, void* stream);
int launch_apply_bs(const ApplyBsArgs& a, void* stream);
int launch_irregular(const IrrArgs& a, void* stream);
constexpr int kSqrtDomainBlocks = (1 << 24) / 256;
int launch_sqrt_domain_check(uint32_t* counts, void* stream);  // counts[kSqrtDomainBlocks]
int launch_philox_radius_check(uint32_t* counts, void* stream);  // counts[kSqrtDomainBlocks]
int launch_philox_fast_radius_check(uint32_t* counts, void* stream);  // per-block maxima
int launch_delta_apply(const DeltaApplyDesc* d, int n, int64_t max_numel, const float* delta, void* stream);
int device_cu_count();

}  // namespace fks
