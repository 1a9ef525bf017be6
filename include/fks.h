/*
 * fks.h -- C ABI of libfks.so, the MI355X (gfx950) FedKSeed codec.
 *
 * The reference's FedKSeed hot path is Python over torch; these entry points are
 * what its "FFI" for the path binds (the Python drop-in under
 * fate-llm_amd/python/fate_llm/algo/fedkseed/ loads them with ctypes).  Each entry
 * point replaces one reference routine:
 *
 *   fks_directional_step  <- zo_utils.directional_derivative_step
 *                            (python/fate_llm/algo/fedkseed/zo_utils.py:23-54), applied
 *                            for K seeds in order: the reconstruct loop of
 *                            ClientTrainer.train_once (fedkseed.py:136-141) is K calls of it
 *   fks_perturb           <- ZerothOrderOptimizer.random_perturb_parameters
 *                            (python/fate_llm/algo/fedkseed/optimizer.py:152-173)
 *   fks_normal            <- the torch.normal(mean=0, std=1, size, dtype) calls at
 *                            zo_utils.py:47 / optimizer.py:170-172, for one seed, written
 *                            into the tensors (stream parity checks)
 *
 * Numerics: the z stream is the one the reference draws after torch.manual_seed(seed)
 * where its parameters live (zo_utils.py:47 draws on param.data.device), selected per
 * call by FKS_STREAM_ROCM: torch's HIP-device generator (Philox4x32-10 + rocrand
 * Box-Muller; the Python drop-in's default for tensors on a GPU, codec.py "auto") or
 * torch's CPU generator (mt19937 + normal_fill Box-Muller, fp32 via the AVX2 Cephes
 * kernel, bf16/f16 per-op rounded; a reference client training on the CPU).  Every
 * update op is rounded exactly as the reference's torch ops.
 *
 * Conventions (all entry points):
 *  - plain pointers and sizes only; tensor data are DEVICE pointers, contiguous,
 *    aligned to the element size; seeds/values are HOST arrays;
 *  - the caller owns the parameters, the workspace (a device buffer of at least
 *    fks_workspace_size() bytes) and the optional z-index buffer (fks_zindex_attach);
 *    the library's only device allocations are its bounded plan cache of per-layout
 *    headers (see fks_plan_cache_clear) -- evicting an entry synchronises the device
 *    that owns it --, the one-seed calls' window cache (624 words per chunk of
 *    2,048: about 5 MB) and the per-device __constant__ tables;
 *  - asynchronous on `stream` (a hipStream_t; NULL = default stream), like torch ops;
 *  - return 0 on success or a negative errno-style code; fks_last_error() gives a
 *    thread-local message; no C++ exception crosses the ABI;
 *  - reentrant; the global state (plan cache, jump-ahead polynomial cache, per-device
 *    setup flags) is guarded by mutexes.
 */
#ifndef FKS_H_
#define FKS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FKS_ABI_VERSION 1

/* dtype codes */
#define FKS_F32 0
#define FKS_BF16 1
#define FKS_F16 2

/* fks_tensor.flags */
#define FKS_HAS_WD 1u   /* weight decay term present: p - lr*(g*z + wd*p)  (zo_utils.py:49)
                           absent:                    p - lr*(g*z)         (zo_utils.py:52)   */
#define FKS_FROZEN 2u   /* draws its z (stream advances) but the tensor is not written         */
#define FKS_STREAM_ROCM 4u  /* z stream: torch's HIP-device generator (Philox4x32-10 + rocrand
                           Box-Muller, torch/include/ATen/native/cuda/DistributionTemplates.h:
                           50-160, 444-471) -- the stream a reference client whose model sits on
                           a GPU draws (zo_utils.py:47 and optimizer.py:170-172 draw on
                           param.data.device).  Without it: torch's CPU generator (mt19937 +
                           normal_fill).  Every tensor of one call must agree. */
#define FKS_FRESH 8u    /* FKS_STREAM_ROCM, f16: in the reference, this parameter's param.data is a
                           tensor torch allocated in an earlier step (zo_utils.py:49 and
                           optimizer.py:173 rebind it), so the call's first `wd * p` reads 16-byte
                           aligned data and takes torch's vectorized path, whatever the alignment of
                           the buffer the drop-in updates in place.  Without it: the buffer's own. */
#define FKS_LIBM 16u    /* CPU generator's stream (no FKS_STREAM_ROCM), fp32 tensors of >= 16
                           elements: z from normal_fill_16<float> with glibc's logf / sinf / cosf,
                           what torch draws under ATen's DEFAULT CPU capability
                           (ATEN_CPU_CAPABILITY=default, or a host without AVX2;
                           DistributionTemplates.h:139-149), instead of normal_fill_16_AVX2's
                           Cephes functions.  Every tensor of a call carries it or none does;
                           bf16 / f16 tensors and tensors of < 16 elements draw the same z either
                           way. */

/* error codes (negated) */
#define FKS_EINVAL 22
#define FKS_ENOTSUP 95
#define FKS_ENOMEM 12
#define FKS_EHIP 200

typedef struct fks_tensor {
  void* data;      /* device pointer, contiguous, numel elements of dtype        */
  int64_t numel;   /* >= 0                                                        */
  int32_t dtype;   /* FKS_F32 / FKS_BF16 / FKS_F16                                */
  uint32_t flags;  /* FKS_HAS_WD | FKS_FROZEN | FKS_STREAM_ROCM | FKS_FRESH | FKS_LIBM */
  float lr;        /* fp32(lr) as the reference's opmath sees it                   */
  float wd;        /* fp32(weight_decay)                                           */
} fks_tensor;

/* Value kinds for fks_directional_step: how the reference multiplies g into z.
 * FKS_VALUE_SCALAR: g is a Python float (train_once): mul(z, g) computes in fp32.
 * FKS_VALUE_TENSOR: g is a 0-dim tensor and the first operand of g*z
 *                   (zeroth_order_step): TensorIterator first casts it to the
 *                   tensor's dtype (bf16/f16 rounding), then computes in fp32.     */
#define FKS_VALUE_SCALAR 0
#define FKS_VALUE_TENSOR 1

/* Workspace bytes needed by fks_directional_step / fks_perturb / fks_normal for
 * this tensor list and up to `k` seeds per call. */
int fks_workspace_size(const fks_tensor* t, int32_t nt, int32_t k, size_t* bytes);

/* For s = 0..k-1 in order: torch.manual_seed(seeds[s]); for every tensor in order:
 * z = normal(size, dtype); p = p - lr*(g_s*z + wd*p)  (or p - lr*(g_s*z) without
 * FKS_HAS_WD).  Exactly K directional_derivative_step calls; zero values are NOT
 * skipped here (train_once's `if grad != 0.0` filter belongs to the caller). */
int fks_directional_step(const fks_tensor* t, int32_t nt, const uint64_t* seeds, const double* values,
                         int32_t k, int32_t value_kind, void* workspace, size_t ws_bytes, void* stream);

/* fks_directional_step restricted to shard `shard` of `nshards` equal runs of whole
 * 624-word MT19937 blocks of the parameter stream: elements outside the shard are not
 * touched.  The union over shards is bit-identical to fks_directional_step (every
 * element still sees every seed in order); used for element-sharded multi-GPU
 * reconstruction (one rank per shard, no collective). */
int fks_directional_step_shard(const fks_tensor* t, int32_t nt, const uint64_t* seeds, const double* values,
                               int32_t k, int32_t value_kind, int32_t shard, int32_t nshards, void* workspace,
                               size_t ws_bytes, void* stream);

/* Reconstruct window cache (a speed cache, caller-owned like the z-index buffer): the
 * generator windows a multi-seed bf16 reconstruct jumps to -- one window set of
 * nchunk-pairs x 624 words per seed -- kept in `buf` on the current device, keyed by the
 * seed and the plan's chunk starts, so that the next reconstruct of the same tensor list
 * (or shard) skips the jumps of every seed it finds there.  A FedKSeed client rebuilds
 * its model from model_0 and the same seed candidates every round
 * (python/fate_llm/algo/fedkseed/fedkseed.py:57-68, :132-141), so from the second round
 * on the reconstruct jumps nothing.  fks_jwin_size: bytes that hold k seeds' sets for
 * this tensor list (0: the call would not use the cache); fks_jwin_size_shard: the same
 * for the element shard `shard` of `nshards` (fks_directional_step_shard), sized from
 * that shard's own plan -- an N-way shard's sets are about 1/N of the whole list's;
 * fks_jwin_attach: attach `buf`
 * (bytes; NULL / 0 detaches), waiting for the last call that used the previous buffer;
 * fks_jwin_stats: seeds found / jumped since the library loaded.  Calls on any stream
 * are ordered by an event; fks_plan_cache_clear drops the contents. */
int fks_jwin_size(const fks_tensor* t, int32_t nt, int32_t k, size_t* bytes);
int fks_jwin_size_shard(const fks_tensor* t, int32_t nt, int32_t k, int32_t shard, int32_t nshards, size_t* bytes);
int fks_jwin_attach(void* buf, size_t bytes);
int fks_jwin_stats(uint64_t* hits, uint64_t* misses);

/* Census of element sharding (no kernel launch): the stream words
 * [word_range[0], word_range[1]) shard `shard` of `nshards` owns, and per tensor the
 * number of elements fks_directional_step_shard writes for it (`written`, nt entries;
 * either output may be NULL).  Over all shards every element of a non-frozen tensor
 * is written exactly once.  For FKS_STREAM_ROCM tensors the shards are runs of whole
 * Philox rows (torch's grid-stride loop iterations: 4 x stride consecutive elements)
 * and word_range is the shard's element range in the concatenation of all nt tensors
 * (frozen and empty ones included); this builds (and caches) the call's tensor table
 * on the current device. */
int fks_shard_census(const fks_tensor* t, int32_t nt, int32_t shard, int32_t nshards, int64_t* word_range,
                     int64_t* written);

/* Number of 32-bit generator words the tensor list consumes per seed (its stream length). */
int fks_stream_length(const fks_tensor* t, int32_t nt, int64_t* words);

/* ---- where the reference leaves torch's global generators ----
 * The reference calls torch.manual_seed(seed) and then draws (zo_utils.py:42,47;
 * optimizer.py:165,170-172), so after a call the generator of the tensors' device has
 * advanced past the seed's draws; every later draw from it (a sampler's permutation, the
 * model's dropout in the zeroth-order closure) starts there.  The codec draws nothing
 * from torch's generators; these give the caller the state to leave behind.
 *
 * fks_cpu_generator_end (host only, no device needed): torch's CPU generator after
 * torch.manual_seed(seed) and the CPU-stream draws of the tensor list -- at::mt19937's
 * state_ (624 untempered words), left_ and next_ (MT19937RNGEngine.h:115-175), and
 * CPUGeneratorImpl's cached normal_distribution<double> value (valid iff numel < 16
 * tensors left the second value of a Box-Muller pair, DistributionsHelper.h:189-221).
 *
 * fks_rocm_offset: the Philox offset torch's generator of the CURRENT device advances by
 * for one seed's FKS_STREAM_ROCM draws of the list (DistributionTemplates.h:50-62,
 * :111-133, including the extra reservations of tensors past 2^31 bytes).
 * fks_rocm_grid_cap: the current device's grid cap of torch's draws, CUs x
 * (maxThreadsPerCU / 256) (2,048 on an MI355X in SPX mode); the FKS_STREAM_ROCM stream of a
 * tensor of more than 256 x cap / 4 elements depends on it, so parties of one federation
 * must agree on it (payload.py carries it). */
int fks_cpu_generator_end(const fks_tensor* t, int32_t nt, uint64_t seed, uint32_t* state624, int32_t* left,
                          uint32_t* next, int32_t* normal_valid, double* normal);
int fks_rocm_offset(const fks_tensor* t, int32_t nt, uint64_t* offset);
int fks_rocm_grid_cap(int64_t* blocks);

/* Instrumentation (bench.py): while enabled, every kernel launch is bracketed by HIP
 * events on the caller's stream; fks_profile_end synchronises them and returns the
 * summed device time of the apply and jump kernels and their launch counts. */
int fks_profile_begin(void);
int fks_profile_end(double* apply_ms, int64_t* n_apply, double* jump_ms, int64_t* n_jump);

/* Every call's static header (MT-block chunk table, jump polynomials, segment / run /
 * element descriptors) is built on the host and uploaded ONCE per distinct tensor list
 * (addresses, sizes, dtypes, flags, lr, wd, perturbation scales, shard), then kept on
 * the device in a bounded LRU plan cache: repeated calls over the same parameters (the
 * optimizer's perturb / update calls, repeated reconstructs) do no host-side layout
 * work and no upload.  fks_plan_cache_clear synchronises the device and frees every
 * cached header (e.g. before freeing the parameters' memory pool).
 *
 * One-seed calls (perturb, perturb_step, a K=1 update) keep the generator windows they
 * jumped to in a library-owned per-device buffer, keyed by the seed and the chunk starts:
 * the zeroth-order step's three calls with one seed over one parameter list jump once.
 * Use across streams is ordered by an event (no host synchronisation); the buffer is
 * freed by fks_plan_cache_clear; FKS_NO_WIN_CACHE in the environment turns it off.
 *
 * One-seed bf16 perturbs also store the Box-Muller table indices of every MT block they
 * cover in the z-index buffer the CALLER attached to the current device (fks_zindex_attach):
 * a later one-seed perturb / perturb_step / K=1 update with the same seed over blocks
 * inside that range replays the indices instead of running the generator -- the
 * zeroth-order step's second and third calls, a streaming pass at 5 B of HBM traffic per
 * parameter.  Values are identical either way; without an attached buffer of
 * fks_zindex_size bytes (or with FKS_ZCACHE=0) every call generates.  fks_plan_cache_clear
 * drops the buffer's contents, not the attachment. */
int fks_plan_cache_clear(void);

/* Bytes of z-index buffer a one-seed call over this tensor list stores (0: the list has no
 * bf16 fast segments).  Host-side; builds / reuses the list's plan. */
int fks_zindex_size(const fks_tensor* t, int32_t nt, size_t* bytes);
/* Attach `bytes` of caller-owned device memory on the current device as its z-index
 * buffer (NULL or 0 detaches).  Returns after the last call that used the previously
 * attached buffer has finished on the device, so the caller may then free or reuse it.
 * The library keeps the pointer until the next attach; it never frees it. */
int fks_zindex_attach(void* buf, size_t bytes);

/* torch.manual_seed(seed); for every tensor i in order: p = p + scales[i]*z, where
 * scales[i] = scaling_factor*eps of the tensor's group, computed in double by the
 * caller (optimizer.py:167,173).  Tensors with requires_grad=False draw nothing in
 * the reference and are simply not passed. */
int fks_perturb(const fks_tensor* t, int32_t nt, uint64_t seed, const double* scales, void* workspace,
                size_t ws_bytes, void* stream);

/* The restore perturbation of zeroth_order_step fused with its directional step
 * (optimizer.py:136 then :147 -> :92 -> zo_utils.py:49): torch.manual_seed(seed); for
 * every tensor i: p = p + scales[i]*z, and, if `update` is nonzero, then with the SAME z
 * p = p - lr*(g*z + wd*p) (or p - lr*g*z without FKS_HAS_WD), g = `value` of
 * `value_kind`.  One pass instead of two; bit-identical to fks_perturb followed by
 * fks_directional_step when both would walk the same tensor list (no frozen tensor in
 * the optimizer's groups). */
int fks_perturb_step(const fks_tensor* t, int32_t nt, uint64_t seed, const double* scales, double value,
                     int32_t value_kind, int32_t update, void* workspace, size_t ws_bytes, void* stream);

/* fks_perturb_step with g and the update decision read ON THE DEVICE when the kernels
 * run, so the caller need not synchronise on the losses (optimizer.py:138-148):
 * dev_value points to two f32 in device memory, written before this call in `stream`
 * order: dev_value[0] = g (rounded to each tensor's dtype like a FKS_VALUE_TENSOR value),
 * dev_value[1] != 0 applies the update; == 0 performs the restore perturbation only (a
 * NaN loss, optimizer.py:138-141, or a clipped g, :41-42). */
int fks_perturb_step_dev(const fks_tensor* t, int32_t nt, uint64_t seed, const double* scales, const float* dev_value,
                         void* workspace, size_t ws_bytes, void* stream);

/* ---- seed-sharded variant (BASELINE config C3) ----
 * The reconstruct loop of ClientTrainer.train_once (fedkseed.py:136-141) applies K
 * seeds in order, p <- p - lr*(g_k*z_k + wd*p), i.e. with a = 1 - lr*wd
 *     p_K = a^K p_0 - sum_k lr g_k a^(K-1-k) z_k.
 * Ranks can split the seeds, accumulate their part of the sum in f32 and all-reduce it
 * (one RCCL call), then every rank applies p_K.  This is NOT the reference's rounding
 * (the reference rounds every op of every seed to the parameter dtype); it is the
 * variant the north star names, reported with its measured deviation.
 *
 * fks_delta_accumulate: for s = 0..k-1 in order, for every non-frozen tensor i and
 * element e: delta[cum_i + e] = fmaf(f32(coefs[s]), z_s(i, e), delta[cum_i + e]),
 * cum_i = sum of numel over tensors before i (the delta buffer is the tensors'
 * concatenation, f32, 8-byte aligned, device memory); z_s is the reference's stream
 * for seeds[s] and the tensor's dtype (either stream: FKS_STREAM_ROCM selects torch's
 * device generator, the counter-mode stream that needs no jumps).  lr/wd/flags of the tensors are ignored (the
 * caller folds them into coefs).  Workspace: fks_delta_workspace_size.
 * fks_delta_apply: for every non-frozen tensor i: p = dtype(fmaf(f32(decay[i]), p,
 * -delta[cum_i + e])).                                                               */
int fks_delta_workspace_size(const fks_tensor* t, int32_t nt, int32_t k, size_t* bytes);
int fks_delta_accumulate(const fks_tensor* t, int32_t nt, const uint64_t* seeds, const double* coefs, int32_t k,
                         float* delta, void* workspace, size_t ws_bytes, void* stream);
int fks_delta_apply(const fks_tensor* t, int32_t nt, const float* delta, const double* decay, void* workspace,
                    size_t ws_bytes, void* stream);

/* torch.manual_seed(seed); for every tensor in order: p = torch.normal(0, 1, size, dtype). */
int fks_normal(const fks_tensor* t, int32_t nt, uint64_t seed, void* workspace, size_t ws_bytes, void* stream);

/* Thread-local description of the last error (empty string if none). */
const char* fks_last_error(void);

/* ABI version (FKS_ABI_VERSION) and the device target the library was built for. */
int32_t fks_abi_version(void);
const char* fks_build_target(void);
/* Identity of the device code in this library: 16 hex digits of the SHA-256 of the
 * compiled kernel object (fate-llm_amd/Makefile).  Hardware counters profiled from one
 * build (profiles/pmc_*.json) carry it, so a report can check that they belong to the
 * kernels it times (bench.py). */
const char* fks_build_id(void);
/* Identity of the sources: 16 hex digits of the SHA-256 of the concatenated source files the
 * library was built from (fate-llm_amd/Makefile SRCS), so that a prebuilt libfks.so can be
 * checked against the tree it travels with (__graft_entry__.ensure_built rebuilds on a
 * mismatch). */
const char* fks_source_id(void);

/* Host-only self checks (no device needed): the jump-ahead window of `seed` at
 * stream block `block` (= the 624-word generator state before block `block` is
 * drawn) computed from the GF(2) jump polynomial; and the bf16/f16 Box-Muller
 * tables.  Used by the CPU test-suite to pin the host math against the oracle. */
int fks_host_jump_window(uint64_t seed, int64_t block, uint32_t* out624);
int fks_host_tables(int32_t dtype, float* radius, float* cosv, float* sinv, int32_t n);

/* Device self checks of a property a kernel relies on; *result = number of violations
 * (0 = holds), synchronous on `stream`.  FKS_CHECK_SQRT_DOMAIN: the fp32 Box-Muller's
 * radius sqrt(-2 log u1) must be correctly rounded (as _mm256_sqrt_ps is) on all 2^24
 * values of u1 the reference can draw, checked against the exact midpoint criterion;
 * workspace >= 262,144 bytes. */
#define FKS_CHECK_SQRT_DOMAIN 1
/* FKS_CHECK_PHILOX_RADIUS: the torch_rocm stream's Box-Muller radius sqrt(-2 log u) as
 * the torch_rocm kernels compute it (trimmed to the inputs Philox can give) must equal
 * ocml's general sqrtf(-2 logf(u)), the instructions torch's device kernel runs, on all
 * 2^32 words (up to the sign of a zero, which the following "+ 0" erases); same
 * workspace. */
#define FKS_CHECK_PHILOX_RADIUS 2
/* FKS_CHECK_PHILOX_BF16_RADIUS: *result = the largest distance in f32 ulps, over all 2^32
 * words, of the radius the torch_rocm kernel's bf16 fast path computes (log2(u) times
 * RN(-2 ln 2) in one rounding, raw v_sqrt_f32) from ocml's sqrtf(-2 logf(u)); the kernel's
 * bf16 midpoint window assumes at most 2.  Same workspace. */
#define FKS_CHECK_PHILOX_BF16_RADIUS 3
int fks_device_selfcheck(int32_t which, uint64_t* result, void* workspace, size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* FKS_H_ */
