// fks_capi.cpp -- the C ABI of libfks.so (include/fks.h): validation, stream layout,
// chunk plan, workspace carving, seed batching and kernel launches.
//
// Reference routines replaced (include/fks.h lists them): zo_utils.directional_derivative_step
// (zo_utils.py:23-54), ZerothOrderOptimizer.random_perturb_parameters (optimizer.py:152-173),
// and the per-seed reconstruct loop of ClientTrainer.train_once (fedkseed.py:136-141).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "fks_internal.h"

namespace fks {
namespace {

thread_local std::string g_last_error;

// Stream layout: where every tensor's draws sit in the per-seed MT19937 stream.
// Consumption per tensor follows normal_kernel (DistributionTemplates.h:231-256):
//   numel >= 16: numel words (+16 fresh words for the tail recompute if numel % 16 != 0)
//   0 < numel < 16: serial normal_distribution<double>: 4 words (two random64) per NEW
//                   Box-Muller pair, the second value of a pair is cached in the
//                   generator and consumed by the next serial draw (DistributionsHelper.h:189-221)
struct Layout {
  int64_t stream_len = 0;
  std::vector<int64_t> offset;  // per tensor
  std::vector<DevSeg> segs[3];  // regular segments per dtype (non-frozen tensors only)
  std::string irregular;        // description of the first unsupported tensor, if any
};

Layout make_layout(const fks_tensor* t, int nt) {
  Layout L;
  L.offset.resize((size_t)nt);
  bool cached = false;
  int64_t pos = 0;
  for (int i = 0; i < nt; i++) {
    const fks_tensor& x = t[i];
    L.offset[(size_t)i] = pos;
    const int64_t n = x.numel;
    const bool frozen = (x.flags & FKS_FROZEN) != 0;
    if (n >= 16) {
      const bool regular = (n % 16 == 0) && (pos % 16 == 0);
      if (!frozen) {
        if (regular) {
          DevSeg s{};
          s.start = pos;
          s.numel = n;
          s.ptr = (uint64_t)(uintptr_t)x.data;
          s.lr = x.lr;
          s.wd = x.wd;
          s.flags = x.flags;
          s.dtype = x.dtype;
          L.segs[x.dtype].push_back(s);
        } else if (L.irregular.empty()) {
          L.irregular = "tensor " + std::to_string(i) + " (numel " + std::to_string(n) + ", stream offset " +
                        std::to_string(pos) + ") is not on the 16-aligned fast path";
        }
      }
      pos += n + (n % 16 ? 16 : 0);
    } else if (n > 0) {
      if (!frozen && L.irregular.empty())
        L.irregular = "tensor " + std::to_string(i) + " has numel " + std::to_string(n) +
                      " < 16 (torch's serial normal_distribution<double> path)";
      for (int64_t e = 0; e < n; e++) {
        if (cached) cached = false;
        else { pos += 4; cached = true; }
      }
    }
  }
  L.stream_len = pos;
  return L;
}

void validate(const fks_tensor* t, int nt) {
  if (nt < 0 || (nt > 0 && !t)) throw Error(-FKS_EINVAL, "bad tensor list");
  for (int i = 0; i < nt; i++) {
    const fks_tensor& x = t[i];
    if (x.numel < 0) throw Error(-FKS_EINVAL, "tensor " + std::to_string(i) + ": negative numel");
    if (x.dtype != FKS_F32 && x.dtype != FKS_BF16 && x.dtype != FKS_F16)
      throw Error(-FKS_EINVAL, "tensor " + std::to_string(i) + ": unsupported dtype code " + std::to_string(x.dtype));
    if (x.dtype == FKS_F16)
      throw Error(-FKS_ENOTSUP, "tensor " + std::to_string(i) + ": float16 parameters are not implemented on the MI355X path yet");
    const size_t es = x.dtype == FKS_F32 ? 4 : 2;
    if (x.numel > 0 && (!x.data || ((uintptr_t)x.data % es) != 0))
      throw Error(-FKS_EINVAL, "tensor " + std::to_string(i) + ": null or misaligned data pointer");
    if (x.flags & ~(FKS_HAS_WD | FKS_FROZEN)) throw Error(-FKS_EINVAL, "tensor " + std::to_string(i) + ": unknown flags");
  }
}

// Chunk plan: MT blocks [chunk_block[c], chunk_block[c+1]) per workgroup.
struct Plan {
  int nchunks = 0;
  std::vector<int64_t> chunk_block;  // nchunks + 1
  std::vector<uint64_t> polys;       // nchunks * 312
};

// MT blocks of the whole stream and the [lo, hi) range shard `shard` of `nshards` owns
struct BlockRange { int64_t lo, hi; };
BlockRange shard_blocks(int64_t stream_len, int shard, int nshards) {
  const int64_t nb = std::max<int64_t>(1, (stream_len + kMtN - 1) / kMtN);
  return {(int64_t)((__int128)nb * shard / nshards), (int64_t)((__int128)nb * (shard + 1) / nshards)};
}

int plan_nchunks(int64_t nblocks) {
  const int64_t target = (int64_t)kApplyWgPerCu * device_cu_count();  // one wave of apply workgroups
  return (int)std::max<int64_t>(1, std::min<int64_t>(nblocks, target));
}

Plan make_plan(BlockRange r) {
  Plan P;
  const int64_t nblocks = std::max<int64_t>(1, r.hi - r.lo);
  P.nchunks = plan_nchunks(nblocks);
  P.chunk_block.resize((size_t)P.nchunks + 1);
  for (int c = 0; c <= P.nchunks; c++)
    P.chunk_block[(size_t)c] = r.lo + (int64_t)((__int128)nblocks * c / P.nchunks);
  std::vector<int64_t> starts(P.chunk_block.begin(), P.chunk_block.end() - 1);
  jump_polys_for_blocks(starts, P.polys);
  return P;
}

// keep only the part of every segment inside the block range (16-aligned cuts)
void clip_segments(Layout& L, BlockRange r) {
  const int64_t lo = r.lo * kMtN, hi = r.hi * kMtN;
  for (int d = 0; d < 3; d++) {
    std::vector<DevSeg> out;
    for (const DevSeg& s : L.segs[d]) {
      const int64_t a = std::max(s.start, lo), b = std::min(s.start + s.numel, hi);
      if (a >= b) continue;
      DevSeg c = s;
      const size_t es = s.dtype == FKS_F32 ? 4 : 2;
      c.ptr = s.ptr + (uint64_t)(a - s.start) * es;
      c.start = a;
      c.numel = b - a;
      out.push_back(c);
    }
    L.segs[d].swap(out);
  }
}

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct WsLayout {
  size_t header = 0;      // bytes of the uploaded header (polys, chunk_block, segs, seeds, g)
  size_t off_polys = 0, off_cb = 0, off_segs = 0, off_seeds = 0, off_g = 0, off_states = 0;
  size_t total = 0;
};

WsLayout ws_layout(int nchunks, int nsegs_total, int k) {
  WsLayout w;
  size_t o = 0;
  w.off_polys = o; o = align_up(o + sizeof(uint64_t) * 312 * (size_t)nchunks, 256);
  w.off_cb = o;    o = align_up(o + sizeof(int64_t) * ((size_t)nchunks + 1), 256);
  w.off_segs = o;  o = align_up(o + sizeof(DevSeg) * (size_t)std::max(nsegs_total, 1), 256);
  w.off_seeds = o; o = align_up(o + sizeof(uint64_t) * (size_t)std::max(k, 1), 256);
  w.off_g = o;     o = align_up(o + sizeof(float) * 3 * (size_t)std::max(k, 1), 256);
  w.header = o;
  w.off_states = o;
  o = align_up(o + sizeof(uint32_t) * kMtN * (size_t)kMaxSeedsPerPass * (size_t)nchunks, 256);
  w.total = o;
  return w;
}

int nsegs_total(const Layout& L) { return (int)(L.segs[0].size() + L.segs[1].size() + L.segs[2].size()); }

inline float round_to_dtype(double v, int dtype) {
  float f = (float)v;
  if (dtype == FKS_F32 || f != f) return f;
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if (dtype == FKS_BF16) {
    u = (u + (((u >> 16) & 1u) + 0x7FFFu)) & 0xFFFF0000u;
    std::memcpy(&f, &u, 4);
    return f;
  }
  return f;  // f16 not reachable (rejected in validate)
}

// Core: run `k` seeds (update / perturb / write-z) over the tensor list.
// launch-time instrumentation (fks_profile_begin/end): events around every launch
struct Prof {
  bool on = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[2];  // 0 = apply, 1 = jump
};
Prof g_prof;
std::mutex g_prof_mu;

template <class F>
int timed(int which, void* stream, F&& launch) {
  std::unique_lock<std::mutex> lk(g_prof_mu);
  if (!g_prof.on) {
    lk.unlock();
    return launch();
  }
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, (hipStream_t)stream);
  const int rc = launch();
  hipEventRecord(b, (hipStream_t)stream);
  g_prof.ev[which].emplace_back(a, b);
  return rc;
}

void run(const fks_tensor* t, int nt, const uint64_t* seeds, const double* values, int k, int value_kind, int mode,
         void* workspace, size_t ws_bytes, void* stream, const double* tensor_scales = nullptr, int shard = 0,
         int nshards = 1) {
  validate(t, nt);
  if (nshards < 1 || shard < 0 || shard >= nshards) throw Error(-FKS_EINVAL, "bad shard");
  if (k < 0 || (k > 0 && (!seeds || !values))) throw Error(-FKS_EINVAL, "bad seed/value arrays");
  if (value_kind != FKS_VALUE_SCALAR && value_kind != FKS_VALUE_TENSOR)
    throw Error(-FKS_EINVAL, "bad value_kind");
  std::vector<fks_tensor> tt;
  if (tensor_scales) {  // perturb: the per-tensor scale rides in the lr slot (kModePerturb reads it)
    tt.assign(t, t + nt);
    for (int i = 0; i < nt; i++) tt[(size_t)i].lr = (float)tensor_scales[i];
    t = tt.data();
  }
  Layout L = make_layout(t, nt);
  if (!L.irregular.empty())
    throw Error(-FKS_ENOTSUP, "irregular tensor layout not supported by the MI355X fast path: " + L.irregular);
  const BlockRange br = shard_blocks(L.stream_len, shard, nshards);
  clip_segments(L, br);
  if (k == 0 || nsegs_total(L) == 0) return;
  Plan P = make_plan(br);
  const WsLayout W = ws_layout(P.nchunks, nsegs_total(L), k);
  if (!workspace || ws_bytes < W.total)
    throw Error(-FKS_EINVAL, "workspace too small: need " + std::to_string(W.total) + " bytes, got " +
                                 std::to_string(ws_bytes));
  // header upload (one async H2D copy from a per-thread host buffer; a pageable
  // source is staged before hipMemcpyAsync returns, so the buffer is reusable)
  thread_local std::vector<uint8_t> host;
  host.assign(W.header, 0);
  std::memcpy(host.data() + W.off_polys, P.polys.data(), sizeof(uint64_t) * P.polys.size());
  std::memcpy(host.data() + W.off_cb, P.chunk_block.data(), sizeof(int64_t) * P.chunk_block.size());
  size_t so = W.off_segs;
  size_t seg_off[3];
  for (int d = 0; d < 3; d++) {
    seg_off[d] = so;
    if (!L.segs[d].empty()) std::memcpy(host.data() + so, L.segs[d].data(), sizeof(DevSeg) * L.segs[d].size());
    so += sizeof(DevSeg) * L.segs[d].size();
  }
  std::memcpy(host.data() + W.off_seeds, seeds, sizeof(uint64_t) * (size_t)k);
  float* gh = reinterpret_cast<float*>(host.data() + W.off_g);
  for (int d = 0; d < 3; d++)
    for (int s = 0; s < k; s++)
      gh[(size_t)d * k + s] = value_kind == FKS_VALUE_TENSOR ? round_to_dtype(values[s], d) : (float)values[s];
  uint8_t* ws = static_cast<uint8_t*>(workspace);
  hipError_t e = hipMemcpyAsync(ws, host.data(), W.header, hipMemcpyHostToDevice, (hipStream_t)stream);
  if (e != hipSuccess) throw Error(-FKS_EHIP, std::string("hipMemcpyAsync: ") + hipGetErrorString(e));

  const int chunks_per_wg = std::max(1, std::min(32, P.nchunks));  // 2 jumps per wave (16 waves)
  for (int s0 = 0; s0 < k; s0 += kMaxSeedsPerPass) {
    const int nb = std::min(kMaxSeedsPerPass, k - s0);
    JumpArgs ja{};
    ja.seeds = reinterpret_cast<const uint64_t*>(ws + W.off_seeds) + s0;
    ja.polys = reinterpret_cast<const uint64_t*>(ws + W.off_polys);
    ja.chunk_block = reinterpret_cast<const int64_t*>(ws + W.off_cb);
    ja.states = reinterpret_cast<uint32_t*>(ws + W.off_states);
    ja.nchunks = P.nchunks;
    ja.chunks_per_wg = chunks_per_wg;
    int rc = timed(1, stream, [&] { return launch_jump(ja, nb, stream); });
    if (rc) throw Error(-FKS_EHIP, std::string("fks_jump_kernel launch: ") + hipGetErrorString((hipError_t)rc));
    for (int d = 0; d < 3; d++) {
      if (L.segs[d].empty()) continue;
      ApplyArgs aa{};
      aa.states = ja.states;
      aa.g = reinterpret_cast<const float*>(ws + W.off_g) + (size_t)d * k + s0;
      aa.segs = reinterpret_cast<const DevSeg*>(ws + seg_off[d]);
      aa.chunk_block = ja.chunk_block;
      aa.nsegs = (int)L.segs[d].size();
      aa.nchunks = P.nchunks;
      aa.nseeds = nb;
      aa.mode = mode;
      rc = timed(0, stream, [&] { return launch_apply(d, aa, stream); });
      if (rc) throw Error(rc < 0 ? rc : -FKS_EHIP, std::string("fks_apply_kernel launch: ") +
                                                         (rc > 0 ? hipGetErrorString((hipError_t)rc) : "unsupported"));
    }
  }
}

template <class F>
int guarded(F&& f) {
  try {
    g_last_error.clear();
    f();
    return 0;
  } catch (const Error& e) {
    g_last_error = e.what();
    return e.code;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return -FKS_EINVAL;
  } catch (...) {
    g_last_error = "unknown error";
    return -FKS_EINVAL;
  }
}

}  // namespace
}  // namespace fks

using namespace fks;

extern "C" {

int fks_workspace_size(const fks_tensor* t, int32_t nt, int32_t k, size_t* bytes) {
  return guarded([&] {
    validate(t, nt);
    if (!bytes || k < 0) throw Error(-FKS_EINVAL, "bad arguments");
    Layout L = make_layout(t, nt);
    const BlockRange br = shard_blocks(L.stream_len, 0, 1);
    *bytes = ws_layout(plan_nchunks(br.hi - br.lo), nsegs_total(L), std::max(k, 1)).total;
  });
}

int fks_directional_step(const fks_tensor* t, int32_t nt, const uint64_t* seeds, const double* values, int32_t k,
                         int32_t value_kind, void* workspace, size_t ws_bytes, void* stream) {
  return guarded([&] { run(t, nt, seeds, values, k, value_kind, kModeUpdate, workspace, ws_bytes, stream); });
}

int fks_directional_step_shard(const fks_tensor* t, int32_t nt, const uint64_t* seeds, const double* values,
                               int32_t k, int32_t value_kind, int32_t shard, int32_t nshards, void* workspace,
                               size_t ws_bytes, void* stream) {
  return guarded([&] {
    run(t, nt, seeds, values, k, value_kind, kModeUpdate, workspace, ws_bytes, stream, nullptr, shard, nshards);
  });
}

int fks_stream_length(const fks_tensor* t, int32_t nt, int64_t* words) {
  return guarded([&] {
    validate(t, nt);
    if (!words) throw Error(-FKS_EINVAL, "null output");
    *words = make_layout(t, nt).stream_len;
  });
}

int fks_profile_begin(void) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_prof.on = true;
  return 0;
}

int fks_profile_end(double* apply_ms, int64_t* n_apply, double* jump_ms, int64_t* n_jump) {
  return guarded([&] {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    double tot[2] = {0.0, 0.0};
    for (int w = 0; w < 2; w++) {
      for (auto& e : g_prof.ev[w]) {
        hipEventSynchronize(e.second);
        float ms = 0.0f;
        hipEventElapsedTime(&ms, e.first, e.second);
        tot[w] += ms;
        hipEventDestroy(e.first);
        hipEventDestroy(e.second);
      }
    }
    if (apply_ms) *apply_ms = tot[0];
    if (jump_ms) *jump_ms = tot[1];
    if (n_apply) *n_apply = (int64_t)g_prof.ev[0].size();
    if (n_jump) *n_jump = (int64_t)g_prof.ev[1].size();
    g_prof.ev[0].clear();
    g_prof.ev[1].clear();
    g_prof.on = false;
  });
}

int fks_perturb(const fks_tensor* t, int32_t nt, uint64_t seed, const double* scales, void* workspace,
                size_t ws_bytes, void* stream) {
  return guarded([&] {
    // optimizer.py:173: scaling_factor * eps is a python double, cast to fp32 opmath
    if (nt > 0 && !scales) throw Error(-FKS_EINVAL, "null scales");
    const double one = 1.0;
    run(t, nt, &seed, &one, 1, FKS_VALUE_SCALAR, kModePerturb, workspace, ws_bytes, stream, scales);
  });
}

int fks_normal(const fks_tensor* t, int32_t nt, uint64_t seed, void* workspace, size_t ws_bytes, void* stream) {
  return guarded([&] {
    const double v = 0.0;
    run(t, nt, &seed, &v, 1, FKS_VALUE_SCALAR, kModeWriteZ, workspace, ws_bytes, stream);
  });
}

const char* fks_last_error(void) { return g_last_error.c_str(); }

int32_t fks_abi_version(void) { return FKS_ABI_VERSION; }

const char* fks_build_target(void) { return "gfx950"; }

int fks_host_jump_window(uint64_t seed, int64_t block, uint32_t* out624) {
  return guarded([&] {
    if (!out624 || block < 0) throw Error(-FKS_EINVAL, "bad arguments");
    host_jump_window(seed, block, out624);
  });
}

int fks_host_tables(int32_t dtype, float* radius, float* cosv, float* sinv, int32_t n) {
  return guarded([&] {
    const Tables& T = tables();
    const int need = dtype == FKS_BF16 ? 256 : (dtype == FKS_F16 ? 2048 : -1);
    if (need < 0 || n < need || !radius || !cosv || !sinv) throw Error(-FKS_EINVAL, "bad arguments");
    const float* r = dtype == FKS_BF16 ? T.r_bf16 : T.r_f16;
    const float* c = dtype == FKS_BF16 ? T.c_bf16 : T.c_f16;
    const float* s = dtype == FKS_BF16 ? T.s_bf16 : T.s_f16;
    std::memcpy(radius, r, sizeof(float) * (size_t)need);
    std::memcpy(cosv, c, sizeof(float) * (size_t)need);
    std::memcpy(sinv, s, sizeof(float) * (size_t)need);
  });
}

}  // extern "C"
