// fks_capi.cpp -- the C ABI of libfks.so (include/fks.h): validation, stream layout,
// chunk plan, workspace carving, seed batching and kernel launches.
//
// Reference routines replaced (include/fks.h lists them): zo_utils.directional_derivative_step
// (zo_utils.py:23-54), ZerothOrderOptimizer.random_perturb_parameters (optimizer.py:152-173),
// and the per-seed reconstruct loop of ClientTrainer.train_once (fedkseed.py:136-141).
#include <unordered_map>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cctype>
#include <cstdlib>
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
  std::vector<DevSeg> segs[3];  // fast-path segments per dtype (non-frozen tensors only)
  std::vector<DevRun> runs;     // irregular 16-block runs (all dtypes), sorted by start
  std::vector<DevTiny> tiny;    // single elements of numel < 16 tensors, sorted by word
  // host-only: the tensor index of every segment / run / element (fks_shard_census)
  std::vector<int> seg_tensor[3], run_tensor, tiny_tensor;
  // seed-sharded variant (fks_delta_accumulate): the descriptors address the f32 delta
  // buffer (element e of tensor i at delta[cum_numel(i) + e]) instead of the parameters;
  // the dtype still selects the z generator
  bool delta = false;
  // the generator after the list's draws: CPUGeneratorImpl::next_double_normal_sample holds
  // the second value of the Box-Muller pair at stream word end_pair (fks_cpu_generator_end)
  bool end_cached = false;
  int64_t end_pair = 0;
};

inline size_t elem_size(int dtype) { return dtype == FKS_F32 ? 4 : 2; }
// bytes per element of what the kernels load and store
inline size_t stor_size(const Layout& L, int dtype) { return L.delta ? 4 : elem_size(dtype); }

// The fast kernel takes a tensor whose 16-blocks sit on 16-aligned stream words (so
// none straddles an MT block), with no tail recompute, f32/bf16, 2-element aligned
// (it moves adjacent element pairs); everything else goes to the irregular kernel.
Layout make_layout(const fks_tensor* t, int nt, const double* scales = nullptr, uint64_t delta_base = 0) {
  Layout L;
  L.delta = delta_base != 0;
  L.offset.resize((size_t)nt);
  int64_t cum = 0;  // concatenated element offset (delta layout)
  bool cached = false;   // CPUGeneratorImpl::next_double_normal_sample
  int64_t cached_pair = 0;
  int64_t pos = 0;
  for (int i = 0; i < nt; i++) {
    const fks_tensor& x = t[i];
    L.offset[(size_t)i] = pos;
    const int64_t n = x.numel;
    const bool live = (x.flags & FKS_FROZEN) == 0;
    const uint64_t ptr = L.delta ? delta_base + 4 * (uint64_t)cum : (uint64_t)(uintptr_t)x.data;
    const size_t es = stor_size(L, x.dtype);
    cum += n;
    // optimizer.py:173: scaling_factor * eps is a python double, cast to the fp32 opmath
    const float ps = scales ? (float)scales[i] : 0.0f;
    if (n >= 16) {
      const bool fast = n % 16 == 0 && pos % 16 == 0 && x.dtype != FKS_F16 && ptr % (2 * es) == 0;
      if (live && fast) {
        DevSeg s{};
        s.start = pos;
        s.numel = n;
        s.ptr = ptr;
        s.lr = x.lr;
        s.wd = x.wd;
        s.flags = x.flags;
        s.dtype = x.dtype;
        s.ps = ps;
        L.segs[x.dtype].push_back(s);
        L.seg_tensor[x.dtype].push_back(i);
      } else if (live) {
        // words [pos, pos + 16F) hold F = n / 16 whole 16-blocks; if n % 16 != 0 the last
        // 16 elements are redrawn from 16 fresh words [pos + n, pos + n + 16) and the head
        // run must not write them (DistributionTemplates.h:118-124 / :221-228)
        const int64_t F = n / 16;
        DevRun r{};
        r.start = pos;
        r.numel = 16 * F;
        r.ptr = ptr;
        r.limit = n % 16 ? n - 16 : n;
        r.lr = x.lr;
        r.wd = x.wd;
        r.flags = x.flags;
        r.dtype = x.dtype;
        r.ps = ps;
        L.runs.push_back(r);
        L.run_tensor.push_back(i);
        if (n % 16) {
          DevRun tl = r;
          tl.start = pos + n;
          tl.numel = 16;
          tl.ptr = ptr + (uint64_t)(n - 16) * es;
          tl.limit = 16;
          L.runs.push_back(tl);
          L.run_tensor.push_back(i);
        }
      }
      pos += n + (n % 16 ? 16 : 0);
    } else if (n > 0) {
      for (int64_t e = 0; e < n; e++) {
        DevTiny d{};
        if (cached) {
          cached = false;
          d.word = cached_pair;
          d.flags = kTinySin;
        } else {
          cached = true;
          cached_pair = d.word = pos;
          pos += 4;
        }
        if (!live) continue;
        d.ptr = ptr + (uint64_t)e * es;
        d.lr = x.lr;
        d.wd = x.wd;
        d.flags |= x.flags & FKS_HAS_WD;
        d.dtype = x.dtype;
        d.ps = ps;
        L.tiny.push_back(d);
        L.tiny_tensor.push_back(i);
      }
    }
  }
  L.stream_len = pos;
  L.end_cached = cached;
  L.end_pair = cached_pair;
  // runs are disjoint and already in stream order; single elements sorted by the
  // block holding their last word, the order the kernel walks them in
  std::vector<size_t> order(L.tiny.size());
  for (size_t j = 0; j < order.size(); j++) order[j] = j;
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return L.tiny[a].word < L.tiny[b].word; });
  std::vector<DevTiny> tiny(order.size());
  std::vector<int> tiny_tensor(order.size());
  for (size_t j = 0; j < order.size(); j++) {
    tiny[j] = L.tiny[order[j]];
    tiny_tensor[j] = L.tiny_tensor[order[j]];
  }
  L.tiny.swap(tiny);
  L.tiny_tensor.swap(tiny_tensor);
  return L;
}

void validate(const fks_tensor* t, int nt) {
  if (nt < 0 || (nt > 0 && !t)) throw Error(-FKS_EINVAL, "bad tensor list");
  for (int i = 0; i < nt; i++) {
    const fks_tensor& x = t[i];
    if (x.numel < 0) throw Error(-FKS_EINVAL, "tensor " + std::to_string(i) + ": negative numel");
    if (x.dtype != FKS_F32 && x.dtype != FKS_BF16 && x.dtype != FKS_F16)
      throw Error(-FKS_EINVAL, "tensor " + std::to_string(i) + ": unsupported dtype code " + std::to_string(x.dtype));
    const size_t es = elem_size(x.dtype);
    if (x.numel > 0 && (!x.data || ((uintptr_t)x.data % es) != 0))
      throw Error(-FKS_EINVAL, "tensor " + std::to_string(i) + ": null or misaligned data pointer");
    if (x.flags & ~(FKS_HAS_WD | FKS_FROZEN | FKS_STREAM_ROCM | FKS_FRESH | FKS_LIBM))
      throw Error(-FKS_EINVAL, "tensor " + std::to_string(i) + ": unknown flags");
    if ((x.flags & (FKS_STREAM_ROCM | FKS_LIBM)) != (t[0].flags & (FKS_STREAM_ROCM | FKS_LIBM)))
      throw Error(-FKS_EINVAL, "tensor " + std::to_string(i) + ": every tensor of a call must use the same z stream");
    if ((x.flags & FKS_STREAM_ROCM) && (x.flags & FKS_LIBM))
      throw Error(-FKS_EINVAL, "tensor " + std::to_string(i) + ": FKS_LIBM is a flavour of the CPU generator's stream");
  }
}

bool rocm_stream(const fks_tensor* t, int nt) { return nt > 0 && (t[0].flags & FKS_STREAM_ROCM) != 0; }
// fp32 z of the CPU stream from normal_fill_16<float> with glibc's functions (kDtF32Libm)
bool libm_flavour(const fks_tensor* t, int nt) { return nt > 0 && (t[0].flags & FKS_LIBM) != 0; }

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

// one wave of apply workgroups: kApplyWgPerCu per CU for the 19-seed passes, more for
// calls of at most kSmallK seeds (little LDS per workgroup, so more independent streams
// per CU hide the per-block latency chain)
int plan_nchunks(int64_t nblocks, bool small = false) {
  const int64_t target = (int64_t)(small ? kSmallWgPerCu : kApplyWgPerCu) * device_cu_count();
  return (int)std::max<int64_t>(1, std::min<int64_t>(nblocks, target));
}

Plan plan_from_blocks(std::vector<int64_t> chunk_block) {
  Plan P;
  P.nchunks = (int)chunk_block.size() - 1;
  P.chunk_block = std::move(chunk_block);
  std::vector<int64_t> starts(P.chunk_block.begin(), P.chunk_block.end() - 1);
  jump_polys_for_blocks(starts, P.polys);
  return P;
}

Plan make_plan(BlockRange r, bool small) {
  const int64_t nblocks = std::max<int64_t>(1, r.hi - r.lo);
  const int nchunks = plan_nchunks(nblocks, small);
  std::vector<int64_t> cb((size_t)nchunks + 1);
  for (int c = 0; c <= nchunks; c++) cb[(size_t)c] = r.lo + (int64_t)((__int128)nblocks * c / nchunks);
  return plan_from_blocks(std::move(cb));
}

// MT block holding stream word w
inline int64_t block_of(int64_t w) { return w / kMtN; }

// keep only the work whose owner block lies in the range: fast segments are cut at
// block boundaries (16-aligned), a run keeps the 16-blocks whose last word is inside,
// a single element stays where its draw pair ends
void clip_segments(Layout& L, BlockRange r) {
  const int64_t lo = r.lo * kMtN, hi = r.hi * kMtN;
  for (int d = 0; d < 3; d++) {
    std::vector<DevSeg> out;
    std::vector<int> out_t;
    for (size_t j = 0; j < L.segs[d].size(); j++) {
      const DevSeg& s = L.segs[d][j];
      const int64_t a = std::max(s.start, lo), b = std::min(s.start + s.numel, hi);
      if (a >= b) continue;
      DevSeg c = s;
      c.ptr = s.ptr + (uint64_t)(a - s.start) * stor_size(L, s.dtype);
      c.start = a;
      c.numel = b - a;
      out.push_back(c);
      out_t.push_back(L.seg_tensor[d][j]);
    }
    L.segs[d].swap(out);
    L.seg_tensor[d].swap(out_t);
  }
  std::vector<DevRun> runs;
  std::vector<int> runs_t;
  for (size_t j = 0; j < L.runs.size(); j++) {
    const DevRun& R = L.runs[j];
    const int64_t nb = R.numel / 16;
    // 16-block i ends at word R.start + 16 i + 15
    auto first_at_or_after = [&](int64_t w) {
      const int64_t d = w - (R.start + 15);
      return std::min(nb, std::max<int64_t>(0, (d + 15) / 16 * (d > 0)));
    };
    const int64_t i0 = first_at_or_after(lo), i1 = first_at_or_after(hi);
    if (i0 >= i1) continue;
    DevRun c = R;
    c.start = R.start + 16 * i0;
    c.numel = 16 * (i1 - i0);
    c.ptr = R.ptr + (uint64_t)(16 * i0) * stor_size(L, R.dtype);
    c.limit = R.limit - 16 * i0;
    runs.push_back(c);
    runs_t.push_back(L.run_tensor[j]);
  }
  L.runs.swap(runs);
  L.run_tensor.swap(runs_t);
  std::vector<DevTiny> tiny;
  std::vector<int> tiny_t;
  for (size_t j = 0; j < L.tiny.size(); j++) {
    const DevTiny& T = L.tiny[j];
    if (T.word + 3 >= lo && T.word + 3 < hi) {
      tiny.push_back(T);
      tiny_t.push_back(L.tiny_tensor[j]);
    }
  }
  L.tiny.swap(tiny);
  L.tiny_tensor.swap(tiny_t);
}

// Chunks of the irregular kernel: the MT blocks that own irregular work, split into at
// most plan_nchunks() groups of about equal work; a chunk twists through the blocks
// between its first and last owner block.
struct IrrChunks {
  std::vector<int64_t> lo, hi;  // chunk c twists blocks [lo[c], hi[c])
};
std::vector<std::pair<int64_t, int64_t>> irregular_owner_intervals(const Layout& L) {
  std::vector<std::pair<int64_t, int64_t>> iv;  // owner block intervals [a, b)
  for (const DevRun& R : L.runs) iv.emplace_back(block_of(R.start + 15), block_of(R.start + R.numel - 1) + 1);
  for (const DevTiny& T : L.tiny) iv.emplace_back(block_of(T.word + 3), block_of(T.word + 3) + 1);
  std::sort(iv.begin(), iv.end());
  std::vector<std::pair<int64_t, int64_t>> merged;
  for (auto& x : iv) {
    if (!merged.empty() && x.first <= merged.back().second) merged.back().second = std::max(merged.back().second, x.second);
    else merged.push_back(x);
  }
  return merged;
}

int64_t irregular_covered_blocks(const Layout& L) {
  int64_t covered = 0;
  for (auto& x : irregular_owner_intervals(L)) covered += x.second - x.first;
  return covered;
}

IrrChunks irregular_chunks(const Layout& L) {
  const auto merged = irregular_owner_intervals(L);
  if (merged.empty()) return IrrChunks{};
  int64_t covered = 0;
  for (auto& x : merged) covered += x.second - x.first;
  const int cap = plan_nchunks(covered);
  const int64_t q = (covered + cap - 1) / cap;  // owner blocks per chunk
  IrrChunks out;
  int64_t in_chunk = 0, chunk_lo = -1, last_hi = -1;
  auto close = [&] {
    out.lo.push_back(chunk_lo);
    out.hi.push_back(last_hi);
    chunk_lo = -1;
    in_chunk = 0;
  };
  for (auto& x : merged) {
    int64_t a = x.first;
    while (a < x.second) {
      if (chunk_lo < 0) chunk_lo = a;
      const int64_t take = std::min(x.second - a, q - in_chunk);
      a += take;
      in_chunk += take;
      last_hi = a;
      if (in_chunk == q) close();
    }
  }
  if (chunk_lo >= 0) close();
  return out;
}

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Static header of a call: everything that depends only on the tensor list, the
// perturbation scales, the shard and the chunk policy -- the chunk table, the jump
// polynomials and the segment / run / element descriptors.  It lives on the device in
// the plan cache (PlanCache below) and is uploaded once per distinct tensor list; the
// per-pass seeds and multipliers travel by value in the kernel arguments.
struct HdrSizes {
  int reg_chunks = 0, irr_chunks = 0, nsegs = 0, nruns = 0, ntiny = 0;
  int bs_chunks = 0;  // the bf16 slice kernel's own chunk plan (0: not used)
};

struct HdrLayout {
  size_t off_polys = 0, off_cb = 0, off_ipolys = 0, off_ilo = 0, off_ihi = 0, off_segs = 0, off_runs = 0,
         off_tiny = 0, off_bs_polys = 0, off_bs_cb = 0;
  size_t total = 0;
};

HdrLayout hdr_layout(const HdrSizes& z) {
  HdrLayout w;
  size_t o = 0;
  auto put = [&](size_t& off, size_t bytes) { off = o; o = align_up(o + std::max<size_t>(bytes, 1), 256); };
  put(w.off_polys, sizeof(uint64_t) * 312 * (size_t)z.reg_chunks);
  put(w.off_cb, sizeof(int64_t) * ((size_t)z.reg_chunks + 1));
  put(w.off_ipolys, sizeof(uint64_t) * 312 * (size_t)z.irr_chunks);
  put(w.off_ilo, sizeof(int64_t) * (size_t)z.irr_chunks);
  put(w.off_ihi, sizeof(int64_t) * (size_t)z.irr_chunks);
  put(w.off_segs, sizeof(DevSeg) * (size_t)z.nsegs);
  put(w.off_runs, sizeof(DevRun) * (size_t)z.nruns);
  put(w.off_tiny, sizeof(DevTiny) * (size_t)z.ntiny);
  put(w.off_bs_polys, sizeof(uint64_t) * 312 * (size_t)z.bs_chunks);
  put(w.off_bs_cb, sizeof(int64_t) * ((size_t)z.bs_chunks + 1));
  w.total = o;
  return w;
}

// Caller's workspace: [sink 4 KB | generator windows of one pass]; the small-K kernel's
// lanes read a whole block's worth of sink when their block is not a fast one
constexpr size_t kWsStatesOff = 4096;
size_t ws_bytes_for(int chunks, int seeds_per_pass) {
  return kWsStatesOff + sizeof(uint32_t) * kMtN * (size_t)seeds_per_pass * (size_t)std::max(chunks, 1);
}

// the slice kernel's plan: two chunks per workgroup, one workgroup per CU (a pass of
// > 32 seeds runs two seed slices on each chunk PAIR, a pass of <= 32 one slice per chunk)
int bs_nchunks(int64_t nblocks) {
  const int64_t wgs = std::max<int64_t>(1, std::min<int64_t>(device_cu_count(), (nblocks + 1) / 2));
  return (int)(kBsChunksPerWg * wgs);
}

Plan make_plan_n(BlockRange r, int nchunks) {
  const int64_t nblocks = std::max<int64_t>(1, r.hi - r.lo);
  std::vector<int64_t> cb((size_t)nchunks + 1);
  for (int c = 0; c <= nchunks; c++) cb[(size_t)c] = r.lo + (int64_t)((__int128)nblocks * c / nchunks);
  return plan_from_blocks(std::move(cb));
}

int nsegs_total(const Layout& L) { return (int)(L.segs[0].size() + L.segs[1].size() + L.segs[2].size()); }

// float -> binary16 -> float, round to nearest even (c10::Half)
inline float round_f16(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint32_t sign = x & 0x80000000u, ax = x & 0x7fffffffu;
  float r;
  if (ax >= 0x477ff000u) {
    x = sign | 0x7f800000u;
  } else if (ax < 0x38800000u) {  // half subnormal: quantum 2^-24
    std::memcpy(&r, &ax, 4);
    r = std::nearbyint(r * 16777216.0f) / 16777216.0f;
    std::memcpy(&x, &r, 4);
    x |= sign;
  } else {
    uint32_t keep = ax & ~0x1fffu;
    const uint32_t rem = ax & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (keep & 0x2000u))) keep += 0x2000u;
    x = sign | keep;
  }
  std::memcpy(&r, &x, 4);
  return r;
}

// a 0-dim fp32 tensor g enters `g * z` as the first operand: torch casts it to the
// parameter dtype first (zo step's g, optimizer.py:147)
inline float round_to_dtype(double v, int dtype) {
  float f = (float)v;
  if (dtype == FKS_F32 || f != f) return f;
  if (dtype == FKS_F16) return round_f16(f);
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u = (u + (((u >> 16) & 1u) + 0x7FFFu)) & 0xFFFF0000u;
  std::memcpy(&f, &u, 4);
  return f;
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
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, (hipStream_t)stream);
  const int rc = launch();
  (void)hipEventRecord(b, (hipStream_t)stream);
  g_prof.ev[which].emplace_back(a, b);
  return rc;
}

// ------------------------------------------------------------------ plan cache
// The static header of a call, resident on the device.  Keyed by every input the
// header depends on (device, CU count, each tensor's address/numel/dtype/flags/lr/wd,
// the perturbation scales as f32, the delta base, the shard, the chunk policy); the
// full key is compared, not only its hash.  The ZO optimizer's perturb / update calls
// and repeated reconstructs of one model hit the cache: a call then does no host-side
// layout work and no upload.  Bounded LRU; entries are never freed while in use
// (launches are stream-ordered after the synchronous upload of their header).
struct CachedPlan {
  std::vector<uint8_t> key;
  uint64_t hash = 0, last_use = 0;
  void* dev = nullptr;
  int device = 0;  // the HIP device `dev` lives on
  HdrLayout H;
  HdrSizes Z;
  size_t seg_off[3] = {0, 0, 0};
  int nsegs[3] = {0, 0, 0};
  int wd_mode[3] = {kModeUpdate, kModeUpdate, kModeUpdate};  // kModeUpdateWd / NoWd when uniform
  bool have_reg = false, have_irr = false;
  bool have_bs = false;  // bf16 fast segments with their slice-kernel plan (non-small calls)
  uint64_t chunk_hash = 0;  // the chunk starts (regular + irregular): what a seed's windows depend on
  int64_t reg_lo = 0, reg_hi = 0;  // MT blocks [reg_lo, reg_hi) the regular chunks cover
  uint64_t bf16_hash = 0;  // the bf16 segments' stream ranges: which blocks a z-index store covers
  uint64_t bs_hash = 0;    // the slice-kernel plan's chunk starts: what its seeds' windows depend on
};

// Table indices of the last one-seed bf16 perturb, per device (ZO step: the second and
// third calls replay them, fks_small2_kernel ZM 2).  A block's indices depend only on
// the seed and the block's stream position, not on the tensors, so any later one-seed
// call with the same seed and the same bf16 segment ranges (a store covers the blocks of
// its own bf16 segments only) whose regular blocks lie inside the stored range replays them.
// The buffer is the CALLER's (fks_zindex_attach: the Python codec allocates it through
// torch's allocator under a memory budget), 1 byte per parameter; without one attached,
// or with FKS_ZCACHE=0, every call generates.  Stream hand-off by event, as WinCache.
struct ZCache {
  int device = -1;
  void* buf = nullptr;
  size_t bytes = 0;
  void* stream = nullptr;
  hipEvent_t done = nullptr;
  bool valid = false;
  uint64_t seed = 0, bf16_hash = 0;
  int64_t lo = 0, hi = 0;
};

// Jumped windows of the last one-seed call, per device.  The ZO step makes three calls
// with the same seed over the same parameters (perturb +eps, perturb -2 eps, restore +
// update), whose plans differ (the perturbation scales) but whose chunk starts -- and
// so the jump-ahead windows -- are the same: the second and third calls skip the jump.
// The windows live in a library-owned buffer; every call that uses it records an event
// on its stream after its launches, and a call on another stream first makes its stream
// wait for that event (no host synchronisation), so the earlier jump is visible and no
// earlier reader is overtaken by a later overwrite.  Guarded by g_cache_mu; freed by
// fks_plan_cache_clear after a device synchronisation.
struct WinCache {
  int device = -1;
  void* buf = nullptr;
  size_t bytes = 0;
  void* stream = nullptr;  // the stream of the last call that used the buffer
  hipEvent_t done = nullptr;  // recorded on `stream` after that call's launches
  bool valid = false;
  uint64_t seed = 0, chunk_hash = 0;
};

// The reconstruct window cache (fks_jwin_attach): the jumped windows of the slice
// kernel's two-slice passes, per seed, in a CALLER-owned device buffer of window SETS
// (one seed's windows at the pass's chunk-pair starts: nch x 624 words).  A client
// reconstructs the same (seed, sum) list from model_0 every round (fedkseed.py:57-68:
// the arbiter keeps the K seed candidates; :132-141), so the windows of one round are the
// next round's: a seed found in the cache skips its jump.  Keyed by the plan's chunk
// starts (bs_hash) -- another layout or shard resets it --; sets are recycled in
// clock order, never one the current pass still needs.  Stream hand-off by event, as
// WinCache.  Guarded by g_cache_mu.
struct JWin {
  int device = -1;
  void* buf = nullptr;
  size_t bytes = 0;
  void* stream = nullptr;
  hipEvent_t done = nullptr;
  uint64_t key = 0;  // bs_hash of the plan the sets belong to (0: none)
  int nch = 0;       // chunk pairs per set
  uint32_t nsets = 0;
  uint32_t clock = 0;
  uint64_t pass = 0;                       // passes seen (stamps the sets a pass uses)
  std::unordered_map<uint64_t, uint32_t> where;  // seed -> set
  std::vector<uint64_t> set_seed;          // set -> seed (valid when set_used[s])
  std::vector<uint8_t> set_used;
  std::vector<uint64_t> set_pass;          // the last pass that used the set
  uint64_t hits = 0, misses = 0;
};

constexpr size_t kPlanCacheEntries = 32;
std::mutex g_cache_mu;
std::vector<CachedPlan*> g_cache;
uint64_t g_cache_clock = 0;
std::vector<WinCache> g_win;
std::vector<ZCache> g_zc;
std::vector<JWin> g_jw;

uint64_t fnv1a(const std::vector<uint8_t>& b) {
  uint64_t h = 1469598103934665603ull;
  for (uint8_t c : b) h = (h ^ c) * 1099511628211ull;
  return h;
}

template <class T>
void key_put(std::vector<uint8_t>& k, const T& v) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(&v);
  k.insert(k.end(), p, p + sizeof(T));
}

// fp32 launches with wd = +-0 keep kModeUpdateWd (the same bits as kModeUpdateWd0, and
// 2.21 vs 2.28 ms per 19-seed launch: profiles/r02n_ab_f32wd0.log)
constexpr bool kWd0F32Mode = false;
std::vector<uint8_t> plan_key(const fks_tensor* t, int nt, const double* scales, uint64_t delta_base, int shard,
                              int nshards, bool small) {
  std::vector<uint8_t> k;
  k.reserve(64 + (size_t)nt * 40);
  int dev = 0;
  (void)hipGetDevice(&dev);
  key_put(k, dev);
  key_put(k, device_cu_count());
  key_put(k, nt);
  key_put(k, delta_base);
  key_put(k, shard);
  key_put(k, nshards);
  key_put(k, (int)small);
  key_put(k, (int)(scales != nullptr));
  for (int i = 0; i < nt; i++) {
    key_put(k, t[i].data);
    key_put(k, t[i].numel);
    key_put(k, t[i].dtype);
    key_put(k, t[i].flags);
    key_put(k, t[i].lr);
    key_put(k, t[i].wd);
    if (scales) key_put(k, (float)scales[i]);
  }
  return k;
}

CachedPlan* build_plan(const fks_tensor* t, int nt, const double* scales, uint64_t delta_base, int shard,
                       int nshards, bool small) {
  Layout L = make_layout(t, nt, scales, delta_base);
  const BlockRange br = shard_blocks(L.stream_len, shard, nshards);
  clip_segments(L, br);
  auto* C = new CachedPlan();
  C->have_reg = nsegs_total(L) > 0;
  C->have_irr = !L.runs.empty() || !L.tiny.empty();
  Plan P;
  if (C->have_reg) P = make_plan(br, small);
  Plan BP;
  C->have_bs = !small && !L.segs[FKS_BF16].empty();
  if (C->have_bs) {
    BP = make_plan_n(br, bs_nchunks(br.hi - br.lo));
    // the slice kernel indexes a chunk's stream words in 32 bits (< 2^31: 3.4 M blocks
    // per plan chunk pair, a 5.6e11-parameter stream at 512 chunks); longer chunks take the 19-seed kernel
    for (int c = 0; C->have_bs && c < BP.nchunks; c++)
      if ((BP.chunk_block[(size_t)std::min(c + 2, BP.nchunks)] - BP.chunk_block[(size_t)c]) * kMtN >= ((int64_t)1 << 31))
        C->have_bs = false;
    if (!C->have_bs) BP = Plan{};
  }
  const IrrChunks IC = irregular_chunks(L);
  std::vector<uint64_t> ipolys;
  if (C->have_irr) jump_polys_for_blocks(IC.lo, ipolys);
  C->Z.reg_chunks = P.nchunks;
  C->Z.irr_chunks = (int)IC.lo.size();
  C->Z.nsegs = nsegs_total(L);
  C->Z.nruns = (int)L.runs.size();
  C->Z.ntiny = (int)L.tiny.size();
  C->Z.bs_chunks = BP.nchunks;
  C->H = hdr_layout(C->Z);
  std::vector<uint8_t> host(C->H.total, 0);
  auto put = [&](size_t off, const void* src, size_t bytes) {
    if (bytes) std::memcpy(host.data() + off, src, bytes);
  };
  put(C->H.off_polys, P.polys.data(), sizeof(uint64_t) * P.polys.size());
  put(C->H.off_cb, P.chunk_block.data(), sizeof(int64_t) * P.chunk_block.size());
  put(C->H.off_ipolys, ipolys.data(), sizeof(uint64_t) * ipolys.size());
  put(C->H.off_ilo, IC.lo.data(), sizeof(int64_t) * IC.lo.size());
  put(C->H.off_ihi, IC.hi.data(), sizeof(int64_t) * IC.hi.size());
  put(C->H.off_bs_polys, BP.polys.data(), sizeof(uint64_t) * BP.polys.size());
  put(C->H.off_bs_cb, BP.chunk_block.data(), sizeof(int64_t) * BP.chunk_block.size());
  size_t so = C->H.off_segs;
  for (int d = 0; d < 3; d++) {
    C->seg_off[d] = so;
    C->nsegs[d] = (int)L.segs[d].size();
    put(so, L.segs[d].data(), sizeof(DevSeg) * L.segs[d].size());
    so += sizeof(DevSeg) * L.segs[d].size();
    size_t nwd = 0, nwd0 = 0;
    for (const DevSeg& sg : L.segs[d]) {
      nwd += (sg.flags & FKS_HAS_WD) ? 1 : 0;
      nwd0 += ((sg.flags & FKS_HAS_WD) && sg.wd == 0.0f) ? 1 : 0;  // +0.0 or -0.0
    }
    if (!L.segs[d].empty() && nwd0 == L.segs[d].size() && (d != FKS_F32 || kWd0F32Mode))
      C->wd_mode[d] = kModeUpdateWd0;
    else if (!L.segs[d].empty() && nwd == L.segs[d].size()) C->wd_mode[d] = kModeUpdateWd;
    else if (!L.segs[d].empty() && nwd == 0) C->wd_mode[d] = kModeUpdateNoWd;
  }
  put(C->H.off_runs, L.runs.data(), sizeof(DevRun) * L.runs.size());
  put(C->H.off_tiny, L.tiny.data(), sizeof(DevTiny) * L.tiny.size());
  {
    std::vector<uint8_t> ck;
    for (int64_t b : P.chunk_block) key_put(ck, b);
    key_put(ck, (int64_t)-1);
    for (int64_t b : IC.lo) key_put(ck, b);
    C->chunk_hash = fnv1a(ck);
    std::vector<uint8_t> bk;
    for (const DevSeg& sg : L.segs[FKS_BF16]) {
      key_put(bk, sg.start);
      key_put(bk, sg.numel);
    }
    C->bf16_hash = fnv1a(bk);
    std::vector<uint8_t> sk;
    for (int64_t b : BP.chunk_block) key_put(sk, b);
    C->bs_hash = BP.chunk_block.empty() ? 0 : (fnv1a(sk) | 1u);
  }
  if (C->have_reg && !P.chunk_block.empty()) {
    C->reg_lo = P.chunk_block.front();
    C->reg_hi = P.chunk_block.back();
  }
  (void)hipGetDevice(&C->device);
  hipError_t e = hipMalloc(&C->dev, std::max<size_t>(C->H.total, 256));
  if (e != hipSuccess) {
    delete C;
    throw Error(-FKS_ENOMEM, std::string("plan cache hipMalloc: ") + hipGetErrorString(e));
  }
  // synchronous: every later launch on any stream finds the header in place
  e = hipMemcpy(C->dev, host.data(), C->H.total, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(C->dev);
    delete C;
    throw Error(-FKS_EHIP, std::string("plan upload: ") + hipGetErrorString(e));
  }
  return C;
}

// Free a cached header after synchronising the device that owns it (which need not be
// the current one: the key holds the device id, so one process may cache plans of
// several GPUs); the current device is restored.
void free_plan(CachedPlan* C) {
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (C->device != cur) (void)hipSetDevice(C->device);
  (void)hipDeviceSynchronize();
  (void)hipFree(C->dev);
  if (C->device != cur) (void)hipSetDevice(cur);
  delete C;
}

// The cached plan for these inputs (built and uploaded on a miss).  The caller holds
// g_cache_mu for as long as it uses the entry (run() holds it across its launches).
// Entries evicted from the LRU are freed after a device synchronisation, so no
// in-flight launch can still read them.
CachedPlan* get_plan(const fks_tensor* t, int nt, const double* scales, uint64_t delta_base, int shard, int nshards,
                     bool small) {
  std::vector<uint8_t> key = plan_key(t, nt, scales, delta_base, shard, nshards, small);
  const uint64_t h = fnv1a(key);
  for (CachedPlan* C : g_cache) {
    if (C->hash == h && C->key == key) {
      C->last_use = ++g_cache_clock;
      return C;
    }
  }
  CachedPlan* C = build_plan(t, nt, scales, delta_base, shard, nshards, small);
  C->key = std::move(key);
  C->hash = h;
  C->last_use = ++g_cache_clock;
  if (g_cache.size() >= kPlanCacheEntries) {
    auto victim = std::min_element(g_cache.begin(), g_cache.end(),
                                   [](const CachedPlan* a, const CachedPlan* b) { return a->last_use < b->last_use; });
    free_plan(*victim);
    g_cache.erase(victim);
  }
  g_cache.push_back(C);
  return C;
}

struct PhxPlan {
  std::vector<uint8_t> key;
  uint64_t hash = 0, last_use = 0;
  void* dev = nullptr;
  int device = 0;
  int nt = 0;           // table entries (tensors with work items)
  int64_t items = 0;    // work items of all tensors
  int wd_mode = kModeUpdate;  // kModeUpdateWd / NoWd / Wd0 when every tensor shares the form
  bool wd_pos0 = false;        // Wd0 with wd = +0.0 on bf16 / f32 tensors only (kModeUpdateWdPos0 candidate)
  float max_lr = 0.0f;         // max |lr| over the table (the WdPos0 bound)
  std::vector<PhxTensor> tab;  // host copy of the table
  std::vector<int64_t> elem0;  // per entry: its first element in the concatenation of ALL the call's tensors
  std::vector<int> tensor_of;  // per entry: the tensor it belongs to (a tensor past 2^31 bytes has several)
  int64_t elems = 0;           // elements of all the call's tensors
  uint64_t off4_total = 0;     // the Philox offset / 4 one seed's draws advance the generator by
};
std::vector<PhxPlan*> g_phx;

void free_phx(PhxPlan* P) {
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (P->device != cur) (void)hipSetDevice(P->device);
  (void)hipDeviceSynchronize();
  (void)hipFree(P->dev);
  if (P->device != cur) (void)hipSetDevice(cur);
  delete P;
}

void clear_plan_cache() {
  std::lock_guard<std::mutex> lk(g_cache_mu);
  for (CachedPlan* C : g_cache) free_plan(C);
  g_cache.clear();
  for (PhxPlan* P : g_phx) free_phx(P);
  g_phx.clear();
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (WinCache& W : g_win) {
    (void)hipSetDevice(W.device);
    (void)hipDeviceSynchronize();
    if (W.buf) (void)hipFree(W.buf);
    if (W.done) (void)hipEventDestroy(W.done);
  }
  for (ZCache& Z : g_zc) {  // the caller's buffers stay attached; their contents are dropped
    (void)hipSetDevice(Z.device);
    (void)hipDeviceSynchronize();
    Z.valid = false;
    Z.stream = nullptr;
  }
  for (JWin& J : g_jw) {  // likewise
    (void)hipSetDevice(J.device);
    (void)hipDeviceSynchronize();
    J.key = 0;
    J.where.clear();
    J.stream = nullptr;
  }
  (void)hipSetDevice(cur);
  g_win.clear();
}

// The z-index cache entry of the current device (created on first use), or nullptr if
// its event cannot be created.  Caller holds g_cache_mu.
ZCache* z_entry() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  for (ZCache& z : g_zc)
    if (z.device == dev) return z.done ? &z : nullptr;
  g_zc.emplace_back();
  ZCache* Z = &g_zc.back();
  Z->device = dev;
  if (hipEventCreateWithFlags(&Z->done, hipEventDisableTiming) != hipSuccess) {
    Z->done = nullptr;
    (void)hipGetLastError();
    return nullptr;
  }
  return Z;
}

// A boolean switch of the environment: on for 1 / true / yes / on (any case), off when
// unset, empty or anything else -- so FKS_NO_JWIN=0 leaves the cache ON (codec._env_on
// reads the same values).
bool env_on(const char* name) {
  const char* e = std::getenv(name);
  if (!e) return false;
  std::string v(e);
  for (char& ch : v) ch = (char)std::tolower((unsigned char)ch);
  return v == "1" || v == "true" || v == "yes" || v == "on";
}

// The z-index cache of the current device, ordered after its last user on `stream`, if
// the attached buffer holds `bytes`; nullptr otherwise (the call then generates).
ZCache* z_cache(void* stream, size_t bytes) {
  const char* env = std::getenv("FKS_ZCACHE");
  if (env && env[0] == '0') return nullptr;
  ZCache* Z = z_entry();
  if (!Z || !Z->buf || Z->bytes < bytes) return nullptr;
  if (Z->stream && Z->stream != stream) {
    if (hipStreamWaitEvent((hipStream_t)stream, Z->done, 0) != hipSuccess) return nullptr;
  }
  Z->stream = stream;
  return Z;
}

// The reconstruct window cache entry of the current device (created on first use), or
// nullptr if its event cannot be created.  Caller holds g_cache_mu.
JWin* jw_entry() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  for (JWin& j : g_jw)
    if (j.device == dev) return j.done ? &j : nullptr;
  g_jw.emplace_back();
  JWin* J = &g_jw.back();
  J->device = dev;
  if (hipEventCreateWithFlags(&J->done, hipEventDisableTiming) != hipSuccess) {
    J->done = nullptr;
    (void)hipGetLastError();
    return nullptr;
  }
  return J;
}

// The reconstruct window cache for a call of the plan with bs_hash `key` and `nch` chunk
// pairs on `stream`, ordered after its last user, or nullptr (none attached, or too small
// for one two-slice pass).  A new key drops every set.
JWin* jw_cache(void* stream, uint64_t key, int nch) {
  if (env_on("FKS_NO_JWIN")) return nullptr;
  JWin* J = jw_entry();
  if (!J || !J->buf) return nullptr;
  const size_t set_bytes = sizeof(uint32_t) * (size_t)kMtN * (size_t)nch;
  const uint32_t nsets = (uint32_t)std::min<size_t>(J->bytes / set_bytes, UINT32_MAX);
  if (nsets < (uint32_t)kBsPassSeeds) return nullptr;
  if (J->stream && J->stream != stream) {
    if (hipStreamWaitEvent((hipStream_t)stream, J->done, 0) != hipSuccess) return nullptr;
  }
  if (J->key != key || J->nch != nch || J->nsets != nsets) {
    J->key = key;
    J->nch = nch;
    J->nsets = nsets;
    J->clock = 0;
    J->where.clear();
    J->set_seed.assign(nsets, 0);
    J->set_used.assign(nsets, 0);
    J->set_pass.assign(nsets, 0);
  }
  J->stream = stream;
  return J;
}

// Sets for the nb seeds of one two-slice pass: slot[j] = seed j's set; the seeds that
// missed (their windows still to be jumped) are listed in miss / miss_slot.  A missing
// seed takes the next set in clock order that this pass does not use.
void jw_assign(JWin* J, const uint64_t* seeds, int nb, uint32_t* slot, uint64_t* miss, uint32_t* miss_slot,
               int& nmiss) {
  const uint64_t pass = ++J->pass;
  nmiss = 0;
  for (int j = 0; j < nb; j++) {
    auto it = J->where.find(seeds[j]);
    if (it != J->where.end()) {
      slot[j] = it->second;
      J->set_pass[it->second] = pass;
      J->hits++;
      continue;
    }
    uint32_t s = J->clock;
    while (J->set_pass[s] == pass) s = (s + 1) % J->nsets;  // nsets >= 64 > nb: terminates
    J->clock = (s + 1) % J->nsets;
    if (J->set_used[s]) J->where.erase(J->set_seed[s]);
    J->set_seed[s] = seeds[j];
    J->set_used[s] = 1;
    J->set_pass[s] = pass;
    J->where[seeds[j]] = s;
    slot[j] = s;
    miss[nmiss] = seeds[j];
    miss_slot[nmiss] = s;
    nmiss++;
    J->misses++;
  }
}

// The window cache of the current device for a one-seed call on `stream` needing
// `bytes` (ordered after the buffer's last user), or nullptr when it cannot be used
// (FKS_NO_WIN_CACHE set, or no memory: the call then jumps into its workspace).
WinCache* win_cache(void* stream, size_t bytes) {
  if (env_on("FKS_NO_WIN_CACHE")) return nullptr;
  int dev = 0;
  (void)hipGetDevice(&dev);
  WinCache* W = nullptr;
  for (WinCache& w : g_win)
    if (w.device == dev) W = &w;
  if (!W) {
    g_win.emplace_back();
    W = &g_win.back();
    W->device = dev;
    if (hipEventCreateWithFlags(&W->done, hipEventDisableTiming) != hipSuccess) {
      W->done = nullptr;
      (void)hipGetLastError();
    }
  }
  if (!W->done) return nullptr;
  if (W->bytes < bytes) {
    if (W->buf) {
      // the last user may still read the old buffer
      if (hipEventSynchronize(W->done) != hipSuccess) return nullptr;
      (void)hipFree(W->buf);
      W->buf = nullptr;
      W->bytes = 0;
    }
    W->valid = false;
    if (hipMalloc(&W->buf, bytes) != hipSuccess) {
      W->buf = nullptr;
      (void)hipGetLastError();
      return nullptr;
    }
    W->bytes = bytes;
  } else if (W->stream && W->stream != stream) {
    // another stream used the buffer last: wait (on the device) for its launches
    if (hipStreamWaitEvent((hipStream_t)stream, W->done, 0) != hipSuccess) return nullptr;
  }
  W->stream = stream;
  return W;
}

// Chunks per jump workgroup (one chunk per wave, 16 waves, one workgroup per CU by
// LDS): enough workgroups to cover every CU before packing chunks into fewer groups.
int jump_chunks_per_wg(int nseeds, int nchunks) {
  const int per_cu = (int)(((int64_t)nseeds * nchunks + device_cu_count() - 1) / device_cu_count());
  return std::max(1, std::min({kJumpMaxCpw, per_cu, nchunks}));
}

// ------------------------------------------------------------------ torch_rocm stream
// The tensor table of a FKS_STREAM_ROCM call (PhxTensor, fks_internal.h), resident on the
// device once per distinct tensor list (same key as the MT plans, bounded LRU, freed by
// fks_plan_cache_clear).  The geometry is torch's calc_execution_policy
// (ATen/native/cuda/DistributionTemplates.h:50-62) on this device.
// The table and geometry alone, on the host (nothing cached, nothing uploaded): what
// fks_shard_census reads; get_phx_plan adds the device copy.  Needs a current device
// (its CU count and threads per CU set torch's grid).
// torch's TensorIteratorBase::can_use_32bit_indexing for a contiguous 1-D draw of m elements of
// es bytes: numel and the largest byte offset + 1 both within INT32_MAX
inline bool phx_fits32(int64_t m, size_t es) {
  return m <= (int64_t)INT32_MAX && 1 + (m - 1) * (int64_t)es <= (int64_t)INT32_MAX;
}
// calc_execution_policy (DistributionTemplates.h:50-62) for m elements: (stride, loop iterations)
inline void phx_policy(int64_t m, int64_t max_grid, int64_t& stride, int64_t& J) {
  const uint32_t grid0 = (uint32_t)(((uint64_t)m + 255u) / 256u);  // dim3 grid((numel + 255) / 256)
  const int64_t grid = std::min<int64_t>(grid0, max_grid);
  stride = 256 * grid;
  J = (m - 1) / (4 * stride) + 1;  // counter_offset / 4
}

void phx_geometry(const fks_tensor* t, int nt, const double* scales, PhxPlan* P, uint64_t delta_base) {
  const int64_t max_grid = (int64_t)device_cu_count() * (device_max_threads_per_cu() / 256);
  std::vector<PhxTensor> tab;
  std::vector<int64_t> elem0;
  std::vector<int> tensor_of;
  uint64_t off4 = 0;
  int64_t items = 0, elems = 0;
  for (int i = 0; i < nt; i++) {
    const int64_t n = t[i].numel;
    elems += n;
    if (n == 0) continue;  // torch draws nothing for an empty tensor (the offset stays)
    const size_t es = elem_size(t[i].dtype);
    const bool live = !(t[i].flags & FKS_FROZEN);
    const uint64_t base = delta_base ? delta_base + 4 * (uint64_t)(elems - n) : (uint64_t)(uintptr_t)t[i].data;
    const size_t ses = delta_base ? 4 : es;  // bytes per stored element
    // distribution_nullary_kernel (DistributionTemplates.h:111-133) first reserves the
    // offset increment of the whole tensor; when the iterator cannot use 32-bit indexing it
    // then draws each piece TensorIterator::with_32bit_indexing yields -- halves split until
    // they fit, first floor(m / 2) elements then the rest, in order -- as a call of its own,
    // which reserves that piece's increment.  A piece is a table entry of its own (its
    // elements, stride and offset).
    auto emit = [&](int64_t start, int64_t m) {
      int64_t stride = 0, J = 0;
      phx_policy(m, max_grid, stride, J);
      const uint64_t my_off4 = off4;
      off4 += (uint64_t)J;
      if (!live) return;
      PhxTensor x{};
      x.ptr = base + (uint64_t)start * ses;
      x.numel = m;
      x.item0 = items;
      x.off4 = my_off4;
      x.stride = (uint32_t)stride;
      x.dtype = t[i].dtype;
      x.lr = t[i].lr;
      x.wd = t[i].wd;
      const bool fresh16 = ((uint64_t)start * es) % 16u == 0;
      // the alignment of the p the call's first wd * p reads in the reference: this buffer's,
      // or (FKS_FRESH) that of the tensor an earlier reference step rebound param.data to
      const bool wd16 = (t[i].flags & FKS_FRESH) ? fresh16 : (x.ptr % 16u) == 0;
      x.flags = (t[i].flags & FKS_HAS_WD) | ((x.ptr % 16u) == 0 ? kPhxP16 : 0u) | (fresh16 ? kPhxFresh16 : 0u) |
                (wd16 ? kPhxWdP16 : 0u);
      x.ps = scales ? (float)scales[i] : 0.0f;
      tab.push_back(x);
      elem0.push_back(elems - n + start);
      tensor_of.push_back(i);
      items += stride * J;
    };
    auto pieces = [&](auto&& self, int64_t start, int64_t m) -> void {
      if (phx_fits32(m, es)) {
        emit(start, m);
        return;
      }
      const int64_t h = m / 2;
      self(self, start, h);
      self(self, start + h, m - h);
    };
    if (phx_fits32(n, es)) {
      emit(0, n);
    } else {
      int64_t stride = 0, J = 0;
      phx_policy(n, max_grid, stride, J);
      off4 += (uint64_t)J;  // the whole tensor's reservation, before the pieces' own
      pieces(pieces, 0, n);
    }
  }
  P->off4_total = off4;
  P->tensor_of = std::move(tensor_of);
  P->nt = (int)tab.size();
  P->items = items;
  P->elems = elems;
  {  // the launch-wide weight-decay form of a reconstruct (as CachedPlan::wd_mode)
    size_t nwd = 0, nwd0 = 0;
    for (const PhxTensor& x : tab) {
      nwd += (x.flags & FKS_HAS_WD) ? 1 : 0;
      nwd0 += ((x.flags & FKS_HAS_WD) && x.wd == 0.0f) ? 1 : 0;  // +0.0 or -0.0
    }
    if (!tab.empty() && nwd0 == tab.size()) P->wd_mode = kModeUpdateWd0;
    else if (!tab.empty() && nwd == tab.size()) P->wd_mode = kModeUpdateWd;
    else if (!tab.empty() && nwd == 0) P->wd_mode = kModeUpdateNoWd;
    bool pos0 = P->wd_mode == kModeUpdateWd0;
    for (const PhxTensor& x : tab) {
      uint32_t wb;
      std::memcpy(&wb, &x.wd, 4);
      pos0 = pos0 && wb == 0u && x.dtype != FKS_F16 && std::isfinite(x.lr);
      P->max_lr = std::max(P->max_lr, std::fabs(x.lr));
    }
    P->wd_pos0 = pos0;
  }
  P->tab = std::move(tab);
  P->elem0 = std::move(elem0);
}

PhxPlan* get_phx_plan(const fks_tensor* t, int nt, const double* scales, uint64_t delta_base = 0) {
  std::vector<uint8_t> key = plan_key(t, nt, scales, delta_base, 0, 1, false);
  key_put(key, (int)0x7068);  // "ph": not an MT plan key
  key_put(key, device_max_threads_per_cu());
  const uint64_t h = fnv1a(key);
  for (PhxPlan* P : g_phx)
    if (P->hash == h && P->key == key) {
      P->last_use = ++g_cache_clock;
      return P;
    }
  auto* P = new PhxPlan();
  try {
    phx_geometry(t, nt, scales, P, delta_base);
  } catch (...) {
    delete P;
    throw;
  }
  P->key = std::move(key);
  P->hash = h;
  P->last_use = ++g_cache_clock;
  (void)hipGetDevice(&P->device);
  const size_t bytes = std::max<size_t>(sizeof(PhxTensor) * P->tab.size(), 256);
  if (const hipError_t e = hipMalloc(&P->dev, bytes); e != hipSuccess) {
    delete P;
    throw Error(-FKS_ENOMEM, std::string("torch_rocm plan hipMalloc: ") + hipGetErrorString(e) + " (" +
                                 std::to_string(bytes) + " bytes)");
  }
  if (!P->tab.empty() &&
      hipMemcpy(P->dev, P->tab.data(), sizeof(PhxTensor) * P->tab.size(), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(P->dev);
    delete P;
    throw Error(-FKS_EHIP, "torch_rocm plan upload");
  }
  if (g_phx.size() >= kPlanCacheEntries) {
    auto victim = std::min_element(g_phx.begin(), g_phx.end(),
                                   [](const PhxPlan* a, const PhxPlan* b) { return a->last_use < b->last_use; });
    free_phx(*victim);
    g_phx.erase(victim);
  }
  g_phx.push_back(P);
  return P;
}

// Element shards of the torch_rocm stream.  Work item r of a tensor is (idx, j) =
// (r % S, r / S) and covers elements idx + S (4 j + i), i < 4: a ROW of S items (one j)
// covers the 4 S consecutive elements [4 j S, 4 (j + 1) S).  Shard boundaries are the
// equal item splits rounded to the nearest row start, so every shard updates whole rows:
// one contiguous run of elements of the call's tensors laid end to end (fks_shard_census).
int phx_entry(const PhxPlan* P, int64_t b) {  // the last entry whose first item is <= b
  int lo = 0, hi = P->nt - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (P->tab[mid].item0 <= b) lo = mid; else hi = mid - 1;
  }
  return lo;
}
int64_t phx_boundary(const PhxPlan* P, int shard, int nshards) {
  const int64_t b = (int64_t)((__int128)P->items * shard / nshards);
  if (b <= 0 || b >= P->items) return std::max<int64_t>(0, std::min(b, P->items));
  const PhxTensor& T = P->tab[phx_entry(P, b)];
  const int64_t S = T.stride, rows = (T.numel - 1) / (4 * S) + 1;
  const int64_t j = std::min(rows, (b - T.item0 + S / 2) / S);
  return T.item0 + j * S;
}
// the first element (in the concatenation of all the call's tensors) of item boundary b
int64_t phx_boundary_elem(const PhxPlan* P, int64_t b) {
  if (b >= P->items) return P->elems;
  const int k = phx_entry(P, b);
  const PhxTensor& T = P->tab[k];
  return P->elem0[k] + std::min<int64_t>(T.numel, 4 * ((b - T.item0) / T.stride) * (int64_t)T.stride);
}

// the torch_rocm stream: seeds in passes of kPhxSeeds (by value in the kernel arguments);
// element shards split the work items
void run_philox(const fks_tensor* t, int nt, const uint64_t* seeds, const double* values, int k, int value_kind,
                int mode, void* stream, const double* scales, int shard, int nshards, const float* gdev,
                uint64_t delta_base) {
  if (mode != kModeUpdate && mode != kModePerturb && mode != kModePerturbUpdate && mode != kModeWriteZ &&
      mode != kModeDelta)
    throw Error(-FKS_ENOTSUP, "the torch_rocm stream supports the reconstruct, perturb, normal and delta calls only");
  std::lock_guard<std::mutex> lk(g_cache_mu);
  const PhxPlan* P = get_phx_plan(t, nt, scales, mode == kModeDelta ? delta_base : 0);
  if (P->nt == 0 || P->items == 0) return;
  PhiloxArgs a{};
  a.t = static_cast<const PhxTensor*>(P->dev);
  a.nt = P->nt;
  a.gdev = gdev;
  a.mode = mode == kModeUpdate ? P->wd_mode : mode;
  a.item_lo = phx_boundary(P, shard, nshards);
  a.item_hi = phx_boundary(P, shard + 1, nshards);
  if (a.item_lo >= a.item_hi) return;
  if (a.mode == kModeUpdateWd0 && P->wd_pos0 && !env_on("FKS_PHX_KEEP_WD_FMA")) {
    // kModeUpdateWdPos0 when |lr g z| stays <= 1e30 for every seed (|z| <= 6.67: the
    // largest Box-Muller radius is sqrt(-2 ln 2^-32) = 6.66): no overflow, so t = gz
    double gmax = 0.0;
    bool finite = std::isfinite((double)P->max_lr);
    for (int j = 0; j < k && finite; j++)
      for (int d = 0; d < 2; d++) {  // FKS_F32, FKS_BF16: the g the kernels see
        const float g = value_kind == FKS_VALUE_TENSOR ? round_to_dtype(values[j], d) : (float)values[j];
        finite = finite && std::isfinite(g);
        gmax = std::max(gmax, (double)std::fabs(g));
      }
    if (finite && gmax * 6.67 <= 1e37 && gmax * 6.67 * (double)P->max_lr <= 1e30) a.mode = kModeUpdateWdPos0;
  }
  for (int s0 = 0; s0 < k; s0 += kPhxSeeds) {
    const int nb = std::min(kPhxSeeds, k - s0);
    for (int j = 0; j < nb; j++) {
      a.seeds[j] = seeds[s0 + j];
      for (int d = 0; d < 3; d++)
        a.g[3 * j + d] = value_kind == FKS_VALUE_TENSOR ? round_to_dtype(values[s0 + j], d) : (float)values[s0 + j];
    }
    a.nseeds = nb;
    a.call_first = s0 == 0 ? 1 : 0;
    const int rc = timed(0, stream, [&] { return launch_philox(a, stream); });
    if (rc) throw Error(rc < 0 ? rc : -FKS_EHIP, std::string("fks_philox_kernel launch: ") +
                                                     (rc > 0 ? hipGetErrorString((hipError_t)rc) : "unsupported"));
  }
}

void run(const fks_tensor* t, int nt, const uint64_t* seeds, const double* values, int k, int value_kind, int mode,
         void* workspace, size_t ws_bytes, void* stream, const double* tensor_scales = nullptr, int shard = 0,
         int nshards = 1, uint64_t delta_base = 0, const float* gdev = nullptr) {
  validate(t, nt);
  if (nshards < 1 || shard < 0 || shard >= nshards) throw Error(-FKS_EINVAL, "bad shard");
  if (k < 0 || (k > 0 && (!seeds || !values))) throw Error(-FKS_EINVAL, "bad seed/value arrays");
  if (value_kind != FKS_VALUE_SCALAR && value_kind != FKS_VALUE_TENSOR)
    throw Error(-FKS_EINVAL, "bad value_kind");
  if (k == 0 || nt == 0) return;
  if (rocm_stream(t, nt)) {
    run_philox(t, nt, seeds, values, k, value_kind, mode, stream, tensor_scales, shard, nshards, gdev, delta_base);
    return;
  }
  const bool small = k <= kSmallK;
  const bool libm = libm_flavour(t, nt);
  std::lock_guard<std::mutex> lk(g_cache_mu);  // no eviction while this call uses its entry
  const CachedPlan* C = get_plan(t, nt, tensor_scales, delta_base, shard, nshards, small);
  if (!C->have_reg && !C->have_irr) return;
  const int per_pass = small ? kSmallK : kMaxSeedsPerPass;
  // bf16 fast segments of a reconstruct (or delta accumulation) of more than one
  // 19-seed pass go to the bit-sliced slice kernel, 32 seeds per pass
  const bool use_bs = C->have_bs && k >= kBsMinSeeds && (mode == kModeUpdate || mode == kModeDelta);
  size_t need = ws_bytes_for(std::max(C->Z.reg_chunks, C->Z.irr_chunks), std::min(per_pass, k));
  // (a slice pass holds <= 64 seeds x half the plan chunks, a split pass <= 32 x all of them)
  if (use_bs) need = std::max(need, ws_bytes_for(C->Z.bs_chunks, std::min(kBsSeeds, k)));
  if (!workspace || ws_bytes < need)
    throw Error(-FKS_EINVAL, "workspace too small: need " + std::to_string(need) + " bytes, got " +
                                 std::to_string(ws_bytes));
  auto check = [](int rc, const char* what) {
    if (rc) throw Error(rc < 0 ? rc : -FKS_EHIP, std::string(what) + " launch: " +
                                                   (rc > 0 ? hipGetErrorString((hipError_t)rc) : "unsupported"));
  };
  uint8_t* ws = static_cast<uint8_t*>(workspace);
  const uint8_t* hdr = static_cast<const uint8_t*>(C->dev);
  uint32_t* states = reinterpret_cast<uint32_t*>(ws + kWsStatesOff);
  // one-seed bf16 calls: store the table indices (a perturb) or replay them (a later call
  // with the same seed inside the stored block range): ZCache
  ZCache* Zc = nullptr;
  int zmode = 0;
  const bool z_mode_ok = mode == kModePerturb || mode == kModePerturbUpdate || mode == kModeUpdate;
  if (k == 1 && small && !use_bs && C->have_reg && C->nsegs[FKS_BF16] > 0 && z_mode_ok) {
    Zc = z_cache(stream, (size_t)kSm2ZidxBytesPerBlock * (size_t)(C->reg_hi - C->reg_lo));
    if (Zc) {
      if (Zc->valid && Zc->seed == seeds[0] && Zc->bf16_hash == C->bf16_hash && Zc->lo <= C->reg_lo &&
          C->reg_hi <= Zc->hi) {
        zmode = 2;
      } else if (mode == kModePerturb) {
        zmode = 1;
        Zc->valid = false;  // until this call's store is launched
        Zc->lo = C->reg_lo;
        Zc->hi = C->reg_hi;
        Zc->bf16_hash = C->bf16_hash;
      } else {
        Zc = nullptr;
      }
    }
  }
  // one-seed calls: the regular and irregular windows in the per-device window cache,
  // jumped only when the seed or the chunk starts changed since the last call
  uint32_t* reg_states = states;
  uint32_t* irr_states = states;
  bool reg_cached = false, irr_cached = false, reg_jumped = false;
  WinCache* W = nullptr;
  if (k == 1 && !use_bs) {
    const size_t reg_words = (size_t)kMtN * (C->have_reg ? C->Z.reg_chunks : 0);
    const size_t irr_words = (size_t)kMtN * (C->have_irr ? C->Z.irr_chunks : 0);
    W = win_cache(stream, sizeof(uint32_t) * std::max<size_t>(reg_words + irr_words, 1));
    if (W) {
      reg_states = static_cast<uint32_t*>(W->buf);
      irr_states = reg_states + reg_words;
      const bool hit = W->valid && W->seed == seeds[0] && W->chunk_hash == C->chunk_hash;
      reg_cached = irr_cached = hit;
      W->valid = false;  // until this call's jumps are launched
    }
  }
  // a launch error still orders the cache buffers after this call's launches already
  // queued (the entries stay invalid), so a next call on another stream cannot overtake them
  struct EventsOnThrow {
    WinCache*& W;
    ZCache*& Z;
    void* stream;
    bool armed = true;
    ~EventsOnThrow() {
      if (!armed) return;
      if (W) (void)hipEventRecord(W->done, (hipStream_t)stream);
      if (Z) (void)hipEventRecord(Z->done, (hipStream_t)stream);
    }
  } on_throw{W, Zc, stream};
  auto gval = [&](int s, int d) -> float {
    return value_kind == FKS_VALUE_TENSOR ? round_to_dtype(values[s], d) : (float)values[s];
  };
  if (use_bs) {
    // Passes of 64 seeds as two slices per chunk pair (one jump per seed and chunk PAIR),
    // the remainder of <= 32 seeds one slice per plan chunk.  The apply costs the same per
    // seed either way (6.785 ms per 64 seeds against 2 x 3.388 ms over 2^28 parameters,
    // profiles/r03y_*ab.log) and half the jumps go: the 7B bench 10.92 s against 11.03 s
    // for 32-seed passes on one box (profiles/r03g_*.log).  FKS_BS_SLICES=1 forces 32-seed
    // passes (diagnostics, A/B).
    int slices = 2;
    if (const char* e = std::getenv("FKS_BS_SLICES")) slices = (e[0] == '1') ? 1 : 2;
    const int per_pass = slices == 2 ? kBsPassSeeds : kBsSeeds;
    // two-slice passes keep their windows in the reconstruct window cache when one is
    // attached (fks_jwin_attach): a seed already there skips its jump
    JWin* J = (slices == 2 && k > kBsSeeds) ? jw_cache(stream, C->bs_hash, C->Z.bs_chunks / kBsChunksPerWg) : nullptr;
    struct JwOnThrow {  // a failed launch leaves sets assigned but not jumped: drop them all
      JWin* J;
      void* stream;
      bool armed = true;
      ~JwOnThrow() {
        if (!J) return;
        if (armed) {
          J->key = 0;
          J->where.clear();
        }
        (void)hipEventRecord(J->done, (hipStream_t)stream);
      }
    } jw_guard{J, stream};
    for (int s0 = 0; s0 < k; s0 += per_pass) {
      const int nb = std::min(per_pass, k - s0);
      // > 32 seeds: two slices per chunk pair (jumps to every other plan boundary);
      // <= 32: one slice per plan chunk
      const bool split = nb <= kBsSeeds;
      const int nch = split ? C->Z.bs_chunks : C->Z.bs_chunks / kBsChunksPerWg;
      JumpArgs ja{};
      ApplyBsArgs ba{};
      int njump = nb;
      for (int j = 0; j < nb; j++) ja.seeds[j] = seeds[s0 + j];
      ja.polys = reinterpret_cast<const uint64_t*>(hdr + C->H.off_bs_polys);
      ja.chunk_block = reinterpret_cast<const int64_t*>(hdr + C->H.off_bs_cb);
      ja.states = states;
      ba.states = states;
      if (J && !split) {
        jw_assign(J, seeds + s0, nb, ba.slot, ja.seeds, ja.slot, njump);
        ja.states = static_cast<uint32_t*>(J->buf);
        ba.states = ja.states;
        ja.use_slot = ba.use_slot = 1;
      }
      ja.nchunks = nch;
      ja.stride = split ? 1 : kBsChunksPerWg;
      ja.chunks_per_wg = std::max(1, std::min(njump * nch >= 4096 ? 32 : 16, nch));
      if (njump > 0) check(timed(1, stream, [&] { return launch_jump(ja, njump, stream); }), "fks_jump_kernel");
      for (int j = 0; j < nb; j++) ba.g[j] = gval(s0 + j, FKS_BF16);
      ba.segs = reinterpret_cast<const DevSeg*>(hdr + C->seg_off[FKS_BF16]);
      ba.chunk_block = ja.chunk_block;
      ba.sink = reinterpret_cast<uint64_t*>(ws);
      ba.nsegs = C->nsegs[FKS_BF16];
      ba.nchunks = nch;
      ba.split = split ? 1 : 0;
      ba.nseeds = nb;
      ba.mode = mode == kModeUpdate ? C->wd_mode[FKS_BF16] : mode;
      check(timed(0, stream, [&] { return launch_apply_bs(ba, stream); }), "fks_apply_bs_kernel");
    }
    jw_guard.armed = false;
  }
  // the 19-seed kernels: every other regular dtype (all of them without the slice kernel)
  bool reg_rest = false;
  for (int d = 0; d < 3; d++) reg_rest = reg_rest || (C->nsegs[d] && !(use_bs && d == FKS_BF16));
  for (int s0 = 0; s0 < k; s0 += kMaxSeedsPerPass) {
    const int nb = std::min(kMaxSeedsPerPass, k - s0);
    if (reg_rest) {
      JumpArgs ja{};
      for (int j = 0; j < nb; j++) ja.seeds[j] = seeds[s0 + j];
      ja.polys = reinterpret_cast<const uint64_t*>(hdr + C->H.off_polys);
      ja.chunk_block = reinterpret_cast<const int64_t*>(hdr + C->H.off_cb);
      ja.states = reg_states;
      ja.nchunks = C->Z.reg_chunks;
      ja.chunks_per_wg = jump_chunks_per_wg(nb, C->Z.reg_chunks);
      // a replay needs no windows unless another dtype's segments still generate
      const bool need_windows = zmode != 2 || C->nsegs[FKS_F32] > 0 || C->nsegs[FKS_F16] > 0;
      if (!reg_cached && need_windows) {
        check(timed(1, stream, [&] { return launch_jump(ja, nb, stream); }), "fks_jump_kernel");
        reg_jumped = true;
      }
      for (int d = 0; d < 3; d++) {
        if (!C->nsegs[d] || (use_bs && d == FKS_BF16)) continue;
        ApplyArgs aa{};
        aa.states = reg_states;
        for (int j = 0; j < nb; j++) aa.g[j] = gval(s0 + j, d);
        aa.segs = reinterpret_cast<const DevSeg*>(hdr + C->seg_off[d]);
        aa.chunk_block = ja.chunk_block;
        aa.sink = reinterpret_cast<uint64_t*>(ws);
        aa.gdev = gdev;
        if (Zc && d == FKS_BF16) {
          aa.zidx = static_cast<uint32_t*>(Zc->buf);
          aa.zlo = Zc->lo;
          aa.zmode = zmode;
        }
        aa.nsegs = C->nsegs[d];
        aa.nchunks = C->Z.reg_chunks;
        aa.nseeds = nb;
        aa.mode = mode == kModeUpdate ? C->wd_mode[d] : mode;  // weight-decay select specialised away
        const int dd = (d == FKS_F32 && libm) ? kDtF32Libm : d;
        check(timed(0, stream, [&] { return launch_apply(dd, aa, stream); }), "fks_apply_kernel");
      }
    }
    if (C->have_irr) {
      JumpArgs ja{};
      for (int j = 0; j < nb; j++) ja.seeds[j] = seeds[s0 + j];
      ja.polys = reinterpret_cast<const uint64_t*>(hdr + C->H.off_ipolys);
      ja.chunk_block = reinterpret_cast<const int64_t*>(hdr + C->H.off_ilo);
      ja.states = irr_states;
      ja.nchunks = C->Z.irr_chunks;
      ja.chunks_per_wg = std::max(1, std::min(32, C->Z.irr_chunks));
      if (!irr_cached) check(timed(1, stream, [&] { return launch_jump(ja, nb, stream); }), "fks_jump_kernel");
      IrrArgs ia{};
      ia.states = irr_states;
      for (int d = 0; d < 3; d++)
        for (int j = 0; j < nb; j++) ia.g[d][j] = gval(s0 + j, d);
      ia.runs = reinterpret_cast<const DevRun*>(hdr + C->H.off_runs);
      ia.tiny = reinterpret_cast<const DevTiny*>(hdr + C->H.off_tiny);
      ia.chunk_lo = ja.chunk_block;
      ia.chunk_hi = reinterpret_cast<const int64_t*>(hdr + C->H.off_ihi);
      ia.gdev = gdev;
      ia.nruns = C->Z.nruns;
      ia.ntiny = C->Z.ntiny;
      ia.nchunks = C->Z.irr_chunks;
      ia.nseeds = nb;
      ia.mode = mode;
      ia.libm = libm ? 1 : 0;
      check(timed(0, stream, [&] { return launch_irregular(ia, stream); }), "fks_irregular_kernel");
    }
  }
  on_throw.armed = false;
  if (W) {  // this call's windows are in the cache (jumped now or reused), stream-ordered
    // (a replay that skipped the jump did not write the regular windows)
    W->valid = reg_cached || reg_jumped || !C->have_reg;
    W->seed = seeds[0];
    W->chunk_hash = C->chunk_hash;
    if (hipEventRecord(W->done, (hipStream_t)stream) != hipSuccess) throw Error(-FKS_EHIP, "window cache event");
  }
  if (Zc) {  // stored now (zmode 1) or read (zmode 2): stream-ordered like the windows
    if (zmode == 1) {
      Zc->valid = true;
      Zc->seed = seeds[0];
    }
    if (hipEventRecord(Zc->done, (hipStream_t)stream) != hipSuccess) throw Error(-FKS_EHIP, "z-index cache event");
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

size_t workspace_total(const fks_tensor* t, int nt, int k, uint64_t delta_base);

}  // namespace
}  // namespace fks

using namespace fks;

extern "C" {

int fks_workspace_size(const fks_tensor* t, int32_t nt, int32_t k, size_t* bytes) {
  return guarded([&] {
    validate(t, nt);
    if (!bytes || k < 0) throw Error(-FKS_EINVAL, "bad arguments");
    *bytes = workspace_total(t, nt, k, 0);
  });
}

int fks_zindex_size(const fks_tensor* t, int32_t nt, size_t* bytes) {
  return guarded([&] {
    validate(t, nt);
    if (!bytes) throw Error(-FKS_EINVAL, "bad arguments");
    if (rocm_stream(t, nt)) {  // the z-index cache serves the CPU stream only
      *bytes = 0;
      return;
    }
    std::lock_guard<std::mutex> lk(g_cache_mu);
    const CachedPlan* C = get_plan(t, nt, nullptr, 0, 0, 1, true);
    *bytes = (C->have_reg && C->nsegs[FKS_BF16] > 0)
                 ? (size_t)kSm2ZidxBytesPerBlock * (size_t)(C->reg_hi - C->reg_lo)
                 : 0;
  });
}

int fks_zindex_attach(void* buf, size_t bytes) {
  return guarded([&] {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    ZCache* Z = z_entry();
    if (!Z) throw Error(-FKS_EHIP, "z-index cache event");
    // the last call that used the old buffer may still be running: the caller may free
    // or reuse it once this returns
    if (Z->buf && Z->stream && hipEventSynchronize(Z->done) != hipSuccess)
      throw Error(-FKS_EHIP, "z-index cache: waiting for the last user");
    Z->buf = bytes ? buf : nullptr;
    Z->bytes = buf ? bytes : 0;
    Z->valid = false;
    Z->stream = nullptr;
  });
}

int fks_jwin_size_shard(const fks_tensor* t, int32_t nt, int32_t k, int32_t shard, int32_t nshards, size_t* bytes) {
  return guarded([&] {
    validate(t, nt);
    if (!bytes || k < 0) throw Error(-FKS_EINVAL, "bad arguments");
    if (nshards < 1 || shard < 0 || shard >= nshards) throw Error(-FKS_EINVAL, "bad shard");
    *bytes = 0;
    if (rocm_stream(t, nt) || k <= kBsSeeds) return;  // the Philox stream jumps nothing
    std::lock_guard<std::mutex> lk(g_cache_mu);
    // the plan the sharded call itself launches with (run() keys jw_cache on its chunks)
    const CachedPlan* C = get_plan(t, nt, nullptr, 0, shard, nshards, false);
    if (!C->have_bs) return;
    const size_t set_bytes = sizeof(uint32_t) * (size_t)kMtN * (size_t)(C->Z.bs_chunks / kBsChunksPerWg);
    *bytes = set_bytes * (size_t)std::max(k, kBsPassSeeds);
  });
}

int fks_jwin_size(const fks_tensor* t, int32_t nt, int32_t k, size_t* bytes) {
  return fks_jwin_size_shard(t, nt, k, 0, 1, bytes);
}

int fks_jwin_attach(void* buf, size_t bytes) {
  return guarded([&] {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    JWin* J = jw_entry();
    if (!J) throw Error(-FKS_EHIP, "window cache event");
    if (J->buf && J->stream && hipEventSynchronize(J->done) != hipSuccess)
      throw Error(-FKS_EHIP, "window cache: waiting for the last user");
    J->buf = bytes ? buf : nullptr;
    J->bytes = buf ? bytes : 0;
    J->key = 0;
    J->where.clear();
    J->stream = nullptr;
  });
}

int fks_jwin_stats(uint64_t* hits, uint64_t* misses) {
  return guarded([&] {
    if (!hits || !misses) throw Error(-FKS_EINVAL, "bad arguments");
    std::lock_guard<std::mutex> lk(g_cache_mu);
    JWin* J = jw_entry();
    *hits = J ? J->hits : 0;
    *misses = J ? J->misses : 0;
  });
}

int fks_delta_workspace_size(const fks_tensor* t, int32_t nt, int32_t k, size_t* bytes) {
  return guarded([&] {
    validate(t, nt);
    if (!bytes || k < 0) throw Error(-FKS_EINVAL, "bad arguments");
    // any 8-byte aligned delta base gives the same layout; fks_delta_apply's tensor
    // descriptors fit in the same workspace
    *bytes = std::max(workspace_total(t, nt, k, 256), sizeof(DeltaApplyDesc) * (size_t)std::max(nt, 1) + 256);
  });
}

int fks_delta_accumulate(const fks_tensor* t, int32_t nt, const uint64_t* seeds, const double* coefs, int32_t k,
                         float* delta, void* workspace, size_t ws_bytes, void* stream) {
  return guarded([&] {
    if (k > 0 && (!delta || ((uintptr_t)delta % 8) != 0)) throw Error(-FKS_EINVAL, "null or misaligned delta buffer");
    run(t, nt, seeds, coefs, k, FKS_VALUE_SCALAR, kModeDelta, workspace, ws_bytes, stream, nullptr, 0, 1,
        (uint64_t)(uintptr_t)delta);
  });
}

int fks_delta_apply(const fks_tensor* t, int32_t nt, const float* delta, const double* decay, void* workspace,
                    size_t ws_bytes, void* stream) {
  return guarded([&] {
    validate(t, nt);
    if (nt == 0) return;
    if (!delta || !decay || !workspace) throw Error(-FKS_EINVAL, "null argument");
    std::vector<DeltaApplyDesc> d;
    int64_t cum = 0, maxn = 0;
    for (int i = 0; i < nt; i++) {
      if (t[i].numel > 0 && !(t[i].flags & FKS_FROZEN)) {
        DeltaApplyDesc x{};
        x.ptr = (uint64_t)(uintptr_t)t[i].data;
        x.numel = t[i].numel;
        x.delta_off = cum;
        x.dtype = t[i].dtype;
        x.decay = (float)decay[i];
        d.push_back(x);
        maxn = std::max(maxn, t[i].numel);
      }
      cum += t[i].numel;
    }
    if (d.empty()) return;
    const size_t need = sizeof(DeltaApplyDesc) * d.size();
    if (ws_bytes < need) throw Error(-FKS_EINVAL, "workspace too small");
    thread_local std::vector<uint8_t> host;
    host.assign(need, 0);
    std::memcpy(host.data(), d.data(), need);
    hipError_t e = hipMemcpyAsync(workspace, host.data(), need, hipMemcpyHostToDevice, (hipStream_t)stream);
    if (e != hipSuccess) throw Error(-FKS_EHIP, std::string("hipMemcpyAsync: ") + hipGetErrorString(e));
    const int rc = launch_delta_apply(static_cast<const DeltaApplyDesc*>(workspace), (int)d.size(), maxn, delta, stream);
    if (rc) throw Error(-FKS_EHIP, std::string("fks_delta_apply_kernel launch: ") + hipGetErrorString((hipError_t)rc));
  });
}

}  // extern "C"

namespace fks {
namespace {
size_t workspace_total(const fks_tensor* t, int nt, int k, uint64_t delta_base) {
  if (rocm_stream(t, nt)) return kWsStatesOff;  // counter-mode: no generator windows
  // upper bound over every shard count: a shard never needs more chunks than the whole
  // stream; the header itself lives in the plan cache, not in the workspace
  const Layout L = make_layout(t, nt, nullptr, delta_base);
  const bool small = k <= kSmallK;
  int chunks = 0;
  const int64_t nblocks = shard_blocks(L.stream_len, 0, 1).hi;
  if (nsegs_total(L)) chunks = plan_nchunks(nblocks, small);
  if (!L.runs.empty() || !L.tiny.empty()) chunks = std::max(chunks, plan_nchunks(irregular_covered_blocks(L)));
  size_t bytes = ws_bytes_for(chunks, std::max(1, std::min(k, small ? kSmallK : kMaxSeedsPerPass)));
  if (!small && k >= kBsMinSeeds && !L.segs[FKS_BF16].empty())  // the slice kernel's windows
    bytes = std::max(bytes, ws_bytes_for(bs_nchunks(nblocks), std::min(k, kBsSeeds)));
  return bytes;
}
}  // namespace
}  // namespace fks

extern "C" {

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

int fks_cpu_generator_end(const fks_tensor* t, int32_t nt, uint64_t seed, uint32_t* state624, int32_t* left,
                          uint32_t* next, int32_t* normal_valid, double* normal) {
  return guarded([&] {
    validate(t, nt);
    if (!state624 || !left || !next || !normal_valid || !normal) throw Error(-FKS_EINVAL, "null output");
    const Layout L = make_layout(t, nt);
    const int64_t W = L.stream_len;
    // at::mt19937::operator() (MT19937RNGEngine.h): a word first decrements left_ and twists
    // the whole state when it reaches 0 (left_ = 624, next_ = 0), then returns state_[next_++];
    // manual_seed leaves left_ = 1, next_ = 0.  After W >= 1 words the state has been twisted
    // ceil(W / 624) times -- the untempered words x[624 t, 624 t + 624) -- and next_ words of it used.
    const int64_t tw = (W + 623) / 624;
    host_jump_window(seed, tw, state624);
    *next = W ? (uint32_t)(W - 624 * (tw - 1)) : 0u;
    *left = W ? 625 - (int32_t)*next : 1;
    *normal_valid = 0;
    *normal = 0.0;
    if (L.end_cached) {  // normal_distribution<double> (DistributionsHelper.h:189-221): r sin(theta) cached
      uint32_t w[4];
      host_x_words(seed, 624 + L.end_pair, 4, w);  // output word k is temper(x[624 + k])
      for (uint32_t& y : w) {
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
      }
      // random64() = (first word << 32) | second; uniform_real_distribution<double>: 53 bits
      const uint64_t m53 = (1ull << 53) - 1;
      const double u1 = (double)((((uint64_t)w[0] << 32) | w[1]) & m53) * (1.0 / 9007199254740992.0);
      const double u2 = (double)((((uint64_t)w[2] << 32) | w[3]) & m53) * (1.0 / 9007199254740992.0);
      const double r = std::sqrt(-2.0 * std::log1p(-u2));
      const double theta = 2.0 * 3.14159265358979323846 * u1;
      *normal = r * std::sin(theta);
      *normal_valid = 1;
    }
  });
}

int fks_rocm_grid_cap(int64_t* blocks) {
  return guarded([&] {
    int dev = 0;
    if (!blocks) throw Error(-FKS_EINVAL, "null output");
    if (hipGetDevice(&dev) != hipSuccess) throw Error(-FKS_EHIP, "no current HIP device");
    *blocks = (int64_t)device_cu_count() * (device_max_threads_per_cu() / 256);
  });
}

int fks_rocm_offset(const fks_tensor* t, int32_t nt, uint64_t* offset) {
  return guarded([&] {
    validate(t, nt);
    if (!offset) throw Error(-FKS_EINVAL, "null output");
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) throw Error(-FKS_EHIP, "no current HIP device");
    PhxPlan geo;
    phx_geometry(t, nt, nullptr, &geo, 0);
    *offset = 4 * geo.off4_total;
  });
}

int fks_shard_census(const fks_tensor* t, int32_t nt, int32_t shard, int32_t nshards, int64_t* word_range,
                     int64_t* written) {
  return guarded([&] {
    validate(t, nt);
    if (nshards < 1 || shard < 0 || shard >= nshards) throw Error(-FKS_EINVAL, "bad shard");
    if (rocm_stream(t, nt)) {  // element runs of whole Philox rows (phx_boundary)
      // host geometry only: no plan cache entry, no device allocation (the scales do not
      // move row boundaries)
      PhxPlan geo;
      phx_geometry(t, nt, nullptr, &geo, 0);
      const PhxPlan* P = &geo;
      const int64_t lo = phx_boundary(P, shard, nshards), hi = phx_boundary(P, shard + 1, nshards);
      if (word_range) {
        word_range[0] = phx_boundary_elem(P, lo);
        word_range[1] = phx_boundary_elem(P, hi);
      }
      if (!written) return;
      for (int i = 0; i < nt; i++) written[i] = 0;
      for (int k = 0; k < P->nt; k++) {  // table entries: the pieces of the non-empty, non-frozen tensors
        const PhxTensor& T = P->tab[k];
        const int64_t a0 = std::max(lo, T.item0), a1 = std::min(hi, T.item0 + T.stride * ((T.numel - 1) / (4 * (int64_t)T.stride) + 1));
        if (a1 > a0)
          written[P->tensor_of[k]] += std::min<int64_t>(T.numel, 4 * ((a1 - T.item0) / T.stride) * (int64_t)T.stride) -
                                      std::min<int64_t>(T.numel, 4 * ((a0 - T.item0) / T.stride) * (int64_t)T.stride);
      }
      return;
    }
    Layout L = make_layout(t, nt);
    const BlockRange br = shard_blocks(L.stream_len, shard, nshards);
    clip_segments(L, br);
    if (word_range) {
      word_range[0] = br.lo * kMtN;
      word_range[1] = br.hi * kMtN;
    }
    if (!written) return;
    for (int i = 0; i < nt; i++) written[i] = 0;
    for (int d = 0; d < 3; d++)
      for (size_t j = 0; j < L.segs[d].size(); j++) written[L.seg_tensor[d][j]] += L.segs[d][j].numel;
    for (size_t j = 0; j < L.runs.size(); j++)
      written[L.run_tensor[j]] += std::max<int64_t>(0, std::min(L.runs[j].limit, L.runs[j].numel));
    for (size_t j = 0; j < L.tiny.size(); j++) written[L.tiny_tensor[j]] += 1;
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
        (void)hipEventSynchronize(e.second);
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, e.first, e.second);
        tot[w] += ms;
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
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

int fks_perturb_step(const fks_tensor* t, int32_t nt, uint64_t seed, const double* scales, double value,
                     int32_t value_kind, int32_t update, void* workspace, size_t ws_bytes, void* stream) {
  return guarded([&] {
    if (nt > 0 && !scales) throw Error(-FKS_EINVAL, "null scales");
    run(t, nt, &seed, &value, 1, value_kind, update ? kModePerturbUpdate : kModePerturb, workspace, ws_bytes, stream,
        scales);
  });
}

int fks_perturb_step_dev(const fks_tensor* t, int32_t nt, uint64_t seed, const double* scales, const float* dev_value,
                         void* workspace, size_t ws_bytes, void* stream) {
  return guarded([&] {
    if (nt > 0 && (!scales || !dev_value)) throw Error(-FKS_EINVAL, "null scales or device value");
    const double unused = 0.0;
    run(t, nt, &seed, &unused, 1, FKS_VALUE_TENSOR, kModePerturbUpdate, workspace, ws_bytes, stream, scales, 0, 1, 0,
        dev_value);
  });
}

int fks_normal(const fks_tensor* t, int32_t nt, uint64_t seed, void* workspace, size_t ws_bytes, void* stream) {
  return guarded([&] {
    const double v = 0.0;
    run(t, nt, &seed, &v, 1, FKS_VALUE_SCALAR, kModeWriteZ, workspace, ws_bytes, stream);
  });
}

int fks_plan_cache_clear(void) {
  return guarded([&] { clear_plan_cache(); });
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

int fks_device_selfcheck(int32_t which, uint64_t* result, void* workspace, size_t ws_bytes, void* stream) {
  return guarded([&] {
    if (!result || (which != FKS_CHECK_SQRT_DOMAIN && which != FKS_CHECK_PHILOX_RADIUS &&
                    which != FKS_CHECK_PHILOX_BF16_RADIUS))
      throw Error(-FKS_EINVAL, "bad arguments");
    const size_t need = sizeof(uint32_t) * (size_t)kSqrtDomainBlocks;
    if (!workspace || ws_bytes < need) throw Error(-FKS_EINVAL, "workspace too small");
    uint32_t* counts = static_cast<uint32_t*>(workspace);
    int rc = which == FKS_CHECK_SQRT_DOMAIN     ? launch_sqrt_domain_check(counts, stream)
             : which == FKS_CHECK_PHILOX_RADIUS ? launch_philox_radius_check(counts, stream)
                                                : launch_philox_fast_radius_check(counts, stream);
    if (rc) throw Error(-FKS_EHIP, std::string("self check launch: ") + hipGetErrorString((hipError_t)rc));
    std::vector<uint32_t> h((size_t)kSqrtDomainBlocks);
    if (hipMemcpyAsync(h.data(), counts, need, hipMemcpyDeviceToHost, (hipStream_t)stream) != hipSuccess ||
        hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
      throw Error(-FKS_EHIP, "sqrt domain check copy");
    uint64_t bad = 0;
    for (uint32_t v : h) bad = which == FKS_CHECK_PHILOX_BF16_RADIUS ? std::max<uint64_t>(bad, v) : bad + v;
    *result = bad;
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
