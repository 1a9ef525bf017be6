// fks_gf2.cpp -- MT19937 jump-ahead in GF(2)[t] / phi(t) (host side of libfks.so).
//
// The reference's per-seed stream is torch's CPU mt19937 (MT19937RNGEngine.h:115-175),
// a sequential generator.  To let thousands of workgroups start mid-stream, every
// chunk start J gets the polynomial c_J(t) = t^J mod phi(t), phi = the MT19937
// characteristic polynomial (degree 19937).  For the word sequence y[n] = x[n+1]
// (x = the untempered MT word sequence, x[0..623] = the seeded state) every bit
// lane obeys phi's recurrence, so
//      y[J + w] = XOR_{i : c_J[i] = 1} y[i + w]        (w = 0..623)
// which the device kernel fks_jump_kernel evaluates per (seed, chunk).
//
// phi is recovered once with Berlekamp-Massey; products mod phi use carry-less
// multiplication (PCLMULQDQ) and an exact Barrett reduction.
#include "fks_internal.h"

#include <immintrin.h>
#include <wmmintrin.h>

#include <cstring>
#include <mutex>
#include <unordered_map>

namespace fks {

namespace {

constexpr int kDeg = 19937;
constexpr int kWords = (kDeg + 63) / 64;  // 312 words hold a residue (degree < 19937)

using Poly = std::vector<uint64_t>;

inline int getbit(const uint64_t* p, int64_t i) { return (int)((p[i >> 6] >> (i & 63)) & 1u); }
inline void flipbit(uint64_t* p, int64_t i) { p[i >> 6] ^= (1ull << (i & 63)); }

// out[0..na+nb) = a * b (carry-less)
void clmul(const uint64_t* a, int na, const uint64_t* b, int nb, uint64_t* out) {
  std::memset(out, 0, sizeof(uint64_t) * (size_t)(na + nb));
  for (int i = 0; i < na; i++) {
    if (!a[i]) continue;
    const __m128i ai = _mm_cvtsi64_si128((long long)a[i]);
    for (int j = 0; j < nb; j++) {
      if (!b[j]) continue;
      const __m128i r = _mm_clmulepi64_si128(ai, _mm_cvtsi64_si128((long long)b[j]), 0x00);
      out[i + j] ^= (uint64_t)_mm_cvtsi128_si64(r);
      out[i + j + 1] ^= (uint64_t)_mm_extract_epi64(r, 1);
    }
  }
}

// dst ^= src << m  (both n words; bits shifted past the end are dropped)
void xor_shl(uint64_t* dst, const uint64_t* src, int n, int64_t m) {
  const int64_t ws = m >> 6;
  const int bs = (int)(m & 63);
  for (int64_t i = n - 1; i >= ws; i--) {
    const int64_t k = i - ws;
    uint64_t v = src[k] << bs;
    if (bs && k > 0) v |= src[k - 1] >> (64 - bs);
    dst[i] ^= v;
  }
}

// floor(p / t^s) for a poly with n words; result written to out (n words, zero padded)
void shr_bits(const uint64_t* p, int n, int64_t s, uint64_t* out, int nout) {
  const int64_t ws = s >> 6;
  const int bs = (int)(s & 63);
  for (int i = 0; i < nout; i++) {
    const int64_t k = i + ws;
    uint64_t lo = k < n ? p[k] : 0, hi = (k + 1) < n ? p[k + 1] : 0;
    out[i] = bs ? ((lo >> bs) | (hi << (64 - bs))) : lo;
  }
}

struct Field {
  Poly phi;  // kWords + 1 words, bit kDeg set
  Poly mu;   // floor(t^(2*kDeg) / phi), degree kDeg
};

// Berlekamp-Massey over GF(2) on bit 0 of the y-sequence of a seeded generator.
Poly berlekamp_massey_phi() {
  // untempered words x[0..], x[0..623] = seeded state (seed 5489)
  const int64_t need = 2 * (int64_t)kDeg + 2;
  std::vector<uint32_t> x((size_t)(need + 624 + 1248));
  x[0] = 5489u;
  for (int j = 1; j < 624; j++) x[j] = 1812433253u * (x[j - 1] ^ (x[j - 1] >> 30)) + (uint32_t)j;
  for (size_t n = 624; n < x.size(); n++) {
    const uint32_t u = x[n - 624], v = x[n - 623];
    x[n] = x[n - 227] ^ ((((u & 0x80000000u) | (v & 0x7fffffffu)) >> 1) ^ ((v & 1u) ? 0x9908b0dfu : 0u));
  }
  const int64_t L2 = 2 * (int64_t)kDeg;
  // s[i] = bit0 of y[i] = x[i+1]; stored reversed so a window dot product is a word scan
  const int SW = (int)((L2 + 64 + 63) / 64);
  std::vector<uint64_t> srev((size_t)SW + 2, 0);  // srev bit (L2-1-i) = s[i]
  for (int64_t i = 0; i < L2; i++)
    if (x[(size_t)i + 1] & 1u) flipbit(srev.data(), L2 - 1 - i);
  const int CW = kWords + 2;
  std::vector<uint64_t> C((size_t)CW, 0), B((size_t)CW, 0), T((size_t)CW, 0), win((size_t)CW, 0);
  C[0] = B[0] = 1;
  int64_t L = 0, m = 1;
  for (int64_t i = 0; i < L2; i++) {
    // d = sum_{j=0..L} C_j s[i-j];  s[i-j] = srev bit (L2-1-i+j)
    shr_bits(srev.data(), SW, L2 - 1 - i, win.data(), (int)((L + 64) / 64) + 1);
    uint64_t acc = 0;
    const int nw = (int)(L / 64) + 1;
    for (int w = 0; w < nw; w++) acc ^= C[w] & win[w];
    // bits of C beyond L are zero, bits of win beyond i are zero (s[negative] absent): mask
    int d = __builtin_parityll(acc);
    if (!d) {
      m++;
      continue;
    }
    if (2 * L <= i) {
      T = C;
      xor_shl(C.data(), B.data(), CW, m);
      L = i + 1 - L;
      B = T;
      m = 1;
    } else {
      xor_shl(C.data(), B.data(), CW, m);
      m++;
    }
  }
  if (L != kDeg) throw Error(-EPROTO, "Berlekamp-Massey: MT19937 linear complexity " + std::to_string(L));
  // phi_i = C_{L-i}
  Poly phi((size_t)kWords + 1, 0);
  for (int64_t i = 0; i <= L; i++)
    if (getbit(C.data(), L - i)) flipbit(phi.data(), i);
  return phi;
}

Field make_field() {
  Field f;
  f.phi = berlekamp_massey_phi();
  // mu = floor(t^(2n) / phi) by long division (bit serial, once)
  const int64_t n = kDeg;
  const int RW = (int)((2 * n + 64) / 64) + 1;
  std::vector<uint64_t> rem((size_t)RW, 0);
  flipbit(rem.data(), 2 * n);
  Poly q((size_t)kWords + 2, 0);
  for (int64_t b = 2 * n; b >= n; b--) {
    if (!getbit(rem.data(), b)) continue;
    flipbit(q.data(), b - n);
    // rem ^= phi << (b - n)
    std::vector<uint64_t> ph((size_t)RW, 0);
    std::memcpy(ph.data(), f.phi.data(), sizeof(uint64_t) * f.phi.size());
    xor_shl(rem.data(), ph.data(), RW, b - n);
  }
  f.mu = q;
  return f;
}

const Field& field() {
  static std::once_flag once;
  static Field* f = nullptr;
  std::call_once(once, [] { f = new Field(make_field()); });
  return *f;
}

// r (kWords words, degree < n) = a mod phi for deg(a) < 2n  (exact Barrett over GF(2))
void barrett(const uint64_t* a, int na, uint64_t* r) {
  const Field& F = field();
  const int64_t n = kDeg;
  const int QW = kWords + 1;
  std::vector<uint64_t> q1((size_t)QW), q2((size_t)(QW + F.mu.size())), q((size_t)QW),
      qp((size_t)(QW + F.phi.size()));
  shr_bits(a, na, n, q1.data(), QW);
  clmul(q1.data(), QW, F.mu.data(), (int)F.mu.size(), q2.data());
  shr_bits(q2.data(), (int)q2.size(), n, q.data(), QW);
  clmul(q.data(), QW, F.phi.data(), (int)F.phi.size(), qp.data());
  for (int i = 0; i < kWords; i++) r[i] = (i < na ? a[i] : 0) ^ qp[(size_t)i];
  r[kWords - 1] &= (1ull << (n - 64 * (kWords - 1))) - 1;  // keep bits < n
}

void mulmod(const uint64_t* a, const uint64_t* b, uint64_t* r) {
  std::vector<uint64_t> prod(2 * (size_t)kWords);
  clmul(a, kWords, b, kWords, prod.data());
  barrett(prod.data(), 2 * kWords, r);
}

// t^e mod phi, left-to-right binary powering (squaring = bit spreading)
Poly powmod_t(uint64_t e) {
  Poly r((size_t)kWords, 0);
  r[0] = 1;
  if (e == 0) return r;
  int top = 63 - __builtin_clzll(e);
  std::vector<uint64_t> sq(2 * (size_t)kWords);
  for (int bit = top; bit >= 0; bit--) {
    // square: spread bits
    for (int i = 0; i < kWords; i++) {
      const __m128i v = _mm_cvtsi64_si128((long long)r[i]);
      const __m128i s = _mm_clmulepi64_si128(v, v, 0x00);
      sq[2 * (size_t)i] = (uint64_t)_mm_cvtsi128_si64(s);
      sq[2 * (size_t)i + 1] = (uint64_t)_mm_extract_epi64(s, 1);
    }
    barrett(sq.data(), 2 * kWords, r.data());
    if ((e >> bit) & 1u) {
      // r *= t
      uint64_t carry = 0;
      for (int i = 0; i < kWords; i++) {
        const uint64_t nc = r[i] >> 63;
        r[i] = (r[i] << 1) | carry;
        carry = nc;
      }
      const int64_t hb = kDeg;  // bit kDeg may now be set (in word kWords-1 since 19937 < 312*64)
      if (getbit(r.data(), hb)) {
        for (int i = 0; i < kWords; i++) r[i] ^= field().phi[(size_t)i];
      }
    }
  }
  return r;
}

std::mutex g_cache_mu;
std::unordered_map<uint64_t, Poly>* g_cache = nullptr;

}  // namespace

int jump_poly_words() { return kWords; }

// c = t^J mod phi for J = 624*block - 1 (block >= 1); cached per block.
void jump_polys_for_blocks(const std::vector<int64_t>& blocks, std::vector<uint64_t>& out) {
  out.assign(blocks.size() * (size_t)kWords, 0);
  std::lock_guard<std::mutex> lk(g_cache_mu);
  if (!g_cache) g_cache = new std::unordered_map<uint64_t, Poly>();
  // incremental: consecutive requested blocks reuse the previous residue times t^(624*delta)
  std::unordered_map<int64_t, Poly> step_cache;
  const Poly* prev = nullptr;
  int64_t prev_block = -1;
  for (size_t c = 0; c < blocks.size(); c++) {
    const int64_t b = blocks[c];
    if (b <= 0) {  // block 0: the seeded state itself; unused
      prev = nullptr;
      continue;
    }
    auto it = g_cache->find((uint64_t)b);
    if (it == g_cache->end()) {
      Poly r;
      if (prev && b > prev_block) {
        const int64_t d = b - prev_block;
        auto st = step_cache.find(d);
        if (st == step_cache.end()) st = step_cache.emplace(d, powmod_t((uint64_t)(624 * d))).first;
        r.assign((size_t)kWords, 0);
        mulmod(prev->data(), st->second.data(), r.data());
      } else {
        r = powmod_t((uint64_t)(624 * b - 1));
      }
      it = g_cache->emplace((uint64_t)b, std::move(r)).first;
    }
    std::memcpy(out.data() + c * (size_t)kWords, it->second.data(), sizeof(uint64_t) * (size_t)kWords);
    prev = &it->second;
    prev_block = b;
  }
}

// CPU evaluation of the jump: window of x at 624*block for `seed` (the generator state
// after `block` twists).  The self checks compare it with the oracle; fks_cpu_generator_end
// uses it to leave torch's CPU generator where the reference leaves it.  One pass over the
// set coefficients of c (about 10^4), each xoring 624 consecutive words into the window.
void host_jump_window(uint64_t seed, int64_t block, uint32_t* out624) {
  std::vector<uint32_t> x(624 + kDeg + 16);
  x[0] = (uint32_t)(seed & 0xffffffffu);
  for (int j = 1; j < 624; j++) x[j] = 1812433253u * (x[j - 1] ^ (x[j - 1] >> 30)) + (uint32_t)j;
  for (size_t n = 624; n < x.size(); n++) {
    const uint32_t u = x[n - 624], v = x[n - 623];
    x[n] = x[n - 227] ^ ((((u & 0x80000000u) | (v & 0x7fffffffu)) >> 1) ^ ((v & 1u) ? 0x9908b0dfu : 0u));
  }
  if (block == 0) {
    std::memcpy(out624, x.data(), 624 * 4);
    return;
  }
  std::vector<uint64_t> c;
  jump_polys_for_blocks({block}, c);
  uint32_t acc[624] = {};
  for (int wi = 0; wi < kWords; wi++) {
    for (uint64_t bits = c[(size_t)wi]; bits; bits &= bits - 1) {
      const int i = 64 * wi + __builtin_ctzll(bits);
      if (i >= kDeg) break;
      const uint32_t* src = x.data() + i + 1;  // y[i + w] = x[i + w + 1]
      for (int w = 0; w < 624; w++) acc[w] ^= src[w];
    }
  }
  std::memcpy(out624, acc, sizeof(acc));
}

// x[first .. first + n) of `seed` (untempered words; x[0..623] = the seeded state): the
// jumped window of the block holding `first`, extended by the recurrence.
void host_x_words(uint64_t seed, int64_t first, int n, uint32_t* out) {
  const int64_t block = first / 624;
  std::vector<uint32_t> x((size_t)(624 + (first - 624 * block) + n + 624));
  host_jump_window(seed, block, x.data());
  for (size_t k = 624; k < x.size(); k++) {
    const uint32_t u = x[k - 624], v = x[k - 623];
    x[k] = x[k - 227] ^ ((((u & 0x80000000u) | (v & 0x7fffffffu)) >> 1) ^ ((v & 1u) ? 0x9908b0dfu : 0u));
  }
  std::memcpy(out, x.data() + (first - 624 * block), sizeof(uint32_t) * (size_t)n);
}

const std::vector<uint64_t>& charpoly() { return field().phi; }

}  // namespace fks
