// Host self-test of the bit-sliced MT19937 primitives (fate-llm_amd/csrc/fks_bitslice.h)
// against the scalar generator: the in-place round schedule of the twist wave (10
// rounds of 64 rows, reads of a round before its writes, U31 from the neighbour lane),
// the low-byte tempering map, both transposes and the byte extraction.
//   g++ -O2 -std=c++17 -I fate-llm_amd/csrc tools/bs/bs_selftest.cpp -o /tmp/bs_selftest && /tmp/bs_selftest
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "fks_bitslice.h"

using namespace fks::bs;

static uint32_t temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}
static void twist(uint32_t* s) {
  for (int i = 0; i < 624; i++) {
    const uint32_t y = (s[i] & 0x80000000u) | (s[(i + 1) % 624] & 0x7fffffffu);
    s[i] = s[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }
}

int main() {
  std::mt19937 rng(1234);
  static uint32_t st[32][624];
  for (auto& r : st)
    for (auto& w : r) w = rng();
  // planes of the state: rows[i][b]
  static uint32_t rows[624][32];
  for (int i = 0; i < 624; i++) {
    uint32_t w[32];
    for (int k = 0; k < 32; k++) w[k] = st[k][i];
    transpose32(w);
    for (int b = 0; b < 32; b++) {
      uint32_t ref = 0;
      for (int k = 0; k < 32; k++) ref |= ((st[k][i] >> b) & 1u) << k;
      if (w[b] != ref) { printf("transpose32 mismatch row %d plane %d\n", i, b); return 1; }
      rows[i][b] = w[b];
    }
  }
  int bad = 0;
  for (int blk = 0; blk < 3; blk++) {
    // scalar
    for (int k = 0; k < 32; k++) twist(st[k]);
    // the twist wave: 10 rounds of 64 lanes, in place
    uint32_t prev63 = rows[0][31];  // old row 0, plane 31 (read before round 0)
    for (int r = 0; r < 10; r++) {
      static uint32_t V[64][32], M[64][32], U[64];
      for (int l = 0; l < 64; l++) {
        const int i = 64 * r + l;
        const int iv = i + 1 == 624 ? 0 : (i < 624 ? i + 1 : 0);
        const int im = i < 227 ? i + 397 : (i < 624 ? i - 227 : 0);
        memcpy(V[l], rows[iv], sizeof V[l]);
        memcpy(M[l], rows[im], sizeof M[l]);
      }
      for (int l = 0; l < 64; l++) U[l] = l == 0 ? prev63 : V[l - 1][31];  // wave_shr:1
      prev63 = V[63][31];
      for (int l = 0; l < 64; l++) {
        const int i = 64 * r + l;
        if (i >= 624) continue;
        twist_row(V[l], M[l], U[l], rows[i]);
      }
    }
    for (int i = 0; i < 624; i++) {
      uint32_t o[8];
      temper_low8(rows[i], o);
      uint32_t T[8];
      memcpy(T, o, sizeof T);
      transpose8(T);
      for (int k = 0; k < 32; k++) {
        uint32_t ref = 0;
        for (int b = 0; b < 32; b++) ref |= ((rows[i][b] >> k) & 1u) << b;
        if (ref != st[k][i]) { if (bad++ < 5) printf("twist mismatch blk %d row %d seed %d\n", blk, i, k); }
        const uint32_t want = temper(st[k][i]) & 0xFFu;
        const int c = k >> 3, j = k & 7;
        const uint32_t got = (T[j] >> (8 * c)) & 0xFFu;
        if (got != want) { if (bad++ < 5) printf("temper/transpose mismatch blk %d row %d seed %d: %02x vs %02x\n", blk, i, k, got, want); }
        uint32_t x4 = 0;
        switch (c) {
          case 0: x4 = byte_x<0, 2>(T[j]); break;
          case 1: x4 = byte_x<1, 2>(T[j]); break;
          case 2: x4 = byte_x<2, 2>(T[j]); break;
          default: x4 = byte_x<3, 2>(T[j]); break;
        }
        if (x4 != want * 4) { if (bad++ < 5) printf("byte_x mismatch\n"); }
      }
    }
  }
  printf(bad ? "bs_selftest FAILED (%d)\n" : "bs_selftest ok: transpose32, 3 blocks of in-place round twist, temper_low8, transpose8, byte_x (%d)\n", bad);
  return bad != 0;
}
