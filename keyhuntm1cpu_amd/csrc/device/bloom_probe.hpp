// Level-1 bloom probe of a giant-step x-coordinate, bit-exact with bloom/bloom.cpp:128-156 and
// xxhash/xxhash.h:2304-2527 (XXH64 v0.8.0) for the fixed 32-byte input keyhunt hashes
// (Int::Get32Bytes of x, keyhunt.cpp:3945-3946).
//
// The probe is split so the GPU pays only for what a miss needs: bit 0 of a probe is
// (a mod bits) and depends on the first hash alone, so the second XXH64 (bloom_rest) runs only
// for the ~50 % of points whose first bit is set — the scan kernel queues those survivors and
// finishes them in full waves; later bit positions (a + b*i) mod bits are stepped incrementally
// (64-bit wrap tracked by the carry, corrected by 2^64 mod bits).
#pragma once
#include <stdint.h>
#include "fe.hpp"

namespace khb {

#define KHB_XP1 0x9E3779B185EBCA87ull
#define KHB_XP2 0xC2B2AE3D27D4EB4Full
#define KHB_XP3 0x165667B19E3779F9ull
#define KHB_XP4 0x85EBCA77C2B2AE63ull
#define KHB_BLOOM_SEED 0x59f2815b16f81798ull   // bloom.cpp:68, 135

KHB_HD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
KHB_HD uint64_t xxh_round(uint64_t acc, uint64_t in) {
  acc += in * KHB_XP2;
  acc = rotl64(acc, 31);
  return acc * KHB_XP1;
}
KHB_HD uint64_t xxh_merge(uint64_t acc, uint64_t v) {
  v = xxh_round(0, v);
  acc ^= v;
  return acc * KHB_XP1 + KHB_XP4;
}

// XXH64 of a 32-byte buffer given as four little-endian 64-bit words.
KHB_HD uint64_t xxh64_32(const uint64_t w[4], uint64_t seed) {
  uint64_t v1 = seed + KHB_XP1 + KHB_XP2, v2 = seed + KHB_XP2, v3 = seed, v4 = seed - KHB_XP1;
  v1 = xxh_round(v1, w[0]);
  v2 = xxh_round(v2, w[1]);
  v3 = xxh_round(v3, w[2]);
  v4 = xxh_round(v4, w[3]);
  uint64_t h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
  h = xxh_merge(h, v1);
  h = xxh_merge(h, v2);
  h = xxh_merge(h, v3);
  h = xxh_merge(h, v4);
  h += 32;
  h ^= h >> 33;
  h *= KHB_XP2;
  h ^= h >> 29;
  h *= KHB_XP3;
  h ^= h >> 32;
  return h;
}

KHB_HD uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}

// The hash input words of Get32Bytes(x): word k = little-endian load of BE bytes 8k..8k+7.
KHB_HD void x_words(uint64_t w[4], const Fe& x) {
#pragma unroll
  for (int k = 0; k < 4; ++k)
    w[k] = ((uint64_t)bswap32(x.v[6 - 2 * k]) << 32) | bswap32(x.v[7 - 2 * k]);
}

// Per-level bloom geometry, precomputed on the host (all 256 sub-blooms share it: the reference
// initialises every sub-bloom with the same entry count, keyhunt.cpp:1232-1244).
struct BloomGeom {
  uint64_t bytes_per_sub;
  uint64_t bits;        // bloom->bits
  uint64_t magic;       // floor(2^64 / bits): Barrett reciprocal for "% bits"
  uint64_t wrap;        // 2^64 mod bits
  uint32_t hashes;      // bloom->hashes
};

// h mod d for 64-bit h, d = g.bits (Barrett with one correction step; exact).
KHB_HD uint64_t mod_bits(uint64_t h, const BloomGeom& g) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t q = __umul64hi(h, g.magic);
#else
  uint64_t q = (uint64_t)(((unsigned __int128)h * g.magic) >> 64);
#endif
  uint64_t r = h - q * g.bits;
  return r >= g.bits ? r - g.bits : r;
}

KHB_HD bool test_bit(const uint8_t* bf, uint64_t bit) { return (bf[bit >> 3] >> (bit & 7)) & 1u; }

// The sub-bloom bloom_bP[xb[0]] of x (keyhunt.cpp:3946-3947); bf_all = 256 concatenated sub-blooms.
KHB_HD const uint8_t* sub_bloom(const uint8_t* __restrict__ bf_all, const BloomGeom& g, const Fe& x) {
  return bf_all + (uint64_t)(x.v[7] >> 24) * g.bytes_per_sub;
}

// Hashes 1..hashes-1 of bloom_check (bloom.cpp:141-150) for an x whose first hash `a` already hit:
// b = XXH64(x, seed = a), bit i at (a + b*i) mod bits.  R bit positions are fetched per round
// (independent loads, one memory round trip); the result is the same AND of all bits for any R.
template <int R>
KHB_HD bool bloom_steps(const uint8_t* __restrict__ bf, const BloomGeom& g, uint64_t a, uint64_t b) {
  uint64_t pos = mod_bits(a, g);
  const uint64_t bm = mod_bits(b, g);
  uint64_t h = a;
  for (uint32_t i = 1; i < g.hashes; i += R) {
    uint64_t ps[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t nh = h + b;
      const bool wrapped = nh < h;
      h = nh;
      pos += bm;
      if (pos >= g.bits) pos -= g.bits;
      if (wrapped) pos = (pos >= g.wrap) ? pos - g.wrap : pos + g.bits - g.wrap;
      ps[r] = pos;
    }
    bool ok = true;
#pragma unroll
    for (int r = 0; r < R; ++r) ok &= (i + r >= g.hashes) || test_bit(bf, ps[r]);
    if (!ok) return false;
  }
  return true;
}

template <int R>
KHB_HD bool bloom_rest_r(const uint8_t* __restrict__ bf, const BloomGeom& g, const uint64_t w[4], uint64_t a) {
  return bloom_steps<R>(bf, g, a, xxh64_32(w, a));
}

// The whole bloom_check for x with first hash a (the gate path: L1 bit 0 not yet read).  The bit-0
// load is issued before the second hash, so the hash runs under the load's latency.
template <int R>
KHB_HD bool bloom_full(const uint8_t* __restrict__ bf, const BloomGeom& g, const uint64_t w[4], uint64_t a) {
  const uint64_t p0 = mod_bits(a, g);
  const uint32_t t0 = bf[p0 >> 3];
  const uint64_t b = xxh64_32(w, a);
  if (!((t0 >> (p0 & 7)) & 1u)) return false;
  return bloom_steps<R>(bf, g, a, b);
}

KHB_HD bool bloom_rest(const uint8_t* __restrict__ bf, const BloomGeom& g, const uint64_t w[4], uint64_t a) {
  return bloom_rest_r<1>(bf, g, w, a);
}

// bloom_check(&bloom_bP[xb[0]], xb, 32) != 0 for x (bloom.cpp:128-156).
KHB_HD bool bloom_probe_x(const uint8_t* __restrict__ bf_all, const BloomGeom& g, const Fe& x) {
  const uint8_t* bf = sub_bloom(bf_all, g, x);
  uint64_t w[4];
  x_words(w, x);
  const uint64_t a = xxh64_32(w, KHB_BLOOM_SEED);
  if (!test_bit(bf, mod_bits(a, g))) return false;
  return bloom_rest(bf, g, w, a);
}

}  // namespace khb
