// Bitcoin hash160 of secp256k1 public keys (RIPEMD-160(SHA-256(pubkey))) and the 20-byte bloom
// probe of keyhunt's -m address / -m rmd160 modes, specialised for the fixed message shapes the
// reference hashes (SECP256K1.cpp:584-789, hash/sha256.cpp, hash/ripemd160.cpp):
//   compressed   : 0x02|0x03 || x (33 bytes, one SHA-256 block)
//   uncompressed : 0x04 || x || y (65 bytes, two SHA-256 blocks)
//   RIPEMD-160 of the 32-byte SHA-256 digest (one block).
// The algorithms are restated from FIPS 180-4 and Dobbertin-Bosselaers-Preneel (1996); host and
// device share this code (KHB_HD) so tests/native checks it on the CPU against the oracle.
//
// Byte conventions: Fe limbs are little-endian words (v[7] most significant), so the big-endian
// serialisation Get32Bytes(x) is the word stream x.v[7], x.v[6], ..., x.v[0].  The 20-byte hash160
// is returned as five RIPEMD-160 state words h[0..4] whose little-endian bytes are the digest bytes.
#pragma once
#include <stdint.h>
#include "fe.hpp"
#include "bloom_probe.hpp"

namespace khb {

// Rotates and three-input boolean functions.  On gfx950 a rotate is one v_alignbit_b32 and any
// three-input boolean function is one v_bitop3_b32 (the 8-bit truth table over x = 0xF0, y = 0xCC,
// z = 0xAA); the compiler forms bitop3 for ch/maj but not for the xor-of-rotates in the SHA-256
// sigmas nor alignbit for RIPEMD-160's left rotates, so they are spelled out (VALU per SHA-256
// block 1690 -> ~1450, RIPEMD-160 1153 -> ~1000).  The host build keeps the plain C expressions.
KHB_HD uint32_t ror32(uint32_t x, int r) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_amdgcn_alignbit(x, x, (uint32_t)r);
#else
  return (x >> r) | (x << (32 - r));
#endif
}
KHB_HD uint32_t rol32(uint32_t x, int r) { return ror32(x, 32 - r); }
template <uint32_t TT>
KHB_HD uint32_t bitop3(uint32_t x, uint32_t y, uint32_t z) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_amdgcn_bitop3_b32(x, y, z, TT);
#else
  uint32_t r = 0;
  if (TT & 0x01u) r |= ~x & ~y & ~z;
  if (TT & 0x02u) r |= ~x & ~y & z;
  if (TT & 0x04u) r |= ~x & y & ~z;
  if (TT & 0x08u) r |= ~x & y & z;
  if (TT & 0x10u) r |= x & ~y & ~z;
  if (TT & 0x20u) r |= x & ~y & z;
  if (TT & 0x40u) r |= x & y & ~z;
  if (TT & 0x80u) r |= x & y & z;
  return r;
#endif
}
KHB_HD uint32_t xor3(uint32_t x, uint32_t y, uint32_t z) { return bitop3<0x96u>(x, y, z); }

// ---- SHA-256 (FIPS 180-4 §6.2) ----
#define KHB_SHA_K                                                                                            \
  {0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,     \
   0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,     \
   0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,     \
   0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,     \
   0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,     \
   0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,     \
   0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,     \
   0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u}

KHB_HD void sha256_init(uint32_t s[8]) {
  s[0] = 0x6a09e667u; s[1] = 0xbb67ae85u; s[2] = 0x3c6ef372u; s[3] = 0xa54ff53au;
  s[4] = 0x510e527fu; s[5] = 0x9b05688cu; s[6] = 0x1f83d9abu; s[7] = 0x5be0cd19u;
}

// One compression of the 16 big-endian message words w (consumed: used as the schedule ring).
KHB_HD void sha256_block(uint32_t s[8], uint32_t w[16]) {
  const uint32_t K[64] = KHB_SHA_K;
  uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      const uint32_t s0 = xor3(ror32(w15, 7), ror32(w15, 18), w15 >> 3);
      const uint32_t s1 = xor3(ror32(w2, 17), ror32(w2, 19), w2 >> 10);
      wi = w[i & 15] = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
    }
    const uint32_t S1 = xor3(ror32(e, 6), ror32(e, 11), ror32(e, 25));
    const uint32_t ch = bitop3<0xCAu>(e, f, g);                  // (e & f) ^ (~e & g)
    const uint32_t t1 = h + S1 + ch + K[i] + wi;
    const uint32_t S0 = xor3(ror32(a, 2), ror32(a, 13), ror32(a, 22));
    const uint32_t maj = bitop3<0xE8u>(a, b, c);                 // (a & b) ^ (a & c) ^ (b & c)
    const uint32_t t2 = S0 + maj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
}

// ---- RIPEMD-160 (one block: the 32-byte SHA-256 digest + padding) ----
KHB_HD uint32_t rmd_f(int j, uint32_t x, uint32_t y, uint32_t z) {
  return j < 16 ? bitop3<0x96u>(x, y, z)     // x ^ y ^ z
       : j < 32 ? bitop3<0xCAu>(x, y, z)     // (x & y) | (~x & z)
       : j < 48 ? bitop3<0x59u>(x, y, z)     // (x | ~y) ^ z
       : j < 64 ? bitop3<0xE4u>(x, y, z)     // (x & z) | (y & ~z)
                : bitop3<0x2Du>(x, y, z);    // x ^ (y | ~z)
}

// digest = SHA-256 state words (big-endian digest bytes); out = RIPEMD-160 state words.
KHB_HD void ripemd160_of_sha(uint32_t out[5], const uint32_t digest[8]) {
  const uint8_t R1[80] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 7, 4, 13, 1, 10, 6, 15, 3, 12, 0,
                          9, 5, 2, 14, 11, 8, 3, 10, 14, 4, 9, 15, 8, 1, 2, 7, 0, 6, 13, 11, 5, 12, 1, 9, 11, 10,
                          0, 8, 12, 4, 13, 3, 7, 15, 14, 5, 6, 2, 4, 0, 5, 9, 7, 12, 2, 10, 14, 1, 3, 8, 11, 6, 15, 13};
  const uint8_t R2[80] = {5, 14, 7, 0, 9, 2, 11, 4, 13, 6, 15, 8, 1, 10, 3, 12, 6, 11, 3, 7, 0, 13, 5, 10, 14, 15,
                          8, 12, 4, 9, 1, 2, 15, 5, 1, 3, 7, 14, 6, 9, 11, 8, 12, 2, 10, 0, 4, 13, 8, 6, 4, 1,
                          3, 11, 15, 0, 5, 12, 2, 13, 9, 7, 10, 14, 12, 15, 10, 4, 1, 5, 8, 7, 6, 2, 13, 14, 0, 3, 9, 11};
  const uint8_t S1[80] = {11, 14, 15, 12, 5, 8, 7, 9, 11, 13, 14, 15, 6, 7, 9, 8, 7, 6, 8, 13, 11, 9, 7, 15, 7, 12,
                          15, 9, 11, 7, 13, 12, 11, 13, 6, 7, 14, 9, 13, 15, 14, 8, 13, 6, 5, 12, 7, 5, 11, 12, 14, 15,
                          14, 15, 9, 8, 9, 14, 5, 6, 8, 6, 5, 12, 9, 15, 5, 11, 6, 8, 13, 12, 5, 12, 13, 14, 11, 8, 5, 6};
  const uint8_t S2[80] = {8, 9, 9, 11, 13, 15, 15, 5, 7, 7, 8, 11, 14, 14, 12, 6, 9, 13, 15, 7, 12, 8, 9, 11, 7, 7,
                          12, 7, 6, 15, 13, 11, 9, 7, 15, 11, 8, 6, 6, 14, 12, 13, 5, 14, 13, 13, 7, 5, 15, 5, 8, 11,
                          14, 14, 6, 14, 6, 9, 12, 9, 12, 5, 15, 8, 8, 5, 12, 9, 12, 5, 14, 6, 8, 13, 6, 5, 15, 13, 11, 11};
  const uint32_t K1[5] = {0x00000000u, 0x5A827999u, 0x6ED9EBA1u, 0x8F1BBCDCu, 0xA953FD4Eu};
  const uint32_t K2[5] = {0x50A28BE6u, 0x5C4DD124u, 0x6D703EF3u, 0x7A6D76E9u, 0x00000000u};
  uint32_t X[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t v = digest[k];   // big-endian digest word -> little-endian message word
    X[k] = (v >> 24) | ((v >> 8) & 0xff00u) | ((v << 8) & 0xff0000u) | (v << 24);
  }
  X[8] = 0x80u;
#pragma unroll
  for (int k = 9; k < 16; ++k) X[k] = 0;
  X[14] = 256u;
  const uint32_t h0 = 0x67452301u, h1 = 0xEFCDAB89u, h2 = 0x98BADCFEu, h3 = 0x10325476u, h4 = 0xC3D2E1F0u;
  uint32_t al = h0, bl = h1, cl = h2, dl = h3, el = h4;
  uint32_t ar = h0, br = h1, cr = h2, dr = h3, er = h4;
#pragma unroll
  for (int j = 0; j < 80; ++j) {
    uint32_t t = rol32(al + rmd_f(j, bl, cl, dl) + X[R1[j]] + K1[j >> 4], S1[j]) + el;
    al = el; el = dl; dl = rol32(cl, 10); cl = bl; bl = t;
    t = rol32(ar + rmd_f(79 - j, br, cr, dr) + X[R2[j]] + K2[j >> 4], S2[j]) + er;
    ar = er; er = dr; dr = rol32(cr, 10); cr = br; br = t;
  }
  const uint32_t t = h1 + cl + dr;
  out[1] = h2 + dl + er;
  out[2] = h3 + el + ar;
  out[3] = h4 + al + br;
  out[4] = h0 + bl + cr;
  out[0] = t;
}

// hash160 of the compressed key prefix || x (prefix 2 or 3).
KHB_HD void hash160_compressed(uint32_t out[5], uint32_t prefix, const Fe& x) {
  uint32_t w[16], s[8];
  w[0] = (prefix << 24) | (x.v[7] >> 8);
#pragma unroll
  for (int k = 1; k < 8; ++k) w[k] = (x.v[8 - k] << 24) | (x.v[7 - k] >> 8);
  w[8] = (x.v[0] << 24) | 0x00800000u;
#pragma unroll
  for (int k = 9; k < 15; ++k) w[k] = 0;
  w[15] = 33u * 8u;
  sha256_init(s);
  sha256_block(s, w);
  ripemd160_of_sha(out, s);
}

// hash160 of the uncompressed key 04 || x || y.
KHB_HD void hash160_uncompressed(uint32_t out[5], const Fe& x, const Fe& y) {
  uint32_t w[16], s[8];
  uint32_t S[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    S[k] = x.v[7 - k];
    S[8 + k] = y.v[7 - k];
  }
  w[0] = (0x04u << 24) | (S[0] >> 8);
#pragma unroll
  for (int k = 1; k < 16; ++k) w[k] = (S[k - 1] << 24) | (S[k] >> 8);
  sha256_init(s);
  sha256_block(s, w);
  w[0] = (S[15] << 24) | 0x00800000u;
#pragma unroll
  for (int k = 1; k < 15; ++k) w[k] = 0;
  w[15] = 65u * 8u;
  sha256_block(s, w);
  ripemd160_of_sha(out, s);
}

// XXH64 (xxhash.h v0.8.0, len < 32 path: XXH64_finalize + avalanche) of the 20 hash160 bytes.
KHB_HD uint64_t xxh64_20(const uint32_t h[5], uint64_t seed) {
  const uint64_t P1 = 0x9E3779B185EBCA87ull, P2 = 0xC2B2AE3D27D4EB4Full, P3 = 0x165667B19E3779F9ull,
                 P4 = 0x85EBCA77C2B2AE63ull, P5 = 0x27D4EB2F165667C5ull;
  uint64_t acc = seed + P5 + 20u;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    uint64_t in = (uint64_t)h[2 * k] | ((uint64_t)h[2 * k + 1] << 32);
    uint64_t r = in * P2;
    r = (r << 31) | (r >> 33);
    r *= P1;
    acc ^= r;
    acc = ((acc << 27) | (acc >> 37)) * P1 + P4;
  }
  acc ^= (uint64_t)h[4] * P1;
  acc = ((acc << 23) | (acc >> 41)) * P2 + P3;
  acc ^= acc >> 33;
  acc *= P2;
  acc ^= acc >> 29;
  acc *= P3;
  acc ^= acc >> 32;
  return acc;
}

// bloom_check(&bloom, hash160, 20) (bloom.cpp:128-156) on the single -m address bloom.
KHB_HD bool bloom_check20(const uint8_t* __restrict__ bf, const BloomGeom& g, const uint32_t h[5]) {
  const uint64_t a = xxh64_20(h, KHB_BLOOM_SEED);
  if (!test_bit(bf, mod_bits(a, g))) return false;
  return bloom_steps<1>(bf, g, a, xxh64_20(h, a));
}

}  // namespace khb
