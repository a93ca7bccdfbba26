#include "bloom_host.hpp"
#include "../device/hash160.hpp"

#include <math.h>
#include <string.h>

namespace khb {

void words_of_bytes32(uint64_t w[4], const uint8_t x[32]) {
  for (int k = 0; k < 4; ++k) memcpy(&w[k], x + 8 * k, 8);   // little-endian host, XXH_readLE64
}

int BloomFilter::init2(uint64_t n_entries, long double err) {
  *this = BloomFilter();
  if (n_entries < 1000 || err <= 0 || err >= 1) return 1;
  entries = n_entries;
  error = err;
  const long double num = -logl(error);
  const long double denom = 0.480453013918201;   // ln(2)^2 as the reference spells it
  bpe = (double)(num / denom);
  const long double allbits = (long double)entries * bpe;
  bits = (uint64_t)allbits;
  bytes = bits / 8 + ((bits % 8) ? 1 : 0);
  hashes = (uint8_t)ceil(0.693147180559945 * bpe);
  bf.assign(bytes, 0);
  ready = true;
  return 0;
}

BloomGeom BloomFilter::geom() const {
  BloomGeom g;
  g.bytes_per_sub = bytes;
  g.bits = bits;
  g.magic = (uint64_t)(((unsigned __int128)1 << 64) / bits);
  g.wrap = (uint64_t)(((unsigned __int128)1 << 64) % bits);
  g.hashes = hashes;
  return g;
}

bool BloomFilter::check32(const uint8_t x[32]) const {
  uint64_t w[4];
  words_of_bytes32(w, x);
  const uint64_t a = xxh64_32(w, KHB_BLOOM_SEED);
  const uint64_t b = xxh64_32(w, a);
  for (uint32_t i = 0; i < hashes; ++i) {
    const uint64_t pos = (a + b * i) % bits;
    if (!((bf[pos >> 3] >> (pos & 7)) & 1)) return false;
  }
  return true;
}

void BloomFilter::add32_atomic(const uint8_t x[32]) {
  uint64_t w[4];
  words_of_bytes32(w, x);
  const uint64_t a = xxh64_32(w, KHB_BLOOM_SEED);
  const uint64_t b = xxh64_32(w, a);
  uint8_t* base = bf.data();
  for (uint32_t i = 0; i < hashes; ++i) {
    const uint64_t pos = (a + b * i) % bits;
    const uint8_t m = (uint8_t)(1u << (pos & 7));
    if (!(__atomic_load_n(&base[pos >> 3], __ATOMIC_RELAXED) & m)) __atomic_fetch_or(&base[pos >> 3], m, __ATOMIC_RELAXED);
  }
}

static void words_of_bytes20(uint32_t h[5], const uint8_t b[20]) {
  for (int k = 0; k < 5; ++k) memcpy(&h[k], b + 4 * k, 4);   // little-endian host
}

bool BloomFilter::check20(const uint8_t hb[20]) const {
  uint32_t h[5];
  words_of_bytes20(h, hb);
  const uint64_t a = xxh64_20(h, KHB_BLOOM_SEED);
  const uint64_t b = xxh64_20(h, a);
  for (uint32_t i = 0; i < hashes; ++i) {
    const uint64_t pos = (a + b * i) % bits;
    if (!((bf[pos >> 3] >> (pos & 7)) & 1)) return false;
  }
  return true;
}

void BloomFilter::add20(const uint8_t hb[20]) {
  uint32_t h[5];
  words_of_bytes20(h, hb);
  const uint64_t a = xxh64_20(h, KHB_BLOOM_SEED);
  const uint64_t b = xxh64_20(h, a);
  for (uint32_t i = 0; i < hashes; ++i) {
    const uint64_t pos = (a + b * i) % bits;
    bf[pos >> 3] |= (uint8_t)(1u << (pos & 7));
  }
}

}  // namespace khb
