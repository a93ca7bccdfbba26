// Host bloom filter: libbloom v2 semantics used by keyhunt (bloom/bloom.h:26-45,
// bloom/bloom.cpp:93-162) for the two key shapes keyhunt hashes: 32-byte x-coordinates (-m bsgs)
// and 20-byte hash160 values (-m address / -m rmd160).
#pragma once
#include <stdint.h>
#include <vector>

#include "../device/bloom_probe.hpp"

namespace khb {

struct BloomFilter {
  uint64_t entries = 0, bits = 0, bytes = 0;
  uint8_t hashes = 0;
  long double error = 0;
  double bpe = 0;
  bool ready = false;
  std::vector<uint8_t> bf;

  // bloom_init2: bits = entries * (-ln(err) / ln(2)^2) in long double, hashes = ceil(ln2 * bpe).
  int init2(uint64_t n_entries, long double err);
  // bloom_check / bloom_add on Get32Bytes(x) (keyhunt.cpp:3945-3946, 4515-4560).
  bool check32(const uint8_t x[32]) const;
  void add32_atomic(const uint8_t x[32]);     // thread-safe byte OR: same bits as mutex + bloom_add
  // bloom_check / bloom_add on a 20-byte hash160 (keyhunt.cpp:6341-6350, 2793-2800)
  bool check20(const uint8_t h[20]) const;
  void add20(const uint8_t h[20]);
  BloomGeom geom() const;
};

void words_of_bytes32(uint64_t w[4], const uint8_t x[32]);

}  // namespace khb
