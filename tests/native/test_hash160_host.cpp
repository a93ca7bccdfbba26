// Host-side check of device/hash160.hpp (compiled for the CPU) against the oracle's spec
// restatements of SHA-256 / RIPEMD-160 / XXH64 / bloom_check.  Test infrastructure.
#include "../../keyhuntm1cpu_amd/csrc/device/hash160.hpp"
extern "C" {
#include "../../oracle/ora.h"
}
#include <cstdio>
#include <cstring>
using namespace khb;

static uint64_t sm = 7;
static uint64_t splitmix() { uint64_t z = (sm += 0x9E3779B97F4A7C15ull); z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; return z ^ (z >> 31); }

static void words_to_bytes(const uint32_t h[5], uint8_t out[20]) {
  for (int k = 0; k < 5; ++k)
    for (int b = 0; b < 4; ++b) out[4 * k + b] = (uint8_t)(h[k] >> (8 * b));
}

int main() {
  int fails = 0;
  ora_secp_init();
  // bloom of 20-byte keys as -m address builds it (initBloomFilter: 10000 entries, 1e-6)
  ora_bloom bl;
  ora_bloom_init2(&bl, 10000, 0.000001L);
  for (int i = 0; i < 3000; ++i) {
    uint8_t v[20];
    for (int k = 0; k < 20; ++k) v[k] = (uint8_t)splitmix();
    ora_bloom_add(&bl, v, 20);
  }
  BloomGeom g;
  g.bytes_per_sub = bl.bytes;
  g.bits = bl.bits;
  g.magic = (uint64_t)(((unsigned __int128)1 << 64) / bl.bits);
  g.wrap = (uint64_t)(((unsigned __int128)1 << 64) % bl.bits);
  g.hashes = bl.hashes;
  int hits = 0;
  for (int it = 0; it < 20000; ++it) {
    ora_point P;
    ora_u256 k;
    for (int w = 0; w < 4; ++w) k.w[w] = splitmix();
    k.w[3] &= 0x7fffffffffffffffull;
    if (it < 8) ora_u256_set64(&k, (uint64_t)it + 1);
    ora_compute_pubkey(&P, &k);
    uint8_t xb[32], yb[32];
    ora_u256_to_be(&P.x, xb);
    ora_u256_to_be(&P.y, yb);
    Fe x, y;
    fe_from_be(x, xb);
    fe_from_be(y, yb);
    uint32_t h[5];
    uint8_t got[20], ref[20];
    for (int kind = 0; kind < 3; ++kind) {
      if (kind < 2) {
        hash160_compressed(h, 2u + (uint32_t)kind, x);
        ora_x_hash160((uint8_t)(2 + kind), &P.x, ref);
      } else {
        hash160_uncompressed(h, x, y);
        ora_pub_hash160(&P, 0, ref);
      }
      words_to_bytes(h, got);
      if (memcmp(got, ref, 20)) {
        if (fails < 5) printf("hash160 mismatch it %d kind %d\n", it, kind);
        ++fails;
      }
      const uint64_t a = xxh64_20(h, KHB_BLOOM_SEED), ar = ora_xxh64(ref, 20, KHB_BLOOM_SEED);
      if (a != ar) {
        if (fails < 5) printf("xxh64_20 mismatch it %d\n", it);
        ++fails;
      }
      const bool c = bloom_check20(bl.bf, g, h);
      const bool cr = ora_bloom_check(&bl, ref, 20) != 0;
      if (c != cr) {
        if (fails < 5) printf("bloom mismatch it %d\n", it);
        ++fails;
      }
    }
    // members must hit (no false negatives): re-add this key's compressed hash and check
    if (it % 97 == 0) {
      ora_x_hash160(2, &P.x, ref);
      ora_bloom_add(&bl, ref, 20);
      hash160_compressed(h, 2u, x);
      if (!bloom_check20(bl.bf, g, h)) { printf("member miss it %d\n", it); ++fails; }
      ++hits;
    }
  }
  ora_bloom_free(&bl);
  printf("hash160 host check: %s (%d fails, %d member probes)\n", fails ? "FAIL" : "ok", fails, hits);
  return fails ? 1 : 0;
}
