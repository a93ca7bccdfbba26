// Host-side check of the device arithmetic headers (compiled for the CPU) against the oracle.
// Test infrastructure: links oracle/liboracle (the checker).
#include "../../keyhuntm1cpu_amd/csrc/device/fe.hpp"
#include "../../keyhuntm1cpu_amd/csrc/device/bloom_probe.hpp"
extern "C" {
#include "../../oracle/ora.h"
}
#include <cstdio>
#include <cstring>
#include <cstdlib>
using namespace khb;

static uint64_t sm = 1;
static uint64_t splitmix() { uint64_t z = (sm += 0x9E3779B97F4A7C15ull); z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; return z ^ (z >> 31); }
static void rnd_fe(uint8_t b[32], int mode) {
  for (int i = 0; i < 32; ++i) b[i] = (uint8_t)splitmix();
  if (mode == 1) memset(b, 0xFF, 28);             // near p
  if (mode == 2) memset(b, 0, 24);                // small
  // reduce mod p (canonical input)
  ora_u256 v; ora_u256_from_be(&v, b);
  while (ora_u256_cmp(&v, ora_prime()) >= 0) ora_u256_sub(&v, &v, ora_prime());
  ora_u256_to_be(&v, b);
}
int main() {
  int fails = 0;
  for (int it = 0; it < 200000; ++it) {
    uint8_t a[32], b[32], r1[32], r2[32];
    rnd_fe(a, it % 5 == 1 ? 1 : it % 5 == 2 ? 2 : 0);
    rnd_fe(b, it % 7 == 1 ? 1 : it % 7 == 2 ? 2 : 0);
    if (it == 3) memset(a, 0, 32);
    Fe fa, fb, fr; fe_from_be(fa, a); fe_from_be(fb, b);
    ora_u256 oa, ob, orr; ora_u256_from_be(&oa, a); ora_u256_from_be(&ob, b);
    for (int op = 0; op < 5; ++op) {
      if (op == 4 && it % 50) continue;
      switch (op) {
        case 0: fe_mul(fr, fa, fb); ora_fe_mul_exact(&orr, &oa, &ob); break;
        case 1: fe_sqr(fr, fa); ora_fe_mul_exact(&orr, &oa, &oa); break;
        case 2: fe_add(fr, fa, fb); ora_fe_add(&orr, &oa, &ob); break;
        case 3: fe_sub(fr, fa, fb); ora_fe_sub(&orr, &oa, &ob); break;
        case 4: fe_inv(fr, fa); ora_fe_inv(&orr, &oa); break;
      }
      fe_to_be(r1, fr); ora_u256_to_be(&orr, r2);
      if (memcmp(r1, r2, 32)) { if (fails++ < 10) printf("op %d mismatch it %d\n", op, it); }
    }
    // xxh64 on 32 bytes
    uint64_t w[4]; x_words(w, fa);
    if (xxh64_32(w, 0x59f2815b16f81798ull) != ora_xxh64(a, 32, 0x59f2815b16f81798ull)) { if (fails++ < 10) printf("xxh mismatch\n"); }
    uint64_t s = splitmix();
    if (xxh64_32(w, s) != ora_xxh64(a, 32, s)) { if (fails++ < 10) printf("xxh seed mismatch\n"); }
  }
  // bloom probe vs ora_bloom_check on a small synthetic bloom
  ora_bloom bl[256];
  for (int i = 0; i < 256; ++i) ora_bloom_init2(&bl[i], 1000, 0.000001);
  uint8_t* cat = (uint8_t*)malloc(bl[0].bytes * 256);
  uint8_t xs[3000][32];
  for (int i = 0; i < 3000; ++i) { rnd_fe(xs[i], 0); ora_bloom_add(&bl[xs[i][0]], xs[i], 32); }
  for (int i = 0; i < 256; ++i) memcpy(cat + bl[0].bytes * i, bl[i].bf, bl[0].bytes);
  BloomGeom g; g.bytes_per_sub = bl[0].bytes; g.bits = bl[0].bits; g.hashes = bl[0].hashes;
  g.magic = (uint64_t)(((unsigned __int128)1 << 64) / g.bits); g.wrap = (uint64_t)(((unsigned __int128)1 << 64) % g.bits);
  int hits = 0;
  for (int i = 0; i < 200000; ++i) {
    uint8_t x[32];
    if (i < 3000) memcpy(x, xs[i], 32); else rnd_fe(x, 0);
    Fe fx; fe_from_be(fx, x);
    bool h1 = bloom_probe_x(cat, g, fx);
    bool h2 = ora_bloom_check(&bl[x[0]], x, 32) != 0;
    hits += h1;
    if (h1 != h2) { if (fails++ < 10) printf("probe mismatch %d\n", i); }
  }
  printf("bloom bits=%llu hashes=%u hits=%d\n", (unsigned long long)g.bits, g.hashes, hits);
  printf(fails ? "FAILED %d\n" : "OK\n", fails);
  return fails != 0;
}
