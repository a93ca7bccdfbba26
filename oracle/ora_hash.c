/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see ora.h).
 * XXH64 (xxhash/xxhash.h:2290-2527, vendored xxHash v0.8.0 — source present in the reference, so
 * not an unpinned dependency) and the bloom filter of bloom/bloom.cpp.
 */
#include "ora.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

#define PR1 0x9E3779B185EBCA87ULL   /* xxhash.h:2290-2294 */
#define PR2 0xC2B2AE3D27D4EB4FULL
#define PR3 0x165667B19E3779F9ULL
#define PR4 0x85EBCA77C2B2AE63ULL
#define PR5 0x27D4EB2F165667C5ULL

static uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }   /* little-endian host */
static uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }

/* XXH64_round xxhash.h:2304-2310 */
static uint64_t xround(uint64_t acc, uint64_t in) { acc += in * PR2; acc = rotl(acc, 31); return acc * PR1; }
/* XXH64_mergeRound xxhash.h:2312-2318 */
static uint64_t xmerge(uint64_t acc, uint64_t v) { v = xround(0, v); acc ^= v; return acc * PR1 + PR4; }

/* XXH64 (xxhash.h:2468-2527) with XXH64_finalize's byte-wise tail (xxhash.h:2333-2456). */
uint64_t ora_xxh64(const void* buf, size_t len, uint64_t seed) {
  const uint8_t* p = (const uint8_t*)buf;
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    const uint8_t* lim = end - 32;
    uint64_t v1 = seed + PR1 + PR2, v2 = seed + PR2, v3 = seed, v4 = seed - PR1;
    do {
      v1 = xround(v1, rd64(p)); p += 8;
      v2 = xround(v2, rd64(p)); p += 8;
      v3 = xround(v3, rd64(p)); p += 8;
      v4 = xround(v4, rd64(p)); p += 8;
    } while (p <= lim);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    h = xmerge(h, v1); h = xmerge(h, v2); h = xmerge(h, v3); h = xmerge(h, v4);
  } else {
    h = seed + PR5;
  }
  h += (uint64_t)len;
  size_t rem = len & 31;
  while (rem >= 8) { h ^= xround(0, rd64(p)); h = rotl(h, 27) * PR1 + PR4; p += 8; rem -= 8; }
  if (rem >= 4) { h ^= (uint64_t)rd32(p) * PR1; h = rotl(h, 23) * PR2 + PR3; p += 4; rem -= 4; }
  while (rem > 0) { h ^= (*p++) * PR5; h = rotl(h, 11) * PR1; --rem; }
  /* XXH64_avalanche xxhash.h:2320-2328 */
  h ^= h >> 33; h *= PR2; h ^= h >> 29; h *= PR3; h ^= h >> 32;
  return h;
}

/* bloom_init2 (bloom.cpp:93-126): long-double sizing exactly as compiled from C++ (log() on a long
 * double argument resolves to the long-double overload). */
int ora_bloom_init2(ora_bloom* b, uint64_t entries, long double error) {
  memset(b, 0, sizeof(*b));
  if (entries < 1000 || error <= 0 || error >= 1) return 1;
  b->entries = entries;
  b->error = error;
  long double num = -logl(b->error);
  long double denom = 0.480453013918201;
  b->bpe = (double)(num / denom);
  long double dentries = (long double)entries;
  long double allbits = dentries * b->bpe;
  b->bits = (uint64_t)allbits;
  b->bytes = b->bits / 8;
  if (b->bits % 8) b->bytes += 1;
  b->hashes = (uint8_t)ceil(0.693147180559945 * b->bpe);
  b->bf = (uint8_t*)calloc(b->bytes, 1);
  if (!b->bf) return 1;
  b->ready = 1;
  b->major = 2;
  b->minor = 201;
  return 0;
}

/* bloom_check (bloom.cpp:128-156): first zero bit returns 0; -1 when not ready. */
int ora_bloom_check(const ora_bloom* b, const void* buf, int len) {
  if (!b->ready) return -1;
  uint64_t a = ora_xxh64(buf, (size_t)len, 0x59f2815b16f81798ULL);
  uint64_t bb = ora_xxh64(buf, (size_t)len, a);
  for (uint8_t i = 0; i < b->hashes; ++i) {
    uint64_t x = (a + bb * i) % b->bits;
    if (!(b->bf[x >> 3] & (1u << (x % 8)))) return 0;
  }
  return 1;
}

/* bloom_check_add with add=1 (bloom.cpp:61-85, 159-162) */
int ora_bloom_add(ora_bloom* b, const void* buf, int len) {
  if (!b->ready) return -1;
  uint64_t a = ora_xxh64(buf, (size_t)len, 0x59f2815b16f81798ULL);
  uint64_t bb = ora_xxh64(buf, (size_t)len, a);
  uint8_t hits = 0;
  for (uint8_t i = 0; i < b->hashes; ++i) {
    uint64_t x = (a + bb * i) % b->bits;
    uint8_t m = (uint8_t)(1u << (x % 8));
    if (b->bf[x >> 3] & m) hits++;
    else b->bf[x >> 3] |= m;
  }
  return hits == b->hashes ? 1 : 0;
}

void ora_bloom_free(ora_bloom* b) {
  if (b->ready) free(b->bf);
  b->ready = 0;
  b->bf = NULL;
}
