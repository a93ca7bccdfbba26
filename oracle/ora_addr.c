/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see ora.h).
 *
 * Plain-C restatement of keyhunt's `-m address` / `-m rmd160` path for BTC P2PKH targets:
 *   - SHA-256 (FIPS 180-4) and RIPEMD-160 (Dobbertin-Bosselaers-Preneel 1996), the algorithms of
 *     hash/sha256.cpp and hash/ripemd160.cpp, restated from their specifications;
 *   - hash160 of public keys: SECP256K1.cpp:584-789 (GetHash160, GetHash160_fromX);
 *   - target file loading: keyhunt.cpp:6300-6358 (forceReadFileAddress) with base58 decoding as
 *     base58/base58.c:39-112 (b58tobin) and encoding as :145-189 (b58enc); the bloom sizing of
 *     initBloomFilter keyhunt.cpp:6559-6576; _sort keyhunt.cpp (memcmp order of 20-byte values);
 *   - searchbinary keyhunt.cpp:2311-2335 (literal, including its probe sequence);
 *   - one group of thread_process keyhunt.cpp:2586-2711 and its checks :2789-2937 (BTC), the key
 *     recovery rules and the chunk claiming of :2546-2567 / :3050-3057; with -e the endomorphism
 *     points (beta*x, beta^2*x: keyhunt.cpp:579-585, 2646-2676, 2685-2711), their 6 compressed and
 *     6 uncompressed hashes (2716-2763) and the lambda key recovery (2800-2937).
 * The -e constants (lambda, lambda^2 mod n; beta, beta^2 mod p) are the reference's literals
 * (keyhunt.cpp:582-585); tests check lambda*G = (beta*G.x, G.y).
 * Pins: tests/1to32.rmd + tests/1to32.txt (hash160 / address of puzzle keys 1..32), tests/66.rmd,
 * published SHA-256 / RIPEMD-160 test vectors (tests/test_oracle_addr.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include "ora.h"

/* ---------------------------------------------------------------- SHA-256 */
static const uint32_t SHA_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static uint32_t ror(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }
static uint32_t rol(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

static void sha256_compress(uint32_t h[8], const uint8_t blk[64]) {
  uint32_t w[64], a, b, c, d, e, f, g, hh;
  for (int i = 0; i < 16; ++i)
    w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) | ((uint32_t)blk[4 * i + 2] << 8) | blk[4 * i + 3];
  for (int i = 16; i < 64; ++i) {
    uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  a = h[0]; b = h[1]; c = h[2]; d = h[3]; e = h[4]; f = h[5]; g = h[6]; hh = h[7];
  for (int i = 0; i < 64; ++i) {
    uint32_t t1 = hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + SHA_K[i] + w[i];
    uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

void ora_sha256(const uint8_t* msg, size_t len, uint8_t out[32]) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint8_t blk[64];
  size_t i = 0;
  for (; i + 64 <= len; i += 64) sha256_compress(h, msg + i);
  size_t rem = len - i;
  memset(blk, 0, 64);
  memcpy(blk, msg + i, rem);
  blk[rem] = 0x80;
  if (rem >= 56) {
    sha256_compress(h, blk);
    memset(blk, 0, 64);
  }
  uint64_t bits = (uint64_t)len * 8;
  for (int k = 0; k < 8; ++k) blk[63 - k] = (uint8_t)(bits >> (8 * k));
  sha256_compress(h, blk);
  for (int k = 0; k < 8; ++k) {
    out[4 * k] = (uint8_t)(h[k] >> 24); out[4 * k + 1] = (uint8_t)(h[k] >> 16);
    out[4 * k + 2] = (uint8_t)(h[k] >> 8); out[4 * k + 3] = (uint8_t)h[k];
  }
}

/* ------------------------------------------------------------- RIPEMD-160 */
static const uint8_t RR1[80] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 7, 4, 13, 1, 10, 6, 15, 3, 12, 0,
                               9, 5, 2, 14, 11, 8, 3, 10, 14, 4, 9, 15, 8, 1, 2, 7, 0, 6, 13, 11, 5, 12, 1, 9, 11, 10,
                               0, 8, 12, 4, 13, 3, 7, 15, 14, 5, 6, 2, 4, 0, 5, 9, 7, 12, 2, 10, 14, 1, 3, 8, 11, 6, 15, 13};
static const uint8_t RR2[80] = {5, 14, 7, 0, 9, 2, 11, 4, 13, 6, 15, 8, 1, 10, 3, 12, 6, 11, 3, 7, 0, 13, 5, 10, 14, 15,
                               8, 12, 4, 9, 1, 2, 15, 5, 1, 3, 7, 14, 6, 9, 11, 8, 12, 2, 10, 0, 4, 13, 8, 6, 4, 1,
                               3, 11, 15, 0, 5, 12, 2, 13, 9, 7, 10, 14, 12, 15, 10, 4, 1, 5, 8, 7, 6, 2, 13, 14, 0, 3, 9, 11};
static const uint8_t RS1[80] = {11, 14, 15, 12, 5, 8, 7, 9, 11, 13, 14, 15, 6, 7, 9, 8, 7, 6, 8, 13, 11, 9, 7, 15, 7, 12,
                               15, 9, 11, 7, 13, 12, 11, 13, 6, 7, 14, 9, 13, 15, 14, 8, 13, 6, 5, 12, 7, 5, 11, 12, 14, 15,
                               14, 15, 9, 8, 9, 14, 5, 6, 8, 6, 5, 12, 9, 15, 5, 11, 6, 8, 13, 12, 5, 12, 13, 14, 11, 8, 5, 6};
static const uint8_t RS2[80] = {8, 9, 9, 11, 13, 15, 15, 5, 7, 7, 8, 11, 14, 14, 12, 6, 9, 13, 15, 7, 12, 8, 9, 11, 7, 7,
                               12, 7, 6, 15, 13, 11, 9, 7, 15, 11, 8, 6, 6, 14, 12, 13, 5, 14, 13, 13, 7, 5, 15, 5, 8, 11,
                               14, 14, 6, 14, 6, 9, 12, 9, 12, 5, 15, 8, 8, 5, 12, 9, 12, 5, 14, 6, 8, 13, 6, 5, 15, 13, 11, 11};

static uint32_t rf(int j, uint32_t x, uint32_t y, uint32_t z) {
  if (j < 16) return x ^ y ^ z;
  if (j < 32) return (x & y) | (~x & z);
  if (j < 48) return (x | ~y) ^ z;
  if (j < 64) return (x & z) | (y & ~z);
  return x ^ (y | ~z);
}

static void rmd_compress(uint32_t h[5], const uint8_t blk[64]) {
  static const uint32_t K1[5] = {0x00000000, 0x5A827999, 0x6ED9EBA1, 0x8F1BBCDC, 0xA953FD4E};
  static const uint32_t K2[5] = {0x50A28BE6, 0x5C4DD124, 0x6D703EF3, 0x7A6D76E9, 0x00000000};
  uint32_t X[16];
  for (int i = 0; i < 16; ++i)
    X[i] = (uint32_t)blk[4 * i] | ((uint32_t)blk[4 * i + 1] << 8) | ((uint32_t)blk[4 * i + 2] << 16) | ((uint32_t)blk[4 * i + 3] << 24);
  uint32_t al = h[0], bl = h[1], cl = h[2], dl = h[3], el = h[4];
  uint32_t ar = h[0], br = h[1], cr = h[2], dr = h[3], er = h[4];
  for (int j = 0; j < 80; ++j) {
    uint32_t t = rol(al + rf(j, bl, cl, dl) + X[RR1[j]] + K1[j / 16], RS1[j]) + el;
    al = el; el = dl; dl = rol(cl, 10); cl = bl; bl = t;
    t = rol(ar + rf(79 - j, br, cr, dr) + X[RR2[j]] + K2[j / 16], RS2[j]) + er;
    ar = er; er = dr; dr = rol(cr, 10); cr = br; br = t;
  }
  uint32_t t = h[1] + cl + dr;
  h[1] = h[2] + dl + er; h[2] = h[3] + el + ar; h[3] = h[4] + al + br; h[4] = h[0] + bl + cr; h[0] = t;
}

void ora_ripemd160(const uint8_t* msg, size_t len, uint8_t out[20]) {
  uint32_t h[5] = {0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0};
  uint8_t blk[64];
  size_t i = 0;
  for (; i + 64 <= len; i += 64) rmd_compress(h, msg + i);
  size_t rem = len - i;
  memset(blk, 0, 64);
  memcpy(blk, msg + i, rem);
  blk[rem] = 0x80;
  if (rem >= 56) {
    rmd_compress(h, blk);
    memset(blk, 0, 64);
  }
  uint64_t bits = (uint64_t)len * 8;
  for (int k = 0; k < 8; ++k) blk[56 + k] = (uint8_t)(bits >> (8 * k));
  rmd_compress(h, blk);
  for (int k = 0; k < 5; ++k) {
    out[4 * k] = (uint8_t)h[k]; out[4 * k + 1] = (uint8_t)(h[k] >> 8);
    out[4 * k + 2] = (uint8_t)(h[k] >> 16); out[4 * k + 3] = (uint8_t)(h[k] >> 24);
  }
}

void ora_hash160(const uint8_t* msg, size_t len, uint8_t out[20]) {
  uint8_t d[32];
  ora_sha256(msg, len, d);
  ora_ripemd160(d, 32, out);
}

/* GetHash160(P2PKH, compressed, P) SECP256K1.cpp:671-705 */
void ora_pub_hash160(const ora_point* p, int compressed, uint8_t out[20]) {
  uint8_t b[65];
  if (compressed) {
    b[0] = (p->y.w[0] & 1) ? 0x03 : 0x02;
    ora_u256_to_be(&p->x, b + 1);
    ora_hash160(b, 33, out);
  } else {
    b[0] = 0x04;
    ora_u256_to_be(&p->x, b + 1);
    ora_u256_to_be(&p->y, b + 33);
    ora_hash160(b, 65, out);
  }
}

/* GetHash160_fromX(P2PKH, prefix, x) SECP256K1.cpp:707-789 */
void ora_x_hash160(uint8_t prefix, const ora_u256* x, uint8_t out[20]) {
  uint8_t b[33];
  b[0] = prefix;
  ora_u256_to_be(x, b + 1);
  ora_hash160(b, 33, out);
}

/* ------------------------------------------------------------------ base58 */
static const char B58[] = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";

static int b58val(unsigned char c) {
  const char* p = (c & 0x80) ? NULL : strchr(B58, c);
  return (p && c) ? (int)(p - B58) : -1;
}

/* b58tobin (base58.c:39-112) into binsz bytes; returns 1 and the canonical size in *outsz. */
int ora_b58decode(const char* s, uint8_t* bin, size_t binsz, size_t* outsz) {
  size_t n = strlen(s), i, zerocount = 0;
  memset(bin, 0, binsz);
  for (i = 0; i < n && s[i] == '1'; ++i) ++zerocount;
  for (; i < n; ++i) {
    int v = b58val((unsigned char)s[i]);
    if (v < 0) return 0;
    uint32_t carry = (uint32_t)v;
    for (size_t k = binsz; k-- > 0;) {
      uint32_t t = (uint32_t)bin[k] * 58u + carry;
      bin[k] = (uint8_t)t;
      carry = t >> 8;
    }
    if (carry) return 0;   /* too big for binsz bytes */
  }
  size_t lz = 0;
  while (lz < binsz && bin[lz] == 0) ++lz;
  *outsz = binsz - lz + zerocount;
  return 1;
}

/* rmd160toaddress_dst (keyhunt.cpp:2274-2284): base58check of 0x00 || rmd */
void ora_rmd_to_address(const uint8_t rmd[20], char* out) {
  uint8_t d[25], h1[32], h2[32];
  d[0] = 0x00;
  memcpy(d + 1, rmd, 20);
  ora_sha256(d, 21, h1);
  ora_sha256(h1, 32, h2);
  memcpy(d + 21, h2, 4);
  size_t zc = 0;
  while (zc < 25 && !d[zc]) ++zc;
  uint8_t buf[40];
  size_t size = (25 - zc) * 138 / 100 + 1;
  memset(buf, 0, sizeof(buf));
  size_t high = size - 1, j;
  for (size_t i = zc; i < 25; ++i, high = j) {
    int carry = d[i];
    for (j = size - 1; (j > high) || carry; --j) {
      carry += 256 * buf[j];
      buf[j] = (uint8_t)(carry % 58);
      carry /= 58;
      if (!j) break;
    }
  }
  for (j = 0; j < size && !buf[j]; ++j) {}
  size_t o = 0;
  for (size_t k = 0; k < zc; ++k) out[o++] = '1';
  for (; j < size; ++j) out[o++] = B58[buf[j]];
  out[o] = 0;
}

/* ---------------------------------------------------------- address table */
struct ora_addr {
  uint8_t* table;     /* N x 20, sorted */
  uint64_t n;
  ora_bloom bloom;
};

static void trim(char* s) {
  const char* seps = " \t\n\r";
  size_t n = strlen(s);
  while (n && strchr(seps, s[n - 1])) s[--n] = 0;
  size_t k = strspn(s, seps);
  if (k) memmove(s, s + k, n + 1 - k);
}

static int is_b58(const char* s) {
  for (; *s; ++s) if (b58val((unsigned char)*s) < 0) return 0;
  return 1;
}

static int is_hex(const char* s) {
  for (; *s; ++s) {
    char c = *s;
    if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'))) return 0;
  }
  return 1;
}

static int hexval(char c) { return c <= '9' ? c - '0' : (c | 32) - 'a' + 10; }

static int cmp20(const void* a, const void* b) { return memcmp(a, b, 20); }

/* forceReadFileAddress (keyhunt.cpp:6300-6358) over the text of a target file (lines). Quirks
 * kept: the bloom is sized by the count of lines longer than 20 characters, before invalid lines
 * are dropped; 25-byte base58 payloads only (checksum not verified); 40-hex rmd lines. */
ora_addr* ora_addr_new(const char* text, int bloom_multiplier) {
  ora_addr* A = (ora_addr*)calloc(1, sizeof(ora_addr));
  const char* p = text;
  uint64_t counted = 0;
  char line[100];
  /* count lines with > 20 characters after trimming (fgets(aux,100,...)) */
  for (const char* q = p; *q;) {
    const char* e = strchr(q, '\n');
    size_t len = e ? (size_t)(e - q) + 1 : strlen(q);
    size_t c = len < 99 ? len : 99;
    memcpy(line, q, c);
    line[c] = 0;
    trim(line);
    if (strlen(line) > 20) ++counted;
    q += len;
  }
  uint64_t items = counted;
  if (items <= 10000) ora_bloom_init2(&A->bloom, 10000, 0.000001L);
  else ora_bloom_init2(&A->bloom, (uint64_t)bloom_multiplier * items, 0.000001L);
  A->table = (uint8_t*)calloc(counted ? counted : 1, 20);
  uint64_t i = 0;
  const char* q = p;
  while (i < items && *q) {
    const char* e = strchr(q, '\n');
    size_t len = e ? (size_t)(e - q) + 1 : strlen(q);
    size_t c = len < 99 ? len : 99;
    memcpy(line, q, c);
    line[c] = 0;
    q += len;
    trim(line);
    size_t r = strlen(line);
    int valid = 0;
    if (r > 0 && r <= 40) {
      if (r < 40 && is_b58(line)) {
        uint8_t raw[25];
        size_t sz = 0;
        if (ora_b58decode(line, raw, 25, &sz) && sz == 25) {
          ora_bloom_add(&A->bloom, raw + 1, 20);
          memcpy(A->table + 20 * i, raw + 1, 20);
          ++i;
          valid = 1;
        }
      }
      if (r == 40 && is_hex(line)) {
        uint8_t raw[20];
        for (int k = 0; k < 20; ++k) raw[k] = (uint8_t)(hexval(line[2 * k]) * 16 + hexval(line[2 * k + 1]));
        ora_bloom_add(&A->bloom, raw, 20);
        memcpy(A->table + 20 * i, raw, 20);
        ++i;
        valid = 1;
      }
    }
    if (!valid) --items;
  }
  A->n = i;
  qsort(A->table, A->n, 20, cmp20);
  return A;
}

void ora_addr_free(ora_addr* A) {
  if (!A) return;
  ora_bloom_free(&A->bloom);
  free(A->table);
  free(A);
}

uint64_t ora_addr_count(const ora_addr* A) { return A->n; }
const uint8_t* ora_addr_table(const ora_addr* A) { return A->table; }
const ora_bloom* ora_addr_bloom(const ora_addr* A) { return &A->bloom; }

/* searchbinary keyhunt.cpp:2311-2335 */
int ora_addr_searchbinary(const ora_addr* A, const uint8_t data[20]) {
  int64_t half, min = 0, max = (int64_t)A->n, current = 0;
  int r = 0;
  half = (int64_t)A->n;
  while (!r && half >= 1) {
    half = (max - min) / 2;
    int rcmp = memcmp(data, A->table + 20 * (current + half), 20);
    if (rcmp == 0) {
      r = 1;
    } else {
      if (rcmp < 0) max = max - half;
      else min = min + half;
      current = min;
    }
  }
  return r;
}

/* -------------------------------------------------------------- group scan */
#define AGRP 1024
#define AHALF 512

struct ora_addr_gen {
  ora_point Gn[AHALF];
  ora_point G2n;
  ora_u256 stride;
};

/* init_generator keyhunt.cpp:4386-4399 */
ora_addr_gen* ora_addr_gen_new(const ora_u256* stride) {
  ora_addr_gen* g = (ora_addr_gen*)calloc(1, sizeof(ora_addr_gen));
  g->stride = *stride;
  ora_point G;
  ora_compute_pubkey(&G, stride);
  g->Gn[0] = G;
  ora_double_direct(&g->Gn[1], &G);
  for (int i = 2; i < AHALF; ++i) ora_add_direct(&g->Gn[i], &g->Gn[i - 1], &G);
  ora_double_direct(&g->G2n, &g->Gn[AHALF - 1]);
  return g;
}
void ora_addr_gen_free(ora_addr_gen* g) { free(g); }

void ora_addr_gen_table(const ora_addr_gen* g, uint8_t out[513 * 64]) {
  for (int i = 0; i < 513; ++i) {
    const ora_point* p = i < AHALF ? &g->Gn[i] : &g->G2n;
    ora_u256_to_be(&p->x, out + 64 * i);
    ora_u256_to_be(&p->y, out + 64 * i + 32);
  }
}

/* keyfound = key + t*stride (mod 2^256 in the reference's Int arithmetic; ranges stay < n) */
static void key_at(ora_u256* r, const ora_u256* base, const ora_u256* stride, uint32_t t) {
  ora_u256 m;
  ora_u256_mul64(&m, stride, t);
  ora_u256_add(r, base, &m);
}

/* -e constants, keyhunt.cpp:582-585 */
static const char* LAMBDA_HEX[2] = {"5363ad4cc05c30e0a5261c028812645a122e22ea20816678df02967c1b23bd72",
                                    "ac9c52b33fa3cf1f5ad9e3fd77ed9ba4a880b9fc8ec739c2e0cfc810b51283ce"};
static const char* BETA_HEX[2] = {"7ae96a2b657c07106e64479eac3434e99cf0497512f58995c1396c28719501ee",
                                  "851695d49a83f8ef919bb86153cbcb16630fb68aed0a766a3ec693d68e6afa40"};

/* keyfound.ModMulK1order(&lambda) (IntMod.cpp ModMulK1order): a*b mod n for a, b < 2^256, by shift-and-add */
static void mulmod_n(ora_u256* r, const ora_u256* a0, const ora_u256* b) {
  const ora_u256* n = ora_order();
  ora_u256 a = *a0, acc;
  while (ora_u256_cmp(&a, n) >= 0) ora_u256_sub(&a, &a, n);
  ora_u256_set64(&acc, 0);
  for (int i = 255; i >= 0; --i) {
    uint64_t c = ora_u256_add(&acc, &acc, &acc);
    if (c || ora_u256_cmp(&acc, n) >= 0) ora_u256_sub(&acc, &acc, n);
    if ((b->w[i / 64] >> (i % 64)) & 1) {
      c = ora_u256_add(&acc, &acc, &a);
      if (c || ora_u256_cmp(&acc, n) >= 0) ora_u256_sub(&acc, &acc, n);
    }
  }
  *r = acc;
}

void ora_mulmod_n(ora_u256* r, const ora_u256* a, const ora_u256* b) { mulmod_n(r, a, b); }

void ora_endo_constants(int i, ora_u256* lambda, ora_u256* beta) {
  if (lambda) ora_u256_from_hex(lambda, LAMBDA_HEX[i]);
  if (beta) ora_u256_from_hex(beta, BETA_HEX[i]);
}

static void neg_mod_n(ora_u256* k) {
  /* keyfound.Neg(); keyfound.Add(&order) */
  ora_u256 z;
  ora_u256_set64(&z, 0);
  ora_u256_sub(k, &z, k);
  ora_u256_add(k, k, ora_order());
}

/* One group of thread_process (keyhunt.cpp:2586-2711 + checks 2789-2937), BTC, no endomorphism.
 * key: the group's first key (key_mpz before the j loop).  search: 0 uncompress, 1 compress,
 * 2 both (keyhunt.cpp:59-61), plus ORA_SEARCH_ENDO (4) for -e.  xy (nullable) receives the 1024
 * points x||y BE in t order.  hits receive every bloom hit as (t << 4 | kind): kind = form | e << 2,
 * form 0 = 02-prefix, 1 = 03-prefix, 2 = uncompressed (x, y), 3 = uncompressed (x, -y) (-e only),
 * e = 0 for the point itself, 1 for (beta*x, y) = lambda*P, 2 for (beta^2*x, y) = lambda^2*P (-e only).
 * keys/nkeys the keys that also passed searchbinary (after the reference's sign fix-up). */
void ora_addr_group(const ora_addr* A, const ora_addr_gen* g, const ora_u256* key, int search, uint8_t* xy,
                    uint32_t* hits, uint32_t hcap, uint32_t* nhits, ora_u256* keys, uint32_t kcap,
                    uint32_t* nkeys) {
  static __thread ora_point pts[AGRP];
  static __thread ora_u256 dx[AHALF + 1], subp[AHALF + 1];
  ora_u256 dy, dyn, s, p, inverse, nv, k512;
  ora_point startP, pp, pn;
  int i;
  *nhits = 0;
  *nkeys = 0;
  key_at(&k512, key, &g->stride, AHALF);
  ora_compute_pubkey(&startP, &k512);
  for (i = 0; i < AHALF - 1; ++i) ora_fe_sub(&dx[i], &g->Gn[i].x, &startP.x);
  ora_fe_sub(&dx[i], &g->Gn[i].x, &startP.x);
  ora_fe_sub(&dx[i + 1], &g->G2n.x, &startP.x);
  /* IntGroup::ModInv (IntGroup.cpp:36-58) */
  subp[0] = dx[0];
  for (int k = 1; k < AHALF + 1; ++k) ora_fe_mulK1(&subp[k], &subp[k - 1], &dx[k]);
  inverse = subp[AHALF];
  ora_fe_inv(&inverse, &inverse);
  for (int k = AHALF; k > 0; --k) {
    ora_fe_mulK1(&nv, &subp[k - 1], &inverse);
    ora_fe_mulK1(&inverse, &inverse, &dx[k]);
    dx[k] = nv;
  }
  dx[0] = inverse;
  const int endo = (search & 4) != 0;
  search &= 3;
  const int calc_y = search == 0 || search == 2;
  pts[AHALF] = startP;
  for (i = 0; i < AHALF - 1; ++i) {
    pp = startP;
    pn = startP;
    ora_fe_sub(&dy, &g->Gn[i].y, &pp.y);
    ora_fe_mulK1(&s, &dy, &dx[i]);
    ora_fe_sqrK1(&p, &s);
    ora_fe_neg(&pp.x, &pp.x);
    ora_fe_add(&pp.x, &pp.x, &p);
    ora_fe_sub(&pp.x, &pp.x, &g->Gn[i].x);
    if (calc_y) {
      ora_fe_sub(&pp.y, &g->Gn[i].x, &pp.x);
      ora_fe_mulK1(&pp.y, &pp.y, &s);
      ora_fe_sub(&pp.y, &pp.y, &g->Gn[i].y);
    }
    ora_fe_neg(&dyn, &g->Gn[i].y);
    ora_fe_sub(&dyn, &dyn, &pn.y);
    ora_fe_mulK1(&s, &dyn, &dx[i]);
    ora_fe_sqrK1(&p, &s);
    ora_fe_neg(&pn.x, &pn.x);
    ora_fe_add(&pn.x, &pn.x, &p);
    ora_fe_sub(&pn.x, &pn.x, &g->Gn[i].x);
    if (calc_y) {
      ora_fe_sub(&pn.y, &g->Gn[i].x, &pn.x);
      ora_fe_mulK1(&pn.y, &pn.y, &s);
      ora_fe_add(&pn.y, &pn.y, &g->Gn[i].y);
    }
    pts[AHALF + (i + 1)] = pp;
    pts[AHALF - (i + 1)] = pn;
  }
  pn = startP;
  ora_fe_neg(&dyn, &g->Gn[i].y);
  ora_fe_sub(&dyn, &dyn, &pn.y);
  ora_fe_mulK1(&s, &dyn, &dx[i]);
  ora_fe_sqrK1(&p, &s);
  ora_fe_neg(&pn.x, &pn.x);
  ora_fe_add(&pn.x, &pn.x, &p);
  ora_fe_sub(&pn.x, &pn.x, &g->Gn[i].x);
  if (calc_y) {
    ora_fe_sub(&pn.y, &g->Gn[i].x, &pn.x);
    ora_fe_mulK1(&pn.y, &pn.y, &s);
    ora_fe_add(&pn.y, &pn.y, &g->Gn[i].y);
  }
  pts[0] = pn;
  if (xy)
    for (int t = 0; t < AGRP; ++t) {
      ora_u256_to_be(&pts[t].x, xy + 64 * t);
      ora_u256_to_be(&pts[t].y, xy + 64 * t + 32);
    }
  /* checks, keyhunt.cpp:2789-2937: per point, compressed then uncompressed.  Without -e: 02, 03,
   * uncompressed.  With -e (2716-2763): l = 0..5 the 02/03 hashes of x, beta*x, beta^2*x (ModMulK1 of x
   * with beta / beta2, 2663-2676 and 2685-2711 for pts[512] and pts[0]), l = 6..11 the uncompressed
   * hashes of (x, y), (x, -y), (beta*x, y), (beta*x, -y), (beta^2*x, y), (beta^2*x, -y). */
  ora_u256 beta[2], lambda[2];
  for (int e = 0; e < 2; ++e) ora_endo_constants(e, &lambda[e], &beta[e]);
  for (int t = 0; t < AGRP; ++t) {
    uint8_t h[12][20];
    int kinds[12], nk = 0;
    ora_point ep[3];
    ep[0] = pts[t];
    if (endo)
      for (int e = 1; e < 3; ++e) {
        ora_fe_mulK1(&ep[e].x, &pts[t].x, &beta[e - 1]);
        ep[e].y = pts[t].y;
      }
    const int ne = endo ? 3 : 1;
    if (search == 1 || search == 2) {
      for (int e = 0; e < ne; ++e) {
        ora_x_hash160(0x02, &ep[e].x, h[nk]); kinds[nk++] = 0 | (e << 2);
        ora_x_hash160(0x03, &ep[e].x, h[nk]); kinds[nk++] = 1 | (e << 2);
      }
    }
    if (search == 0 || search == 2) {
      for (int e = 0; e < ne; ++e) {
        ora_pub_hash160(&ep[e], 0, h[nk]); kinds[nk++] = 2 | (e << 2);
        if (endo) {
          ora_point q;
          ora_negation(&q, &ep[e]);       /* secp->Negation (SECP256K1.cpp) */
          ora_pub_hash160(&q, 0, h[nk]); kinds[nk++] = 3 | (e << 2);
        }
      }
    }
    for (int l = 0; l < nk; ++l) {
      if (!ora_bloom_check(&A->bloom, h[l], 20)) continue;
      if (*nhits < hcap) hits[*nhits] = ((uint32_t)t << 4) | (uint32_t)kinds[l];
      ++*nhits;
      if (!ora_addr_searchbinary(A, h[l])) continue;
      ora_u256 kf;
      key_at(&kf, key, &g->stride, (uint32_t)t);
      const int form = kinds[l] & 3, e = kinds[l] >> 2;
      ora_point pub;
      if (!endo) {
        if (form < 2) {
          /* compressed x-only hit: the key or its negation (keyhunt.cpp:2811-2822) */
          uint8_t hh[20];
          ora_compute_pubkey(&pub, &kf);
          ora_pub_hash160(&pub, 1, hh);
          if (memcmp(h[l], hh, 20) != 0) neg_mod_n(&kf);
        }
      } else if (form < 2) {
        /* keyhunt.cpp:2800-2860: the parity of the ORIGINAL key's y (lambda*P has the same y) decides the
         * sign; for beta / beta^2 hits the key is multiplied by lambda / lambda^2 first */
        ora_compute_pubkey(&pub, &kf);
        if (e) mulmod_n(&kf, &kf, &lambda[e - 1]);
        const int odd = (int)(pub.y.w[0] & 1);
        if ((form == 0 && odd) || (form == 1 && !odd)) neg_mod_n(&kf);
      } else {
        /* keyhunt.cpp:2876-2920: lambda^e first, then the uncompressed hash of the key's own public key
         * decides the sign */
        uint8_t hh[20];
        if (e) mulmod_n(&kf, &kf, &lambda[e - 1]);
        ora_compute_pubkey(&pub, &kf);
        ora_pub_hash160(&pub, 0, hh);
        if (memcmp(h[l], hh, 20) != 0) neg_mod_n(&kf);
      }
      if (*nkeys < kcap) keys[*nkeys] = kf;
      ++*nkeys;
    }
  }
}
