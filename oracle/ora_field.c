/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see ora.h).
 * 256-bit integers and the secp256k1 field with the reference's exact semantics
 * (secp256k1/IntMod.cpp, secp256k1/Int.cpp).
 */
#include "ora.h"
#include <string.h>
#include <ctype.h>

typedef unsigned __int128 u128;

static const ora_u256 P = {{0xFFFFFFFEFFFFFC2FULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL}};
/* 2^256 mod p: the fold constant of ModMulK1 (IntMod.cpp:898, 906) */
#define K1FOLD 0x1000003D1ULL

const ora_u256* ora_prime(void) { return &P; }

int ora_u256_cmp(const ora_u256* a, const ora_u256* b) {
  for (int i = 3; i >= 0; --i) {
    if (a->w[i] != b->w[i]) return a->w[i] < b->w[i] ? -1 : 1;
  }
  return 0;
}

uint64_t ora_u256_add(ora_u256* r, const ora_u256* a, const ora_u256* b) {
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c += (u128)a->w[i] + b->w[i];
    r->w[i] = (uint64_t)c;
    c >>= 64;
  }
  return (uint64_t)c;
}

uint64_t ora_u256_sub(ora_u256* r, const ora_u256* a, const ora_u256* b) {
  uint64_t borrow = 0;
  for (int i = 0; i < 4; ++i) {
    uint64_t ai = a->w[i], bi = b->w[i];
    uint64_t d = ai - bi - borrow;
    borrow = (ai < bi) || (ai == bi && borrow) ? 1 : 0;
    r->w[i] = d;
  }
  return borrow;
}

void ora_u256_set64(ora_u256* r, uint64_t v) {
  r->w[0] = v; r->w[1] = r->w[2] = r->w[3] = 0;
}

int ora_u256_is_zero(const ora_u256* a) {
  return (a->w[0] | a->w[1] | a->w[2] | a->w[3]) == 0;
}

void ora_u256_mul64(ora_u256* r, const ora_u256* a, uint64_t m) {
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c += (u128)a->w[i] * m;
    r->w[i] = (uint64_t)c;
    c >>= 64;
  }
}

/* Int::SetBase16 (Int.cpp SetBaseN): accepts upper/lower case hex digits. */
int ora_u256_from_hex(ora_u256* r, const char* hex) {
  ora_u256 v = {{0, 0, 0, 0}};
  if (hex[0] == '0' && (hex[1] == 'x' || hex[1] == 'X')) hex += 2;
  for (const char* p = hex; *p; ++p) {
    int d;
    if (*p >= '0' && *p <= '9') d = *p - '0';
    else if (*p >= 'a' && *p <= 'f') d = *p - 'a' + 10;
    else if (*p >= 'A' && *p <= 'F') d = *p - 'A' + 10;
    else return -1;
    v.w[3] = (v.w[3] << 4) | (v.w[2] >> 60);
    v.w[2] = (v.w[2] << 4) | (v.w[1] >> 60);
    v.w[1] = (v.w[1] << 4) | (v.w[0] >> 60);
    v.w[0] = (v.w[0] << 4) | (uint64_t)d;
  }
  *r = v;
  return 0;
}

/* Int::GetBase16 (Int.cpp:953-957, 1019-1057): lowercase, no leading zeros, "0" for zero. */
void ora_u256_to_hex(const ora_u256* a, char out[65]) {
  static const char* dg = "0123456789abcdef";
  char tmp[65];
  int n = 0;
  for (int i = 63; i >= 0; --i) {
    int nib = (int)((a->w[i / 16] >> ((i % 16) * 4)) & 15);
    if (n == 0 && nib == 0) continue;
    tmp[n++] = dg[nib];
  }
  if (n == 0) tmp[n++] = '0';
  tmp[n] = 0;
  memcpy(out, tmp, (size_t)n + 1);
}

/* Int::Get32Bytes (Int.cpp:308-316): big-endian 32 bytes. */
void ora_u256_to_be(const ora_u256* a, uint8_t out[32]) {
  for (int i = 0; i < 32; ++i) out[i] = (uint8_t)(a->w[3 - i / 8] >> (56 - 8 * (i % 8)));
}

void ora_u256_from_be(ora_u256* r, const uint8_t in[32]) {
  for (int i = 0; i < 4; ++i) {
    uint64_t v = 0;
    for (int j = 0; j < 8; ++j) v = (v << 8) | in[(3 - i) * 8 + j];
    r->w[i] = v;
  }
}

/* Int::ModAdd(Int*,Int*) IntMod.cpp:51-57: add, then subtract P when the sum is >= P. */
void ora_fe_add(ora_u256* r, const ora_u256* a, const ora_u256* b) {
  ora_u256 s;
  uint64_t c = ora_u256_add(&s, a, b);
  if (c || ora_u256_cmp(&s, &P) >= 0) ora_u256_sub(&s, &s, &P);
  *r = s;
}

/* Int::ModSub(Int*,Int*) IntMod.cpp:97-101: subtract, add P when negative. */
void ora_fe_sub(ora_u256* r, const ora_u256* a, const ora_u256* b) {
  ora_u256 d;
  if (ora_u256_sub(&d, a, b)) ora_u256_add(&d, &d, &P);
  *r = d;
}

/* Int::ModNeg IntMod.cpp:105-108: P - a, NOT reduced (ModNeg(0) == P). */
void ora_fe_neg(ora_u256* r, const ora_u256* a) {
  ora_u256 d;
  ora_u256_sub(&d, &P, a);
  *r = d;
}

/* Int::ModMulK1 IntMod.cpp:855-915.  Exact 512-bit product, then two folds by 2^256 = 0x1000003D1
 * (mod p).  The final carry is dropped and no final subtraction of P is performed — the result is
 * < 2^256, equal to the canonical value except with probability < 2^-190 per call.  Restated
 * literally so the oracle reproduces the reference even in that case. */
void ora_fe_mulK1(ora_u256* r, const ora_u256* a, const ora_u256* b) {
  uint64_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) {
      c += (u128)a->w[j] * b->w[i] + w[i + j];
      w[i + j] = (uint64_t)c;
      c >>= 64;
    }
    w[i + 4] = (uint64_t)c;
  }
  /* 512 -> 320: t = hi256 * 0x1000003D1 (IntMod.cpp:898) */
  uint64_t t[5];
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c += (u128)w[4 + i] * K1FOLD;
    t[i] = (uint64_t)c;
    c >>= 64;
  }
  t[4] = (uint64_t)c;
  c = 0;
  for (int i = 0; i < 4; ++i) {
    c += (u128)w[i] + t[i];
    w[i] = (uint64_t)c;
    c >>= 64;
  }
  /* 320 -> 256 (IntMod.cpp:906-913) */
  u128 u = (u128)(t[4] + (uint64_t)c) * K1FOLD;
  u128 s = (u128)w[0] + (uint64_t)u;
  r->w[0] = (uint64_t)s;
  s = (u128)w[1] + (uint64_t)(u >> 64) + (uint64_t)(s >> 64);
  r->w[1] = (uint64_t)s;
  s = (u128)w[2] + (uint64_t)(s >> 64);
  r->w[2] = (uint64_t)s;
  s = (u128)w[3] + (uint64_t)(s >> 64);
  r->w[3] = (uint64_t)s;   /* carry dropped: bits64[4] = 0 */
}

/* Int::ModSquareK1 IntMod.cpp:977-1093 computes the same exact 512-bit square and the identical
 * two-fold reduction, so it equals ModMulK1(a,a) bit for bit. */
void ora_fe_sqrK1(ora_u256* r, const ora_u256* a) { ora_fe_mulK1(r, a, a); }

/* Canonical a*b mod p (what Montgomery Int::ModMul returns, IntMod.cpp:655+): the same two folds
 * as ModMulK1 but with the final carry folded back and a final conditional subtraction. */
void ora_fe_mul_exact(ora_u256* r, const ora_u256* a, const ora_u256* b) {
  uint64_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) {
      c += (u128)a->w[j] * b->w[i] + w[i + j];
      w[i + j] = (uint64_t)c;
      c >>= 64;
    }
    w[i + 4] = (uint64_t)c;
  }
  uint64_t t[5];
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c += (u128)w[4 + i] * K1FOLD;
    t[i] = (uint64_t)c;
    c >>= 64;
  }
  t[4] = (uint64_t)c;
  c = 0;
  for (int i = 0; i < 4; ++i) {
    c += (u128)w[i] + t[i];
    w[i] = (uint64_t)c;
    c >>= 64;
  }
  u128 u = (u128)(t[4] + (uint64_t)c) * K1FOLD;
  ora_u256 v;
  c = (u128)w[0] + (uint64_t)u;           v.w[0] = (uint64_t)c; c >>= 64;
  c += (u128)w[1] + (uint64_t)(u >> 64);  v.w[1] = (uint64_t)c; c >>= 64;
  c += w[2];                               v.w[2] = (uint64_t)c; c >>= 64;
  c += w[3];                               v.w[3] = (uint64_t)c; c >>= 64;
  if (c) {   /* value = v + 2^256 = v + 0x1000003D1 (mod p); v is tiny here */
    ora_u256 k = {{K1FOLD, 0, 0, 0}};
    ora_u256_add(&v, &v, &k);
  }
  while (ora_u256_cmp(&v, &P) >= 0) ora_u256_sub(&v, &v, &P);
  *r = v;
}

static void sqr_n(ora_u256* r, const ora_u256* a, int n) {
  ora_u256 t = *a;
  for (int i = 0; i < n; ++i) ora_fe_mul_exact(&t, &t, &t);
  *r = t;
}

void ora_fe_pow(ora_u256* r, const ora_u256* a, const ora_u256* e) {
  ora_u256 res, base = *a;
  ora_u256_set64(&res, 1);
  while (ora_u256_cmp(&base, &P) >= 0) ora_u256_sub(&base, &base, &P);
  for (int i = 255; i >= 0; --i) {
    ora_fe_mul_exact(&res, &res, &res);
    if ((e->w[i / 64] >> (i % 64)) & 1) ora_fe_mul_exact(&res, &res, &base);
  }
  *r = res;
}

/* Int::ModInv (DRS62, IntMod.cpp:382-511): canonical inverse of a mod p, 0 when a == 0 mod p
 * (the CLEAR() at :497-500).  Restated as a^(p-2) (Fermat) over the standard secp256k1 addition
 * chain (blocks of 1s of lengths 223, 22, 2, 1 in p-2); same canonical value. */
void ora_fe_inv(ora_u256* r, const ora_u256* a0) {
  ora_u256 a = *a0, x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223, t;
  while (ora_u256_cmp(&a, &P) >= 0) ora_u256_sub(&a, &a, &P);
  sqr_n(&x2, &a, 1);    ora_fe_mul_exact(&x2, &x2, &a);
  sqr_n(&x3, &x2, 1);   ora_fe_mul_exact(&x3, &x3, &a);
  sqr_n(&x6, &x3, 3);   ora_fe_mul_exact(&x6, &x6, &x3);
  sqr_n(&x9, &x6, 3);   ora_fe_mul_exact(&x9, &x9, &x3);
  sqr_n(&x11, &x9, 2);  ora_fe_mul_exact(&x11, &x11, &x2);
  sqr_n(&x22, &x11, 11); ora_fe_mul_exact(&x22, &x22, &x11);
  sqr_n(&x44, &x22, 22); ora_fe_mul_exact(&x44, &x44, &x22);
  sqr_n(&x88, &x44, 44); ora_fe_mul_exact(&x88, &x88, &x44);
  sqr_n(&x176, &x88, 88); ora_fe_mul_exact(&x176, &x176, &x88);
  sqr_n(&x220, &x176, 44); ora_fe_mul_exact(&x220, &x220, &x44);
  sqr_n(&x223, &x220, 3); ora_fe_mul_exact(&x223, &x223, &x3);
  sqr_n(&t, &x223, 23); ora_fe_mul_exact(&t, &t, &x22);
  sqr_n(&t, &t, 5);     ora_fe_mul_exact(&t, &t, &a);
  sqr_n(&t, &t, 3);     ora_fe_mul_exact(&t, &t, &x2);
  sqr_n(&t, &t, 2);     ora_fe_mul_exact(&t, &t, &a);
  *r = t;
}

/* Int::HasSqrt IntMod.cpp:563-574: Euler's criterion a^((p-1)/2) == 1. */
int ora_fe_has_sqrt(const ora_u256* a) {
  ora_u256 e = P, one, t;
  ora_u256_set64(&one, 1);
  ora_u256_sub(&e, &e, &one);
  /* shift right 1 */
  for (int i = 0; i < 4; ++i) e.w[i] = (e.w[i] >> 1) | (i < 3 ? (e.w[i + 1] << 63) : 0);
  ora_fe_pow(&t, a, &e);
  return ora_u256_cmp(&t, &one) == 0;
}

/* Int::ModSqrt IntMod.cpp:578-652, p = 3 mod 4 branch (:590-596): a^((p+1)/4); CLEAR when no root. */
void ora_fe_sqrt(ora_u256* r, const ora_u256* a) {
  if (!ora_fe_has_sqrt(a)) { ora_u256_set64(r, 0); return; }
  ora_u256 e = P, one;
  ora_u256_set64(&one, 1);
  ora_u256_add(&e, &e, &one);   /* p+1 < 2^256 */
  for (int i = 0; i < 4; ++i) e.w[i] = (e.w[i] >> 2) | (i < 3 ? (e.w[i + 1] << 62) : 0);
  ora_fe_pow(r, a, &e);
}
