// Host secp256k1 field on 4 x 64-bit limbs (unsigned __int128 products): the CPU-side twin of
// device/fe.hpp for setup and candidate confirmation, where x86-64's 64x64->128 multiplier makes
// it ~5x faster than the 8 x 32-bit GPU layout.  Canonical values in [0, p), same results as the
// reference's IntMod.cpp (see fe.hpp).
#pragma once
#include <stdint.h>
#include <string.h>

namespace khb {

struct Fh {
  uint64_t w[4];
};

typedef unsigned __int128 fh_u128;
static const uint64_t kFhK = 0x1000003D1ull;   // 2^256 mod p

static inline bool fe_is_zero(const Fh& a) { return (a.w[0] | a.w[1] | a.w[2] | a.w[3]) == 0; }
static inline bool fe_eq(const Fh& a, const Fh& b) {
  return ((a.w[0] ^ b.w[0]) | (a.w[1] ^ b.w[1]) | (a.w[2] ^ b.w[2]) | (a.w[3] ^ b.w[3])) == 0;
}
static inline Fh fh_one() { return Fh{{1, 0, 0, 0}}; }
static inline Fh fh_small(uint64_t v) { return Fh{{v, 0, 0, 0}}; }

// t (< 2^256 + 2^256) given as t + carry*2^256: canonicalise.
static inline void fh_final(Fh& r, uint64_t t0, uint64_t t1, uint64_t t2, uint64_t t3, uint64_t carry) {
  // u = t + K; if carry or u overflows, result = u mod 2^256 (= t - p), else t
  fh_u128 e = (fh_u128)t0 + kFhK;
  uint64_t u0 = (uint64_t)e;
  e = (e >> 64) + t1;
  uint64_t u1 = (uint64_t)e;
  e = (e >> 64) + t2;
  uint64_t u2 = (uint64_t)e;
  e = (e >> 64) + t3;
  uint64_t u3 = (uint64_t)e;
  const bool sel = carry || (uint64_t)(e >> 64);
  r.w[0] = sel ? u0 : t0;
  r.w[1] = sel ? u1 : t1;
  r.w[2] = sel ? u2 : t2;
  r.w[3] = sel ? u3 : t3;
}

static inline void fe_add(Fh& r, const Fh& a, const Fh& b) {
  fh_u128 c = (fh_u128)a.w[0] + b.w[0];
  uint64_t t0 = (uint64_t)c;
  c = (c >> 64) + a.w[1] + b.w[1];
  uint64_t t1 = (uint64_t)c;
  c = (c >> 64) + a.w[2] + b.w[2];
  uint64_t t2 = (uint64_t)c;
  c = (c >> 64) + a.w[3] + b.w[3];
  uint64_t t3 = (uint64_t)c;
  fh_final(r, t0, t1, t2, t3, (uint64_t)(c >> 64));
}

static inline void fe_sub(Fh& r, const Fh& a, const Fh& b) {
  uint64_t br = 0, t[4];
  for (int i = 0; i < 4; ++i) {
    fh_u128 d = (fh_u128)a.w[i] - b.w[i] - br;
    t[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  // borrow: add p == subtract K mod 2^256
  uint64_t m = br ? kFhK : 0;
  fh_u128 d = (fh_u128)t[0] - m;
  r.w[0] = (uint64_t)d;
  uint64_t b2 = (uint64_t)(d >> 64) & 1;
  for (int i = 1; i < 4; ++i) {
    d = (fh_u128)t[i] - b2;
    r.w[i] = (uint64_t)d;
    b2 = (uint64_t)(d >> 64) & 1;
  }
}

static inline void fh_reduce(Fh& r, const uint64_t w[8]) {
  fh_u128 c = 0;
  uint64_t t[4];
  for (int i = 0; i < 4; ++i) {
    c += (fh_u128)w[4 + i] * kFhK + w[i];
    t[i] = (uint64_t)c;
    c >>= 64;
  }
  // c < 2^34: fold again
  c = (fh_u128)(uint64_t)c * kFhK + t[0];
  t[0] = (uint64_t)c;
  c >>= 64;
  for (int i = 1; i < 4; ++i) {
    c += t[i];
    t[i] = (uint64_t)c;
    c >>= 64;
  }
  fh_final(r, t[0], t[1], t[2], t[3], (uint64_t)c);
}

static inline void fe_mul(Fh& r, const Fh& a, const Fh& b) {
  uint64_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) {
    fh_u128 c = 0;
    for (int j = 0; j < 4; ++j) {
      c += (fh_u128)a.w[j] * b.w[i] + w[i + j];
      w[i + j] = (uint64_t)c;
      c >>= 64;
    }
    w[i + 4] = (uint64_t)c;
  }
  fh_reduce(r, w);
}

static inline void fe_sqr(Fh& r, const Fh& a) {
  // cross products once, doubled, plus squares
  uint64_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 3; ++i) {
    fh_u128 c = 0;
    for (int j = i + 1; j < 4; ++j) {
      c += (fh_u128)a.w[i] * a.w[j] + w[i + j];
      w[i + j] = (uint64_t)c;
      c >>= 64;
    }
    w[i + 4] = (uint64_t)c;
  }
  w[7] = w[6] >> 63;
  for (int k = 6; k > 0; --k) w[k] = (w[k] << 1) | (w[k - 1] >> 63);
  w[0] <<= 1;
  fh_u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c += (fh_u128)a.w[i] * a.w[i] + w[2 * i];
    w[2 * i] = (uint64_t)c;
    c >>= 64;
    c += w[2 * i + 1];
    w[2 * i + 1] = (uint64_t)c;
    c >>= 64;
  }
  fh_reduce(r, w);
}

static inline void fh_sqr_n(Fh& r, const Fh& a, int n) {
  r = a;
  for (int i = 0; i < n; ++i) fe_sqr(r, r);
}

// a^(p-2), standard chain (see fe.hpp fe_inv); inv(0) == 0.
static inline void fe_inv(Fh& r, const Fh& a) {
  Fh x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223, t;
  fe_sqr(x2, a);            fe_mul(x2, x2, a);
  fe_sqr(x3, x2);           fe_mul(x3, x3, a);
  fh_sqr_n(x6, x3, 3);      fe_mul(x6, x6, x3);
  fh_sqr_n(x9, x6, 3);      fe_mul(x9, x9, x3);
  fh_sqr_n(x11, x9, 2);     fe_mul(x11, x11, x2);
  fh_sqr_n(x22, x11, 11);   fe_mul(x22, x22, x11);
  fh_sqr_n(x44, x22, 22);   fe_mul(x44, x44, x22);
  fh_sqr_n(x88, x44, 44);   fe_mul(x88, x88, x44);
  fh_sqr_n(x176, x88, 88);  fe_mul(x176, x176, x88);
  fh_sqr_n(x220, x176, 44); fe_mul(x220, x220, x44);
  fh_sqr_n(x223, x220, 3);  fe_mul(x223, x223, x3);
  fh_sqr_n(t, x223, 23);    fe_mul(t, t, x22);
  fh_sqr_n(t, t, 5);        fe_mul(t, t, a);
  fh_sqr_n(t, t, 3);        fe_mul(t, t, x2);
  fh_sqr_n(t, t, 2);        fe_mul(r, t, a);
}

static inline void fe_from_be(Fh& r, const uint8_t* b) {
  for (int i = 0; i < 4; ++i) {
    uint64_t v = 0;
    for (int j = 0; j < 8; ++j) v = (v << 8) | b[(3 - i) * 8 + j];
    r.w[i] = v;
  }
}
static inline void fe_to_be(uint8_t* b, const Fh& a) {
  for (int i = 0; i < 32; ++i) b[i] = (uint8_t)(a.w[3 - i / 8] >> (56 - 8 * (i % 8)));
}

}  // namespace khb
