// secp256k1 base-field arithmetic on 8 x 32-bit limbs, written for the CDNA4 VALU.
//
// Every value is canonical (in [0, p)), so every result equals the canonical value the reference
// computes with secp256k1/IntMod.cpp (ModAdd :51-57, ModSub :97-101, ModMulK1 :855-915,
// ModSquareK1 :977-1093, ModInv :112-513).  The reference's ModMulK1 drops a final carry and skips
// the last subtraction of p; its result differs from canonical only with probability < 2^-190
// per call ("Deviations").
//
// Limbs are little-endian; 32x32->64 products map onto v_mad_u64_u32, which measured at ~0.87x
// the issue rate of a plain 32-bit add on gfx950 (tools/microbench/intops.hip), so a schoolbook
// 8x8 product is the right shape here — no Karatsuba, no MFMA.
//
// The same source compiles for the host (g++/hipcc host pass) so the arithmetic is unit-tested on
// the CPU against the oracle before it runs on the GPU.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define KHB_HD __host__ __device__ __forceinline__
#else
#define KHB_HD static inline
#endif

namespace khb {

struct Fe {
  uint32_t v[8];
};

// p = 2^256 - 0x1000003D1
#define KHB_P0 0xFFFFFC2Fu
#define KHB_P1 0xFFFFFFFEu

KHB_HD void fe_set(Fe& r, const Fe& a) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = a.v[i];
}

KHB_HD bool fe_is_zero(const Fe& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a.v[i];
  return o == 0;
}

KHB_HD bool fe_eq(const Fe& a, const Fe& b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a.v[i] ^ b.v[i];
  return o == 0;
}

// r = (u + 0x1000003D1) if sel, else u — the "subtract p" step written as an add mod 2^256.
// Returns the carry out of the add.
KHB_HD uint32_t fe_add_k1fold(uint32_t w[8], const uint32_t u[8]) {
  uint64_t c = (uint64_t)u[0] + 0x3D1u;
  w[0] = (uint32_t)c;
  c = (uint64_t)u[1] + 1u + (c >> 32);
  w[1] = (uint32_t)c;
#pragma unroll
  for (int i = 2; i < 8; ++i) {
    c = (uint64_t)u[i] + (c >> 32);
    w[i] = (uint32_t)c;
  }
  return (uint32_t)(c >> 32);
}

// a + b mod p (canonical inputs -> canonical output)
KHB_HD void fe_add(Fe& r, const Fe& a, const Fe& b) {
  uint32_t s[8], w[8];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c = (uint64_t)a.v[i] + b.v[i] + (c >> 32);
    s[i] = (uint32_t)c;
  }
  uint32_t cs = (uint32_t)(c >> 32);
  uint32_t cw = fe_add_k1fold(w, s);
  bool sel = (cs | cw) != 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = sel ? w[i] : s[i];
}

// a - b mod p
KHB_HD void fe_sub(Fe& r, const Fe& a, const Fe& b) {
  uint32_t d[8];
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c = (int64_t)a.v[i] - (int64_t)b.v[i] + (c >> 32);
    d[i] = (uint32_t)c;
  }
  // borrow: add p = 2^256 - 0x1000003D1, i.e. subtract 0x1000003D1 mod 2^256
  uint32_t m = (c < 0) ? 0xFFFFFFFFu : 0u;
  int64_t e = (int64_t)d[0] - (int64_t)(0x3D1u & m);
  r.v[0] = (uint32_t)e;
  e = (int64_t)d[1] - (int64_t)(1u & m) + (e >> 32);
  r.v[1] = (uint32_t)e;
#pragma unroll
  for (int i = 2; i < 8; ++i) {
    e = (int64_t)d[i] + (e >> 32);
    r.v[i] = (uint32_t)e;
  }
}

// Reduce a 512-bit product t[0..15] mod p: two folds by 2^256 = 2^32 + 977, then one
// conditional subtraction.  Output canonical.
KHB_HD void fe_reduce512(Fe& r, const uint32_t t[16]) {
  uint32_t u[8];
  // u = L + H*977  (top carry < 2^11)
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c = (uint64_t)t[8 + i] * 977u + t[i] + (c >> 32);
    u[i] = (uint32_t)c;
  }
  uint64_t top = c >> 32;
  // u += H << 32
  c = 0;
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    c = (uint64_t)u[i] + t[8 + i - 1] + (c >> 32);
    u[i] = (uint32_t)c;
  }
  top += (uint64_t)t[15] + (c >> 32);   // < 2^33
  // second fold: top * (2^32 + 977)
  c = (uint64_t)u[0] + top * 977u;
  u[0] = (uint32_t)c;
  c = (uint64_t)u[1] + top + (c >> 32);
  u[1] = (uint32_t)c;
  c >>= 32;
#pragma unroll
  for (int i = 2; i < 8; ++i) {
    c += u[i];
    u[i] = (uint32_t)c;
    c >>= 32;
  }
  // value = u + c*2^256 (c in {0,1}); canonical = u + 0x1000003D1 (mod 2^256) when c or u >= p
  uint32_t w[8];
  uint32_t cw = fe_add_k1fold(w, u);
  bool sel = ((uint32_t)c | cw) != 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = sel ? w[i] : u[i];
}

KHB_HD void fe_mul(Fe& r, const Fe& a, const Fe& b) {
  uint32_t t[16];
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    c = (uint64_t)a.v[0] * b.v[j] + (c >> 32);
    t[j] = (uint32_t)c;
  }
  t[8] = (uint32_t)(c >> 32);
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      c = (uint64_t)a.v[i] * b.v[j] + t[i + j] + (c >> 32);
      t[i + j] = (uint32_t)c;
    }
    t[i + 8] = (uint32_t)(c >> 32);
  }
  fe_reduce512(r, t);
}

KHB_HD void fe_sqr(Fe& r, const Fe& a) {
  uint32_t t[16];
  uint64_t c = 0;
  // cross products a_i*a_j, i<j
  t[0] = 0;
#pragma unroll
  for (int j = 1; j < 8; ++j) {
    c = (uint64_t)a.v[0] * a.v[j] + (c >> 32);
    t[j] = (uint32_t)c;
  }
  t[8] = (uint32_t)(c >> 32);
#pragma unroll
  for (int i = 1; i < 7; ++i) {
    c = 0;
#pragma unroll
    for (int j = i + 1; j < 8; ++j) {
      c = (uint64_t)a.v[i] * a.v[j] + t[i + j] + (c >> 32);
      t[i + j] = (uint32_t)c;
    }
    t[i + 8] = (uint32_t)(c >> 32);
  }
  // t[1..14] holds the cross sum; double it
  t[15] = t[14] >> 31;
#pragma unroll
  for (int k = 14; k > 1; --k) t[k] = (t[k] << 1) | (t[k - 1] >> 31);
  t[1] = t[1] << 1;
  // add the squares a_i^2 at limb 2i
  c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c = (uint64_t)a.v[i] * a.v[i] + t[2 * i] + (c >> 32);
    t[2 * i] = (uint32_t)c;
    c = (uint64_t)t[2 * i + 1] + (c >> 32);
    t[2 * i + 1] = (uint32_t)c;
  }
  fe_reduce512(r, t);
}

KHB_HD void fe_sqr_n(Fe& r, const Fe& a, int n) {
  fe_set(r, a);
  for (int i = 0; i < n; ++i) fe_sqr(r, r);
}

// a^(p-2) over the standard secp256k1 chain (blocks of 1s of lengths 223, 22, 2, 1 in p-2):
// 255 squarings + 15 multiplications.  inv(0) == 0, matching Int::ModInv's CLEAR().
KHB_HD void fe_inv(Fe& r, const Fe& a) {
  Fe x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223, t;
  fe_sqr(x2, a);            fe_mul(x2, x2, a);
  fe_sqr(x3, x2);           fe_mul(x3, x3, a);
  fe_sqr_n(x6, x3, 3);      fe_mul(x6, x6, x3);
  fe_sqr_n(x9, x6, 3);      fe_mul(x9, x9, x3);
  fe_sqr_n(x11, x9, 2);     fe_mul(x11, x11, x2);
  fe_sqr_n(x22, x11, 11);   fe_mul(x22, x22, x11);
  fe_sqr_n(x44, x22, 22);   fe_mul(x44, x44, x22);
  fe_sqr_n(x88, x44, 44);   fe_mul(x88, x88, x44);
  fe_sqr_n(x176, x88, 88);  fe_mul(x176, x176, x88);
  fe_sqr_n(x220, x176, 44); fe_mul(x220, x220, x44);
  fe_sqr_n(x223, x220, 3);  fe_mul(x223, x223, x3);
  fe_sqr_n(t, x223, 23);    fe_mul(t, t, x22);
  fe_sqr_n(t, t, 5);        fe_mul(t, t, a);
  fe_sqr_n(t, t, 3);        fe_mul(t, t, x2);
  fe_sqr_n(t, t, 2);        fe_mul(r, t, a);
}

// Big-endian 32 bytes (Int::Get32Bytes, secp256k1/Int.cpp:308-316) <-> limbs.
KHB_HD void fe_from_be(Fe& r, const uint8_t* b) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint8_t* q = b + 28 - 4 * i;
    r.v[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}
KHB_HD void fe_to_be(uint8_t* b, const Fe& a) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint8_t* q = b + 28 - 4 * i;
    q[0] = (uint8_t)(a.v[i] >> 24); q[1] = (uint8_t)(a.v[i] >> 16);
    q[2] = (uint8_t)(a.v[i] >> 8);  q[3] = (uint8_t)a.v[i];
  }
}

}  // namespace khb
