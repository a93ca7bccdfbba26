// secp256k1 base field in 9 unsaturated 29-bit limbs, for the -m bsgs walk on gfx950.
//
// Why: the 8 x 32-bit product (fe_asm.hpp) spends one carry-counting add per partial product, a
// column fold and two reduction carry chains on top of its 64 v_mad_u64_u32 — about 200 VALU
// instructions per multiply.  With 29-bit limbs a column of up to nine partial products stays below
// 2^64, so each partial product is exactly one v_mad_u64_u32 (its 64-bit addend is the column) and
// carries are resolved once per product, by 64-bit shifts, when the columns are folded and
// normalised.  A multiply is 81 + 32 + 27 + ~9 instructions, a squaring 45 + 9 + 68.
//
// Value contract:
//   * an F9 holds x = sum v[i] 2^(29 i), congruent to the field element, not reduced;
//   * "strict" limbs: v[i] < 2^29 + 2^20 (every f9_mul / f9_sqr result; f9_from_fe output < 2^29);
//   * f9_mul / f9_sqr accept limbs < 2^30.4 on both operands (a column of nine products then stays
//     below 9 * 2^60.8 < 2^64 and the folds below add < 2^51), so the sum of two strict values
//     (f9_add) is a valid operand; more generally any operands whose limb bounds multiply to less
//     than 2^60.8 (e.g. < 2^31.6 against a strict product result);
//   * f9_gate_words returns the low 64 bits of the canonical value (x mod p) for limbs < 2^30.6,
//     and flags the rare inputs (probability ~2^-22) for which that fast path is not exact;
//   * f9_to_fe returns the canonical 8 x 32 form of any value with limbs < 2^31.
//
// Reduction: 2^261 = 2^5 * 2^256 == 2^5 (2^32 + 977) = 2^37 + 31264 (mod p), and 2^37 = 2^29 * 2^8,
// so a value v at limb 9 + j equals v * 31264 at limb j plus v * 256 at limb j + 1.
#pragma once
#include <stdint.h>

#include "fe.hpp"

namespace khb {

struct F9 {
  uint32_t v[9];
};

#define KHB_M29 0x1FFFFFFFu

// x = a + b, limb-wise (no carries): for strict a, b the limbs stay < 2^30 + 2^21.
KHB_HD void f9_add(F9& r, const F9& a, const F9& b) {
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = a.v[i] + b.v[i];
}

// x = a + 2p - b, limb-wise with 2p written so that every limb is >= 2^29 (>= 2^24 for limb 8):
// for strict b (limbs < 2^29, limb 8 < 2^24: canonical values from f9_from_fe) no limb borrows, and
// the limbs of the result stay < a + 2^30.
KHB_HD void f9_add_neg(F9& r, const F9& a, const F9& b) {
  const uint32_t K[9] = {0x3ffff85eu, 0x3fffffeeu, 0x3ffffffeu, 0x3ffffffeu, 0x3ffffffeu,
                         0x3ffffffeu, 0x3ffffffeu, 0x3ffffffeu, 0x1fffffeu};
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = a.v[i] + (K[i] - b.v[i]);
}

// A constant the compiler cannot see through (an SGPR written by s_mov_b32): products by it stay
// one v_mad_u64_u32 each, where the known powers of two 256 / 2048 would become 64-bit shifts of
// zero-extended operands (two moves and a shift more per fold).  Inline-asm multiplies would do the
// same at the price of an s_nop after each (the compiler pads asm for the VCC / SGPR hazards).
KHB_HD uint32_t f9_k(uint32_t k) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("s_mov_b32 %0, %1" : "=s"(r) : "i"(k));
  return r;
#else
  return k;
#endif
}

// acc += a * b
KHB_HD void f9_mad(uint64_t& acc, uint32_t a, uint32_t b) { acc += (uint64_t)a * b; }

// Scheduling fence (KHB_F9_FENCE): keeps the compiler from hoisting every partial product of a
// multiply to its start, which would hold all 17 columns live at once (register pressure at 4
// waves/SIMD); the products of one column still issue back to back.
#ifndef KHB_F9_FENCE
#define KHB_F9_FENCE 1
#endif
KHB_HD void f9_fence() {
#if defined(__HIP_DEVICE_COMPILE__) && KHB_F9_FENCE
  __builtin_amdgcn_sched_barrier(0);
#endif
}

// ---- product and square: high columns first, carried by their high words; low columns seeded ----
// Column k of a*b is c_k = sum a_i b_(k-i).  With limb bounds A, B (A * B < 2^60.8) a column of up to
// nine products stays below 2^64.  The reduction uses 2^261 == 2^37 + 31264 (mod p): a value at limb
// 9 + m equals itself * 31264 at limb m plus * 256 at limb m + 1.
//  1. high columns k = 9..16, each seeded with 8 * hi32 of the previous one (hi32 of column k sits at
//     limb k + 1, times 2^3): only the low words lo_k = lo32(c'_k) remain, plus h17 = hi32(c'_16);
//  2. low columns j = 0..8 in order, each seeded with the carry (t >> 29) of the previous one and
//     folding lo_(9+j) * 31264 and lo_(8+j) * 256 (and h17 * 8 * 31264 into column 8) in the same
//     v_mad_u64_u32 chain: no 64-bit additions, one shift and one mask per limb;
//  3. the value at limb 9, t9 = (t >> 29) + h17 * 8 * 256 (< 2^41), folded into limbs 0..2.
// Every partial product, seed and fold is one v_mad_u64_u32 (multipliers that are powers of two come
// from SGPRs, f9_k, so they stay mads).  Output: limbs < 2^29, limb 2 < 2^29 + 2^21 ("strict").
KHB_HD void f9_final(F9& r, uint64_t t9, uint32_t k256) {
  const uint32_t e9 = (uint32_t)t9 & KHB_M29, e10 = (uint32_t)(t9 >> 29);      // e10 < 2^12
  uint64_t t0 = r.v[0];
  f9_mad(t0, e9, 31264u);                                                   // < 2^45
  uint64_t t1 = (uint64_t)(r.v[1] + (uint32_t)(t0 >> 29));                  // < 2^29 + 2^16
  f9_mad(t1, e9, k256);
  f9_mad(t1, e10, 31264u);                                                  // < 2^38
  r.v[0] = (uint32_t)t0 & KHB_M29;
  r.v[1] = (uint32_t)t1 & KHB_M29;
  r.v[2] += (uint32_t)(t1 >> 29) + e10 * 256u;                              // < 2^9 + 2^20
}

KHB_HD void f9_mul(F9& r, const F9& a_, const F9& b_) {
  const F9 a = a_, b = b_;            // r may alias a or b (limbs are written as the low columns complete)
  const uint32_t k8 = f9_k(8u), k256 = f9_k(256u), k2048 = f9_k(2048u);
  uint32_t lo[8], hi = 0;
#pragma unroll
  for (int k = 9; k < 17; ++k) {
    f9_fence();
    uint64_t s = 0;
    if (k > 9) s = (uint64_t)hi * k8;
#pragma unroll
    for (int i = k - 8; i <= 8; ++i) s += (uint64_t)a.v[i] * b.v[k - i];
    lo[k - 9] = (uint32_t)s;
    hi = (uint32_t)(s >> 32);
  }
  uint64_t t = 0;
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    f9_fence();
    uint64_t s = j ? (t >> 29) : 0;
#pragma unroll
    for (int i = 0; i <= j; ++i) s += (uint64_t)a.v[i] * b.v[j - i];
    if (j < 8) s += (uint64_t)lo[j] * 31264u;
    if (j > 0) s += (uint64_t)lo[j - 1] * k256;
    if (j == 8) s += (uint64_t)hi * 250112u;                                  // h17 * 8 * 31264
    r.v[j] = (uint32_t)s & KHB_M29;
    t = s;
  }
  f9_final(r, (t >> 29) + (uint64_t)hi * k2048, k256);                       // + h17 * 8 * 256
}

// a^2: 45 products (cross terms against the doubled operand), the same columns and reduction.
KHB_HD void f9_sqr(F9& r, const F9& a_) {
  const F9 a = a_;                    // r may alias a
  const uint32_t k8 = f9_k(8u), k256 = f9_k(256u), k2048 = f9_k(2048u);
  uint32_t d[9];
#pragma unroll
  for (int i = 1; i < 9; ++i) d[i] = a.v[i] << 1;
  uint32_t lo[8], hi = 0;
#pragma unroll
  for (int k = 9; k < 17; ++k) {
    f9_fence();
    uint64_t s = 0;
    if (k > 9) s = (uint64_t)hi * k8;
    if (!(k & 1)) s += (uint64_t)a.v[k >> 1] * a.v[k >> 1];
#pragma unroll
    for (int i = k - 8; 2 * i < k; ++i) s += (uint64_t)a.v[i] * d[k - i];
    lo[k - 9] = (uint32_t)s;
    hi = (uint32_t)(s >> 32);
  }
  uint64_t t = 0;
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    f9_fence();
    uint64_t s = j ? (t >> 29) : 0;
    if (!(j & 1)) s += (uint64_t)a.v[j >> 1] * a.v[j >> 1];
#pragma unroll
    for (int i = 0; 2 * i < j; ++i) s += (uint64_t)a.v[i] * d[j - i];
    if (j < 8) s += (uint64_t)lo[j] * 31264u;
    if (j > 0) s += (uint64_t)lo[j - 1] * k256;
    if (j == 8) s += (uint64_t)hi * 250112u;
    r.v[j] = (uint32_t)s & KHB_M29;
    t = s;
  }
  f9_final(r, (t >> 29) + (uint64_t)hi * k2048, k256);
}

KHB_HD void f9_sqr_n(F9& r, const F9& a, int n) {
  r = a;
  for (int i = 0; i < n; ++i) f9_sqr(r, r);
}

// a^(p-2) (inv(0) = 0), the addition chain of fm_inv (fe_asm.hpp).
KHB_HD void f9_inv(F9& r, const F9& a) {
  F9 x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223, t;
  f9_sqr(x2, a);            f9_mul(x2, x2, a);
  f9_sqr(x3, x2);           f9_mul(x3, x3, a);
  f9_sqr_n(x6, x3, 3);      f9_mul(x6, x6, x3);
  f9_sqr_n(x9, x6, 3);      f9_mul(x9, x9, x3);
  f9_sqr_n(x11, x9, 2);     f9_mul(x11, x11, x2);
  f9_sqr_n(x22, x11, 11);   f9_mul(x22, x22, x11);
  f9_sqr_n(x44, x22, 22);   f9_mul(x44, x44, x22);
  f9_sqr_n(x88, x44, 44);   f9_mul(x88, x88, x44);
  f9_sqr_n(x176, x88, 88);  f9_mul(x176, x176, x88);
  f9_sqr_n(x220, x176, 44); f9_mul(x220, x220, x44);
  f9_sqr_n(x223, x220, 3);  f9_mul(x223, x223, x3);
  f9_sqr_n(t, x223, 23);    f9_mul(t, t, x22);
  f9_sqr_n(t, t, 5);        f9_mul(t, t, a);
  f9_sqr_n(t, t, 3);        f9_mul(t, t, x2);
  f9_sqr_n(t, t, 2);        f9_mul(r, t, a);
}

// 8 x 32 (any value < 2^256) -> 9 x 29, strict (limb 8 < 2^24).
KHB_HD void f9_from_fe(F9& r, const Fe& a) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int b = 29 * i, w = b >> 5, s = b & 31;
    uint64_t x = a.v[w];
    if (w + 1 < 8) x |= (uint64_t)a.v[w + 1] << 32;
    r.v[i] = (uint32_t)(x >> s) & KHB_M29;
  }
}

// Canonical 8 x 32 form (x mod p) of any F9 with limbs < 2^31.
KHB_HD void f9_to_fe(Fe& r, const F9& a) {
  // exact carry pass: y = sum y_i 2^(29 i) with y_i < 2^29 (i < 8), top = bits >= 256
  uint32_t y[9];
  uint64_t t = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    t += a.v[i];
    y[i] = (uint32_t)t & KHB_M29;
    t >>= 29;
  }
  uint64_t top = (t << 5) | (y[8] >> 24);               // value >> 256 (< 2^8)
  y[8] &= 0xFFFFFFu;
  // fold top * 2^256 == top * (2^32 + 977) until the value is < 2^256 (at most twice)
  for (int round = 0; round < 2; ++round) {
    t = (uint64_t)y[0] + top * 977u;
    y[0] = (uint32_t)t & KHB_M29;
    t = (t >> 29) + y[1] + top * 8u;                      // 2^32 = 8 * 2^29
    y[1] = (uint32_t)t & KHB_M29;
    t >>= 29;
    for (int i = 2; i < 9; ++i) {
      t += y[i];
      y[i] = (uint32_t)t & (i < 8 ? KHB_M29 : 0xFFFFFFFFu);
      t >>= (i < 8 ? 29 : 32);
    }
    top = y[8] >> 24;
    y[8] &= 0xFFFFFFu;
  }
  // pack into 8 x 32
  uint32_t w[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int b = 32 * k, i = b / 29, s = b % 29;
    uint64_t x = (uint64_t)y[i] >> s;
    if (i + 1 < 9) x |= (uint64_t)y[i + 1] << (29 - s);
    if (i + 2 < 9 && 58 - s < 32) x |= (uint64_t)y[i + 2] << (58 - s);
    w[k] = (uint32_t)x;
  }
  // x >= p  <=>  x + 0x1000003D1 carries out of 2^256
  Fe f, g;
#pragma unroll
  for (int k = 0; k < 8; ++k) f.v[k] = w[k];
  const uint32_t c = fe_add_k1fold(g.v, f.v);
#pragma unroll
  for (int k = 0; k < 8; ++k) r.v[k] = c ? g.v[k] : f.v[k];
}

// Low 64 bits of the canonical value (x mod p) for limbs < 2^30.6: with V = sum v_i 2^(29 i),
// q = floor(V / 2^256) = v_8 >> 24 (the lower limbs carry < 4 into limb 8) and x = V - q p, so
// x mod 2^64 = (V + q * 0x1000003D1) mod 2^64.  Exact unless limb 8's low 24 bits are within 4 of
// 2^24 (a carry could reach bit 256, or V - q p could still be >= p): *rare = true there, and the
// caller uses f9_to_fe.
KHB_HD void f9_gate_words(uint32_t& w0, uint32_t& w1, bool& rare, const F9& a) {
  const uint32_t q = a.v[8] >> 24;
  rare = (a.v[8] & 0xFFFFFFu) >= 0xFFFFFCu;
  uint64_t v = (uint64_t)a.v[1] * (1u << 29) + a.v[0];   // < 2^60
  v += (uint64_t)(a.v[2] << 26) << 32;                  // limb 2's bits below 2^64 (bits 58..63)
  v += (uint64_t)q * 977u + ((uint64_t)q << 32);
  w0 = (uint32_t)v;
  w1 = (uint32_t)(v >> 32);
}

}  // namespace khb
