// The second and third check of a level-1 candidate, for the device (k_check, khb_check) and compiled
// for the host by the CPU tests (tests/native/test_confirm_host.cpp): SURVEY §8(f)3.
//
//   bsgs_secondcheck   keyhunt.cpp:4271-4304   32 x of Q + AMP2[i], Q = T - base*G, into the level-2 bloom
//   bsgs_thirdcheck    keyhunt.cpp:4306-4368   32 x of Q' + AMP3[i] into the level-3 bloom, bPtable, key
//   bsgs_searchbinary  keyhunt.cpp:3748-3773   (its exact probe sequence: with equal 6-byte keys the index
//                                               it lands on, and so the key tried, is the reference's)
//   calcualteindex     keyhunt.cpp:6680-6689
//   ComputePublicKey   secp256k1/SECP256K1.cpp:61-82 over the reference's GTable layout (29-54)
//   AddDirect          secp256k1/SECP256K1.cpp:242-265 (dx = 0 gives inverse 0: IntMod.cpp:497-500)
//
// This path confirms ~30 candidates per second per GPU in the gated product, so it is
// written for exactness, not speed: the portable canonical field (fe.hpp), one lane per candidate,
// Jacobian accumulation for the scalar multiplications (the point, not the formula, is what the
// reference's Add2 + Reduce returns), 32-element Montgomery batches for the AMP additions.
#pragma once
#include <stdint.h>

#include "bloom_probe.hpp"
#include "fe.hpp"

#if defined(__HIPCC__)
#define KHB_HDN static __host__ __device__ __noinline__   // the big steps stay out of line (code size, compile time)
#else
#define KHB_HDN static
#endif

namespace khb {

struct CPt {
  Fe x, y;
};

// Unsigned 256-bit integers modulo 2^256, little-endian 32-bit limbs (the reference's Int values on this
// path stay below 2^256: range bases plus multiples of M, M2, M3).
struct U8 {
  uint32_t v[8];
};

// r = m * k + b
KHB_HD void u8_mul32_add(U8& r, const U8& m, uint32_t k, const U8& b) {
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t t = (uint64_t)m.v[i] * k + b.v[i] + carry;   // <= 2^64 - 1
    r.v[i] = (uint32_t)t;
    carry = t >> 32;
  }
}

// r = a + s (neg = false) or a - s (neg = true), s < 2^64
KHB_HD void u8_addsub64(U8& r, const U8& a, uint64_t s, bool neg) {
  uint64_t c = 0;
  if (!neg) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint64_t w = i == 0 ? (uint32_t)s : i == 1 ? (uint32_t)(s >> 32) : 0u;
      const uint64_t t = (uint64_t)a.v[i] + w + c;
      r.v[i] = (uint32_t)t;
      c = t >> 32;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint64_t w = (i == 0 ? (uint32_t)s : i == 1 ? (uint32_t)(s >> 32) : 0u) + c;
      const uint64_t t = (uint64_t)a.v[i] - w;
      r.v[i] = (uint32_t)t;
      c = (uint64_t)a.v[i] < w ? 1u : 0u;
    }
  }
}

KHB_HD void fe_neg(Fe& r, const Fe& a) {
  Fe z{};
  fe_sub(r, z, a);
}

// ---- ComputePublicKey ------------------------------------------------------------------------------
struct JPt {
  Fe x, y, z;
  bool inf;
};

KHB_HDN void jac_dbl(JPt& r, const JPt& p) {
  if (p.inf || fe_is_zero(p.y)) {
    r.inf = true;
    return;
  }
  Fe a, b, c, d, e, f, t, x3, y3, z3;
  fe_sqr(a, p.x);
  fe_sqr(b, p.y);
  fe_sqr(c, b);
  fe_add(t, p.x, b);
  fe_sqr(t, t);
  fe_sub(t, t, a);
  fe_sub(t, t, c);
  fe_add(d, t, t);               // D = 2((X + B)^2 - A - C)
  fe_add(e, a, a);
  fe_add(e, e, a);               // E = 3A
  fe_sqr(f, e);
  fe_sub(x3, f, d);
  fe_sub(x3, x3, d);
  fe_sub(t, d, x3);
  fe_mul(y3, e, t);
  fe_add(c, c, c);
  fe_add(c, c, c);
  fe_add(c, c, c);
  fe_sub(y3, y3, c);             // Y3 = E (D - X3) - 8C
  fe_mul(z3, p.y, p.z);
  fe_add(z3, z3, z3);
  r.x = x3;
  r.y = y3;
  r.z = z3;
  r.inf = false;
}

// r = p + q, q affine (q never the point at infinity: GTable entries)
KHB_HDN void jac_madd(JPt& r, const JPt& p, const CPt& q) {
  if (p.inf) {
    r.x = q.x;
    r.y = q.y;
    r.z = Fe{{1u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}};
    r.inf = false;
    return;
  }
  Fe z1z1, u2, s2, h, rr, t;
  fe_sqr(z1z1, p.z);
  fe_mul(u2, q.x, z1z1);
  fe_mul(s2, q.y, p.z);
  fe_mul(s2, s2, z1z1);
  fe_sub(h, u2, p.x);
  fe_sub(rr, s2, p.y);
  if (fe_is_zero(h)) {
    if (fe_is_zero(rr)) {
      const JPt pp = p;
      jac_dbl(r, pp);
    } else {
      r.inf = true;
    }
    return;
  }
  Fe hh, hhh, v, x3, y3, z3;
  fe_sqr(hh, h);
  fe_mul(hhh, h, hh);
  fe_mul(v, p.x, hh);
  fe_sqr(x3, rr);
  fe_sub(x3, x3, hhh);
  fe_sub(x3, x3, v);
  fe_sub(x3, x3, v);
  fe_sub(t, v, x3);
  fe_mul(y3, rr, t);
  fe_mul(t, p.y, hhh);
  fe_sub(y3, y3, t);
  fe_mul(z3, p.z, h);
  r.x = x3;
  r.y = y3;
  r.z = z3;
  r.inf = false;
}

// k*G by the reference's byte windows: gtab[256*i + b - 1] = b * 2^(8i) * G for b in 1..255
// (Secp256K1::Init's GTable), byte i of k little-endian (Int::GetByte).  k = 0 gives (0, 0).
KHB_HDN void ck_mul_g(CPt& r, const U8& k, const CPt* __restrict__ gtab) {
  JPt acc;
  acc.inf = true;
  for (int i = 0; i < 32; ++i) {
    const uint32_t b = (k.v[i >> 2] >> (8 * (i & 3))) & 0xffu;
    if (b) {
      const CPt q = gtab[256 * i + b - 1];
      jac_madd(acc, acc, q);
    }
  }
  if (acc.inf) {
    r.x = Fe{};
    r.y = Fe{};
    return;
  }
  Fe zi, zi2, zi3;
  fe_inv(zi, acc.z);
  fe_sqr(zi2, zi);
  fe_mul(zi3, zi2, zi);
  fe_mul(r.x, acc.x, zi2);
  fe_mul(r.y, acc.y, zi3);
}

// AddDirect(p1, p2), SECP256K1.cpp:242-265
KHB_HD void add_direct_ref(CPt& r, const CPt& p1, const CPt& p2) {
  Fe dy, dx, s, p, x, y;
  fe_sub(dy, p2.y, p1.y);
  fe_sub(dx, p2.x, p1.x);
  fe_inv(dx, dx);
  fe_mul(s, dy, dx);
  fe_sqr(p, s);
  fe_sub(x, p, p1.x);
  fe_sub(x, x, p2.x);
  fe_sub(y, p2.x, x);
  fe_mul(y, y, s);
  fe_sub(y, y, p2.y);
  r.x = x;
  r.y = y;
}

// x of AddDirect(q, tab[i]) for i < 32 with one inversion; an element with dx = 0 gets inverse 0 (as its
// own AddDirect would) and is kept out of the chained product.
KHB_HDN void add_direct_x32(Fe* __restrict__ xs, const CPt& q, const CPt* __restrict__ tab) {
  Fe pre[32];
  Fe acc = Fe{{1u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}};
  for (int i = 0; i < 32; ++i) {
    Fe dx;
    fe_sub(dx, tab[i].x, q.x);
    pre[i] = acc;                              // product of the nonzero dx before i
    if (!fe_is_zero(dx)) fe_mul(acc, acc, dx);
  }
  Fe inv;
  fe_inv(inv, acc);
  for (int i = 31; i >= 0; --i) {
    Fe dx, di, dy, s, p, x;
    fe_sub(dx, tab[i].x, q.x);
    if (fe_is_zero(dx)) {
      di = Fe{};
    } else {
      fe_mul(di, inv, pre[i]);
      fe_mul(inv, inv, dx);
    }
    fe_sub(dy, tab[i].y, q.y);
    fe_mul(s, dy, di);
    fe_sqr(p, s);
    fe_sub(x, p, q.x);
    fe_sub(x, x, tab[i].x);
    xs[i] = x;
  }
}

// ---- tables ----------------------------------------------------------------------------------------
struct CheckTables {
  const CPt* gtab;                 // 32 * 256 points (entry 255 of each window unused)
  const CPt* amp2;                 // BSGS_AMP2[32], keyhunt.cpp:1339-1350
  const CPt* amp3;                 // BSGS_AMP3[32]
  const uint8_t* l2;               // bloom_bPx2nd, 256 sub-blooms concatenated
  const uint8_t* l3;               // bloom_bPx3rd
  const uint8_t* bp;               // bPtable: m3 x struct bsgs_xvalue (16 B: value[6], pad[2], index u64 LE)
  BloomGeom g2, g3;
  uint64_t n_bp;                   // bsgs_m3 (bPtable entries)
  U8 m_double, m2_double, m3, m3_double;
};

struct CheckResult {
  U8 key;
  uint32_t found;                  // 1: key found (bsgs_secondcheck returned 1)
  uint32_t l2_hits;                // level-2 bloom hits of the second check (third checks run)
  uint32_t l3_hits;                // level-3 bloom hits of those third checks
  uint32_t bp_hits;                // bPtable matches (each followed by the key verification)
};

// bsgs_searchbinary's exact loop, keyhunt.cpp:3748-3773
KHB_HD bool search_bp(const uint8_t* __restrict__ bp, int64_t n, const uint8_t* xb, uint64_t& idx) {
  int64_t min = 0, max = n, half = n, current = 0;
  while (half >= 1) {
    half = (max - min) / 2;
    const uint8_t* v = bp + 16 * (current + half);
    int rc = 0;
    for (int b = 0; b < 6 && rc == 0; ++b) rc = (int)xb[16 + b] - (int)v[b];
    if (rc == 0) {
      uint64_t ix = 0;
      for (int b = 7; b >= 0; --b) ix = (ix << 8) | v[8 + b];
      idx = ix;
      return true;
    }
    if (rc < 0) max = max - half;
    else min = min + half;
    current = min;
  }
  return false;
}

KHB_HD void calc_index(U8& r, const CheckTables& T, uint32_t i) {   // calcualteindex
  u8_mul32_add(r, T.m3_double, i, T.m3);
}

// bsgs_thirdcheck(start_range = base, a = i2)
KHB_HDN bool third_check(const CheckTables& T, const U8& base, uint32_t i2, const CPt& target, CheckResult& res) {
  U8 base2;
  u8_mul32_add(base2, T.m2_double, i2, base);
  CPt bpnt, neg, q;
  ck_mul_g(bpnt, base2, T.gtab);
  neg.x = bpnt.x;
  fe_neg(neg.y, bpnt.y);
  add_direct_ref(q, target, neg);
  Fe xs[32];
  add_direct_x32(xs, q, T.amp3);
  for (uint32_t i = 0; i < 32; ++i) {
    if (bloom_probe_x(T.l3, T.g3, xs[i])) {
      res.l3_hits++;
      uint8_t xb[32];
      fe_to_be(xb, xs[i]);
      uint64_t j = 0;
      if (search_bp(T.bp, (int64_t)T.n_bp, xb, j)) {
        res.bp_hits++;
        U8 ci, key;
        calc_index(ci, T, i);
        for (int sgn = 0; sgn < 2; ++sgn) {
          u8_addsub64(key, ci, j + 1, sgn == 1);
          u8_mul32_add(key, key, 1u, base2);
          CPt kp;
          ck_mul_g(kp, key, T.gtab);
          if (fe_eq(kp.x, target.x)) {
            res.key = key;
            return true;
          }
        }
      }
    } else if (fe_eq(q.x, T.amp3[i].x)) {    // AddDirect(P, -P), keyhunt.cpp:4352-4364
      U8 ci;
      calc_index(ci, T, i);
      u8_mul32_add(res.key, ci, 1u, base2);
      return true;
    }
  }
  return false;
}

// bsgs_secondcheck(start_range = chunk base, a = giant step, target): true with res.key on a find.
KHB_HDN bool second_check(const CheckTables& T, const U8& start, uint32_t a, const CPt& target, CheckResult& res) {
  U8 base;
  u8_mul32_add(base, T.m_double, a, start);
  CPt bpnt, neg, q;
  ck_mul_g(bpnt, base, T.gtab);
  neg.x = bpnt.x;
  fe_neg(neg.y, bpnt.y);
  add_direct_ref(q, target, neg);
  Fe xs[32];
  add_direct_x32(xs, q, T.amp2);
  for (uint32_t i = 0; i < 32; ++i) {
    if (bloom_probe_x(T.l2, T.g2, xs[i])) {
      res.l2_hits++;
      if (third_check(T, base, i, target, res)) return true;
    }
  }
  return false;
}

}  // namespace khb
