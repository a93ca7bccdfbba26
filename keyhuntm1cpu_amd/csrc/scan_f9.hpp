// The -m bsgs gated walk in 9 x 29-bit limbs (device/fe29.hpp): an alternative to the product's 8 x 32
// walk, built only by `make variants` (lib/libkhbsgs_f9.so, KHB_F9WALK=1) and kept parity-tested
// (tests/test_gpu_f9walk.py).  Included by scan_kernels.hpp inside namespace khbk.
//
// Why it is not the product (profiles/r02_f9_walk.md, profiles/r03c_f9_ab.txt, r03g): it executes
// ~19 % fewer VALU instructions per giant step (PMC SQ_INSTS_VALU 7.70e10 vs 9.48e10 per 2^33 steps),
// but 90 % of them are 64-bit-class (v_mad_u64_u32, v_lshrrev_b64, v_lshl_add_u64) at ~4.7 SIMD
// cycles each against the product mix's ~3.9, and the multiplier-dense stream runs at a lower shader
// clock (2175 vs 2240 MHz, khb_stats.shader_mhz): 46.4 vs 48.4 G steps/s on 4096-chunk launches.
#pragma once

// ---- the product walk in 9 x 29-bit limbs (kScanG, kScanG1, kDumpG; device/fe29.hpp) -----------

// GSn in 9 x 29 limbs (khb_load_giant_table): x of rows 0..512, then y, then p - x; wave-uniform
// rows through the constant address space (scalar loads), as GsnTable.
struct Gsn9 {
  const F9* p;
  typedef const __attribute__((address_space(4))) uint32_t* CW;
  __device__ __forceinline__ F9 ld(uint32_t row) const {
    CW w = (CW)p + 9 * row;
    F9 r;
#pragma unroll
    for (int k = 0; k < 9; ++k) r.v[k] = w[k];
    return r;
  }
  __device__ __forceinline__ F9 x(uint32_t i) const { return ld(i); }
  __device__ __forceinline__ F9 y(uint32_t i) const { return ld(KHB_GIANT_TABLE + i); }
  __device__ __forceinline__ F9 nx(uint32_t i) const { return ld(2 * KHB_GIANT_TABLE + i); }
};

// Lane-private scratch of the F9 path: 36 bytes per lane per entry, split by limbs so that every
// access is an aligned, fully coalesced wave-wide block: entry e occupies 36 * lanes bytes at
// e * 36 * lanes, limbs 0-3 of all lanes (16 B each), then limbs 4-7, then limb 8 (4 B each).  An
// 8 x 32 value (centres) uses the first two parts.
struct Scr9 {
  uint8_t* s;
  size_t S;
  uint32_t lane;
  __device__ __forceinline__ v4u* p0(uint32_t e) const { return reinterpret_cast<v4u*>(s + (size_t)e * 36 * S) + lane; }
  __device__ __forceinline__ v4u* p1(uint32_t e) const {
    return reinterpret_cast<v4u*>(s + (size_t)e * 36 * S + 16 * S) + lane;
  }
  __device__ __forceinline__ uint32_t* p2(uint32_t e) const {
    return reinterpret_cast<uint32_t*>(s + (size_t)e * 36 * S + 32 * S) + lane;
  }
  __device__ __forceinline__ F9 ld9(uint32_t e) const {
    const v4u a = *p0(e), b = *p1(e);
    return F9{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, *p2(e)}};
  }
  __device__ __forceinline__ void st9(uint32_t e, const F9& v) const {
    *p0(e) = v4u{v.v[0], v.v[1], v.v[2], v.v[3]};
    *p1(e) = v4u{v.v[4], v.v[5], v.v[6], v.v[7]};
    *p2(e) = v.v[8];
  }
  __device__ __forceinline__ Fe ldfe(uint32_t e) const {
    const v4u a = *p0(e), b = *p1(e);
    return Fe{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}};
  }
  __device__ __forceinline__ void stfe(uint32_t e, const Fe& v) const {
    *p0(e) = v4u{v.v[0], v.v[1], v.v[2], v.v[3]};
    *p1(e) = v4u{v.v[4], v.v[5], v.v[6], v.v[7]};
  }
};

__device__ __forceinline__ F9 f9_small(uint32_t v) {
  F9 r;
#pragma unroll
  for (int k = 0; k < 9; ++k) r.v[k] = k ? 0u : v;
  return r;
}

// Low 64 bits of canonical x (the gate's words, f9_gate_words); the rare inputs whose fast words
// are not exact take the full conversion behind a wave-uniform branch.
__device__ __forceinline__ void gate_words(const F9& x, uint32_t& w0, uint32_t& w1) {
  bool rare;
  f9_gate_words(w0, w1, rare, x);
  if (__builtin_expect(__ballot(rare) != 0, 0)) {
    if (rare) {
      Fe c;
      f9_to_fe(c, x);
      w0 = c.v[0];
      w1 = c.v[1];
    }
  }
}

__device__ __forceinline__ uint32_t gate_bits_w(const ScanArgs& A, uint32_t w1) {
  const uint32_t b0 = w1 & 63u, b1 = A.gate_probes > 1 ? (w1 >> 6) & 63u : b0;
  const uint32_t b2 = A.gate_probes > 2 ? (w1 >> 12) & 63u : b1;
  return b0 | (b1 << 6) | (b2 << 12);
}

// The gate test of one x from its canonical words: the 64-bit block load is issued here and waited
// for in pass(), so a step issues both x's loads before testing either (GatePend).  With the stage-1
// fold the fold's block is tested first and the full gate's block is read only for its survivors.
template <bool STAGE1>
struct Gate9 {
  uint32_t lo, hi, bits, w0;
  __device__ __forceinline__ void issue(const ScanArgs& A, uint32_t a0, uint32_t a1) {
    const uint2 w = reinterpret_cast<const uint2*>(STAGE1 ? A.gate1 : A.gate)[a0 & (STAGE1 ? A.gate1_mask : A.gate_mask)];
    lo = w.x;
    hi = w.y;
    bits = gate_bits_w(A, a1);
    w0 = a0;
  }
};

template <bool STAGE1>
__device__ __forceinline__ void gate_resolve(const ScanArgs& A, const Gate9<STAGE1>& g1, bool has2,
                                             const Gate9<STAGE1>& g2, bool& h1, bool& h2) {
  if constexpr (STAGE1) {
    const bool s1 = gate_block_pass(g1.lo, g1.hi, g1.bits), s2 = has2 && gate_block_pass(g2.lo, g2.hi, g2.bits);
    h1 = h2 = false;
    if (__ballot(s1 || s2) == 0) return;
    uint2 w1 = make_uint2(0u, 0u), w2 = make_uint2(0u, 0u);
    if (s1) w1 = reinterpret_cast<const uint2*>(A.gate)[g1.w0 & A.gate_mask];
    if (s2) w2 = reinterpret_cast<const uint2*>(A.gate)[g2.w0 & A.gate_mask];
    h1 = s1 && gate_block_pass(w1.x, w1.y, g1.bits);
    h2 = s2 && gate_block_pass(w2.x, w2.y, g2.bits);
  } else {
    h1 = gate_block_pass(g1.lo, g1.hi, g1.bits);
    h2 = has2 && gate_block_pass(g2.lo, g2.hi, g2.bits);
  }
}

__device__ __forceinline__ void x_dump9(const ScanArgs& A, const F9& x, uint32_t step) {
  Fe c;
  f9_to_fe(c, x);
  fe_to_be(A.xdump + ((uint64_t)step - (uint64_t)A.group_begin * KHB_GROUP) * 32, c);
}

// walk_group_g in 9 x 29 limbs: the same points in the same order (pts[511 - i] = C - GSn[i],
// pts[513 + i] = C + GSn[i], pts[512] = C), x = s^2 + nu with nu = (p - GSn.x) + (p - C.x), the
// prefix of step i - 1 loaded right after step i's last use of the prefix register.  inv is the
// inverse of the group's 512 dx; sg.ld9(e0 + e) is prefix e of this group.
// Register budget (128 VGPRs at 4 waves/SIMD): the first x of a step is reduced to its gate words
// and its gate load before the second is computed, and is recomputed (from idx) only for a gate
// survivor; -C.y is not held (f9_add_neg forms GSn.y - C.y from C.y).
// p - C.x (which = 0) and C.y (which = 1) of the walked group: parked in LDS by walk_group_g9 and
// read where used (volatile: no hoisting back into registers).
#ifndef KHB_CN_LDS
#define KHB_CN_LDS 3              // F9 walk: bit 0 p - C.x, bit 1 C.y parked in LDS (else held in registers)
#endif
__device__ __forceinline__ F9 cn_load(const ProbeQueue& Q, int which) {
  const uint32_t wl = threadIdx.x & 63u;
  F9 r;
#pragma unroll
  for (int k = 0; k < 9; ++k) r.v[k] = Q.cn[(9 * which + k) * 64 + wl];
  return r;
}

template <int MODE>
__device__ __forceinline__ void walk_group_g9(const ScanArgs& A, ProbeQueue& Q, const AffPt& C, F9 inv,
                                              uint32_t job, uint32_t j, const Scr9& sg, uint32_t e0) {
  constexpr bool STAGE1 = MODE == kScanG1;
  const Gsn9 g9{A.gsn9};
  const uint32_t base = j * KHB_GROUP;
  // p - C.x and C.y: in LDS (KHB_CN_LDS bit 0: p - C.x, bit 1: C.y) or in registers
#if KHB_CN_LDS & 1
#define ncx cn_load(Q, 0)
#else
  F9 ncx;
#endif
#if KHB_CN_LDS & 2
#define cy cn_load(Q, 1)
#else
  F9 cy;
#endif
  {
    Fe p, t;
    F9 ncx_, cy_;
#pragma unroll
    for (int k = 0; k < 8; ++k) p.v[k] = k == 0 ? KHB_P0 : (k == 1 ? KHB_P1 : 0xFFFFFFFFu);
    fm_sub(t, p, C.x);
    f9_from_fe(ncx_, t);
    f9_from_fe(cy_, C.y);
    const uint32_t wl = threadIdx.x & 63u;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      if (KHB_CN_LDS & 1) Q.cn[k * 64 + wl] = ncx_.v[k];
      if (KHB_CN_LDS & 2) Q.cn[(9 + k) * 64 + wl] = cy_.v[k];
    }
#if !(KHB_CN_LDS & 1)
    ncx = ncx_;
#endif
#if !(KHB_CN_LDS & 2)
    cy = cy_;
#endif
  }
  F9 pre = sg.ld9(e0 + kHalf - 2);
  F9 idx, dx, s, x;
  {   // step 511: pts[0] = C - GSn[511] only
    f9_mul(idx, inv, pre);
    pre = sg.ld9(e0 + kHalf - 3);
    f9_add(dx, g9.x(kHalf - 1), ncx);
    f9_mul(inv, inv, dx);
    f9_add(s, g9.y(kHalf - 1), cy);
    f9_mul(s, s, idx);
    f9_sqr(x, s);
    f9_add(x, x, g9.nx(kHalf - 1));
    f9_add(x, x, ncx);
    if constexpr (MODE == kDumpG) {
      x_dump9(A, x, base);
    } else {
      uint32_t a0, a1;
      gate_words(x, a0, a1);
      Gate9<STAGE1> q;
      q.issue(A, a0, a1);
      bool h1, h2;
      gate_resolve<STAGE1>(A, q, false, q, h1, h2);
      if (__ballot(h1) != 0) {
        Fe c = Fe{};
        if (h1) f9_to_fe(c, x);
        q_push(Q, h1, c, job, base);
        q_drain(A, Q, kDrainAt);
      }
    }
  }
  for (int i = (int)kHalf - 2; i >= 0; --i) {
    if (i > 0) {
      f9_mul(idx, inv, pre);
      pre = sg.ld9(e0 + (i >= 2 ? i - 2 : 0));    // i = 1: a harmless reload of prefix 0
      f9_add(dx, g9.x(i), ncx);
      f9_mul(inv, inv, dx);
    } else {
      idx = inv;
    }
    const uint32_t t1 = base + kHalf - 1 - (uint32_t)i, t2 = base + kHalf + 1 + (uint32_t)i;
    // C - GSn[i]: s' = (GSn.y + C.y) / dx, x = s'^2 + nu
    f9_add(s, g9.y(i), cy);
    f9_mul(s, s, idx);
    f9_sqr(x, s);
    f9_add(x, x, g9.nx(i));
    f9_add(x, x, ncx);
    Gate9<STAGE1> q1, q2;
    if constexpr (MODE == kDumpG) {
      x_dump9(A, x, t1);
    } else {
      uint32_t a0, a1;
      gate_words(x, a0, a1);
      q1.issue(A, a0, a1);
    }
    // C + GSn[i]: s = (GSn.y - C.y) / dx
    f9_add_neg(s, g9.y(i), cy);
    f9_mul(s, s, idx);
    f9_sqr(x, s);
    f9_add(x, x, g9.nx(i));
    f9_add(x, x, ncx);
    if constexpr (MODE == kDumpG) {
      x_dump9(A, x, t2);
    } else {
      uint32_t a0, a1;
      gate_words(x, a0, a1);
      q2.issue(A, a0, a1);
      bool h1, h2;
      gate_resolve<STAGE1>(A, q1, true, q2, h1, h2);
      // ~0.04 % of x pass: their canonical forms go to the queue, one x at a time (the second x
      // first, then the first recomputed from idx), so this rare path needs few registers
      if (__ballot(h2) != 0) {
        Fe c = Fe{};
        if (h2) f9_to_fe(c, x);
        q_push(Q, h2, c, job, t2);
        q_drain(A, Q, kDrainAt);
      }
      if (__ballot(h1) != 0) {
        Fe c = Fe{};
        if (h1) {
          f9_add(s, g9.y(i), cy);
          f9_mul(s, s, idx);
          f9_sqr(x, s);
          f9_add(x, x, g9.nx(i));
          f9_add(x, x, ncx);
          f9_to_fe(c, x);
        }
        q_push(Q, h1, c, job, t1);
        q_drain(A, Q, kDrainAt);
      }
    }
  }
#if KHB_CN_LDS & 1
#undef ncx
#endif
#if KHB_CN_LDS & 2
#undef cy
#endif
  if constexpr (MODE == kDumpG) {
    fe_to_be(A.xdump + ((uint64_t)(j - A.group_begin) * KHB_GROUP + kHalf) * 32, C.x);
  } else {
    probe<false>(A, Q, C.x, job, j, kHalf);      // the centre, pts[512] (canonical)
  }
}

// scan_batch for the F9 walk: step 0 (centres) in 8 x 32 as scan_batch; steps 1-3 (forward
// prefix products, one inversion for the batch, the walks) in 9 x 29 limbs.  Scratch entries are
// 36 bytes (Scr9), numbered as in scan_batch: g*512 + i prefixes, g*512 + 511 = T_g then inv(T_g),
// kBatch*512 + 2g (+1) = C_g.x (.y), kBatch*514 + g = chained products.
template <int MODE>
__device__ __forceinline__ uint32_t scan_batch9(const ScanArgs& A, ProbeQueue& Q, uint32_t job, uint32_t g0,
                                                uint32_t g1, uint32_t lane) {
  const Scr9 sr{reinterpret_cast<uint8_t*>(A.scratch), (size_t)A.stride, lane};
  const Gsn9 g9{A.gsn9};
  const GsnTable gsn{A.gsn};
  const uint32_t nb = g1 - g0;
  constexpr uint32_t SC = kBatch * kHalf, SQ = kBatch * (kHalf + 2);
  const AffPt P = A.centres[job];
  // 0. centres (as scan_batch, 8 x 32)
  uint32_t skip = 0;
  {
    Fe acc;
    for (uint32_t g = 0; g < nb; ++g) {
      const uint32_t jg = g0 + g;
      Fe d = fe_small(1);
      if (jg != 0) {
        fm_sub(d, A.gofs[jg].x, P.x);
        Fe dc;
        fm_canon(dc, d);
        if (fe_is_zero(dc)) {
          d = fe_small(1);
          skip |= 1u << g;
          if (MODE != kDumpG) {
            const uint32_t k = atomicAdd(&A.counters[1], 1u);
            if (k < A.degen_cap) A.degen[k] = khb_degenerate{job, jg | 0x80000000u};
          }
        }
      } else {
        skip |= 1u << g;
      }
      if (g == 0) acc = d; else fm_mul(acc, acc, d);
      sr.stfe(SQ + g, acc);
    }
    Fe inv;
    fm_inv(inv, acc);
    for (int g = (int)nb - 1; g >= 0; --g) {
      const uint32_t jg = g0 + (uint32_t)g;
      const AffPt O = A.gofs[jg];
      Fe ig;
      if (g > 0) {
        fm_mul(ig, inv, sr.ldfe(SQ + g - 1));
        Fe d = fe_small(1);
        if (!((skip >> g) & 1u)) fm_sub(d, O.x, P.x);
        fm_mul(inv, inv, d);
      } else {
        ig = inv;
      }
      AffPt C = P;
      if (jg != 0) {
        if ((skip >> g) & 1u) ig = fe_small(0);
        Fe s, x, y;
        fm_sub(s, O.y, P.y);
        fm_mul(s, s, ig);
        fm_sqr(x, s);
        fm_sub(x, x, P.x);
        fm_sub(x, x, O.x);
        fm_canon(x, x);
        fm_sub(y, O.x, x);
        fm_mul(y, y, s);
        fm_sub(y, y, O.y);
        fm_canon(y, y);
        C.x = x;
        C.y = y;
      }
      sr.stfe(SC + 2 * g, C.x);
      sr.stfe(SC + 2 * g + 1, C.y);
    }
  }
  // 1. forward passes (F9): prefixes of dx_i = GSn[i].x + (p - C.x)
  const Fe g2x = gsn.x(kHalf);
  uint32_t degen = 0;
  F9 acc;
  for (uint32_t g = 0; g < nb; ++g) {
    const uint32_t e0 = g * kHalf;
    const Fe cx = sr.ldfe(SC + 2 * g);
    F9 ncx;
    {
      Fe p, t;
#pragma unroll
      for (int k = 0; k < 8; ++k) p.v[k] = k == 0 ? KHB_P0 : (k == 1 ? KHB_P1 : 0xFFFFFFFFu);
      fm_sub(t, p, cx);
      f9_from_fe(ncx, t);
    }
    F9 a, dx;
    f9_add(a, g9.x(0), ncx);
    sr.st9(e0, a);
    for (uint32_t i = 1; i < kHalf - 1; ++i) {
      f9_add(dx, g9.x(i), ncx);
      f9_mul(a, a, dx);
      sr.st9(e0 + i, a);
    }
    f9_add(dx, g9.x(kHalf - 1), ncx);
    f9_mul(a, a, dx);
    Fe ac;
    f9_to_fe(ac, a);
    if (fe_is_zero(ac) || fe_eq(g2x, cx)) {
      degen |= 1u << g;
      a = f9_small(1);
    }
    sr.st9(e0 + kHalf - 1, a);
    if (g == 0) acc = a; else f9_mul(acc, acc, a);
    sr.st9(SQ + g, acc);
  }
  // 2. one inversion for the batch
  F9 inv;
  f9_inv(inv, acc);
  for (int g = (int)nb - 1; g >= 0; --g) {
    const uint32_t e0 = (uint32_t)g * kHalf;
    F9 ig;
    if (g > 0) {
      f9_mul(ig, inv, sr.ld9(SQ + g - 1));
      f9_mul(inv, inv, sr.ld9(e0 + kHalf - 1));
    } else {
      ig = inv;
    }
    if ((degen >> g) & 1u) ig = f9_small(0);
    sr.st9(e0 + kHalf - 1, ig);
  }
  // 3. backward walks
  uint32_t walked = 0;
  for (uint32_t g = 0; g < nb; ++g, ++walked) {
    const uint32_t e0 = g * kHalf;
    asm volatile("" ::: "memory");
    const AffPt C{sr.ldfe(SC + 2 * g), sr.ldfe(SC + 2 * g + 1)};
    walk_group_g9<MODE>(A, Q, C, sr.ld9(e0 + kHalf - 1), job, g0 + g, sr, e0);
    if (MODE != kDumpG && ((degen >> g) & 1u)) {
      const uint32_t k = atomicAdd(&A.counters[1], 1u);
      if (k < A.degen_cap) A.degen[k] = khb_degenerate{job, g0 + g};
    }
  }
  return walked;
}

