// gfx950 fast path for the secp256k1 field: hand-placed carry chains.
//
// Why: the scan kernel is VALU-issue-bound (profiles/r01_pmc.txt).  The portable fe.hpp compiles
// to 390 VALU instructions per multiply — 216 of them v_mov_b32 materialising zero-extended
// 64-bit addends.  Here each 32x32 partial product is one v_mad_u64_u32 whose carry-out (VCC)
// is absorbed by one VOP2 v_addc_co_u32 (product scanning), and add/sub are single carry chains.
//
// gfx950 hazard: a VALU that writes VCC (v_add_co/v_sub_co/v_mad_u64_u32 carry-out) needs one
// wait state before a VALU reads that VCC as carry-in — hipcc pads its own chains with `s_nop 0`
// (seen in its ISA for __builtin_addc), but nothing inside an asm string is padded
// (cdna_hip_programming.md §5.7 item 2), so every carry consumer below is preceded by `s_nop 0`.
//
// Value contract (checked by tests/test_gpu_scan.py::test_field_ops and every x-dump test):
//   * fm_mul / fm_sqr return a value < 2^256 congruent to a*b mod p, not necessarily < p ("lazy").
//   * fm_sub(a, b) is correct for a < 2^256 and b < p; its result is < 2^256 (< p if it borrowed).
//   * fm_add(a, b) needs a, b < p and returns a canonical value.
//   * fm_canon brings any value < 2^256 into [0, p).  Values that are hashed, compared or used as a
//     subtrahend (x-coordinates, centres) are canonicalised, so every observable equals the
//     reference's canonical Int (IntMod.cpp) bit for bit.
#pragma once
#include <stdint.h>

#include "fe.hpp"

namespace khb {

#define FM_DEV __device__ __forceinline__

// Rare carries: carry/borrow propagation past limb 1/2 that happens with probability ~2^-30 per call
// (the fold of 2^256 = 0x1000003D1 into a random 256-bit value) runs behind a wave-uniform branch
// taken only when some lane needs it; the common path stops the chain at the limb that produces
// the carry.  The branch body is the full propagation, a no-op for lanes whose carry is 0.
// KHB_NOP: the one wait state between a VCC (carry) write and its VALU reader.  (A timing-only build
// without it was 1.1 % faster, profiles/r01_nonop_ab.txt; the pads stay as the hazard rule asks.)
#define KHB_NOP "s_nop 0\n\t"
#if KHB_RARE_FORCE    // test builds: always take the rare branch (its full propagation is a no-op at c = 0)
FM_DEV bool fm_any(uint32_t) { return true; }
#else
FM_DEV bool fm_any(uint32_t c) { return __builtin_expect(__ballot(c != 0) != 0, 0); }
#endif

// r[k..7] += c (c in {0, 1} per lane), carry-out returned.
template <int K>
FM_DEV uint32_t fm_propagate(uint32_t* r, uint32_t c) {
  uint32_t co = c;
#pragma unroll
  for (int i = K; i < 8; ++i) {
    const uint64_t t = (uint64_t)r[i] + co;
    r[i] = (uint32_t)t;
    co = (uint32_t)(t >> 32);
  }
  return co;
}

// acc += a*b ; c2 += carry-out
FM_DEV void fm_madc(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(c2)
      : "v"(a), "v"(b)
      : "vcc");
}

// ---- 512-bit products without accumulator shuffling ----------------------------------------
// Column k (sum of a_i*b_{k-i}) accumulates in its own 64-bit pair A[k]; the carries out of A[k]
// (weight 2^(32k+64)) are counted in cw[k] and seed A[k+2], which they align with exactly.  So no
// register is ever moved between columns; one add chain at the end folds hi(A[k-1]) into word k:
//   sum_k A[k] 2^(32k) (+ cw[13] 2^480) == a*b.
// The first product of a column cannot overflow (seed < 2^4), the others carry into cw[k].

// acc += a*b; cw = carry-out (first carry of a column: no zero-initialisation needed)
FM_DEV void fm_madc_first(uint64_t& acc, uint32_t& cw, uint32_t a, uint32_t b) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %1, vcc, 0, %4, vcc"
      : "+v"(acc), "=v"(cw)
      : "v"(a), "v"(b), "v"(0u)
      : "vcc");
}

// Column K of a*b (generic product): A seeded, cw receives its carries.
template <int K>
FM_DEV void fm_colx(uint64_t& A, uint32_t& cw, const uint32_t* a, const uint32_t* b) {
  constexpr int lo = K > 7 ? K - 7 : 0, hi = K < 7 ? K : 7;
  A += (uint64_t)a[lo] * b[K - lo];
  if constexpr (hi > lo) {
    fm_madc_first(A, cw, a[lo + 1], b[K - lo - 1]);
#pragma unroll
    for (int i = lo + 2; i <= hi; ++i) fm_madc(A, cw, a[i], b[K - i]);
  }
}

// t[k] = lo(A[k]) + hi(A[k-1]) + carry, k = 1..14; t[15] = cw13 + hi(A[14]) + carry.
FM_DEV void fm_fold_cols(uint32_t t[16], const uint64_t A[15], uint32_t cw13) {
#define FM_LO(k) "v"((uint32_t)A[k])
#define FM_HI(k) "v"((uint32_t)(A[k] >> 32))
  t[0] = (uint32_t)A[0];
  asm("v_add_co_u32_e32 %0, vcc, %15, %16\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %1, vcc, %17, %18, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %2, vcc, %19, %20, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %3, vcc, %21, %22, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %4, vcc, %23, %24, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %5, vcc, %25, %26, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %6, vcc, %27, %28, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %7, vcc, %29, %30, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %8, vcc, %31, %32, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %9, vcc, %33, %34, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %10, vcc, %35, %36, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %11, vcc, %37, %38, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %12, vcc, %39, %40, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %13, vcc, %41, %42, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %14, vcc, %43, %44, vcc"
      : "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]), "=&v"(t[5]), "=&v"(t[6]), "=&v"(t[7]),
        "=&v"(t[8]), "=&v"(t[9]), "=&v"(t[10]), "=&v"(t[11]), "=&v"(t[12]), "=&v"(t[13]), "=&v"(t[14]),
        "=&v"(t[15])
      : FM_LO(1), FM_HI(0), FM_LO(2), FM_HI(1), FM_LO(3), FM_HI(2), FM_LO(4), FM_HI(3), FM_LO(5), FM_HI(4),
        FM_LO(6), FM_HI(5), FM_LO(7), FM_HI(6), FM_LO(8), FM_HI(7), FM_LO(9), FM_HI(8), FM_LO(10), FM_HI(9),
        FM_LO(11), FM_HI(10), FM_LO(12), FM_HI(11), FM_LO(13), FM_HI(12), FM_LO(14), FM_HI(13), "v"(cw13),
        FM_HI(14)
      : "vcc");
#undef FM_LO
#undef FM_HI
}

FM_DEV void fm_mul512x(uint32_t t[16], const uint32_t* a, const uint32_t* b) {
  uint64_t A[15];
  uint32_t cw[14];
  A[0] = (uint64_t)a[0] * b[0];
  A[1] = 0;
  fm_colx<1>(A[1], cw[1], a, b);
  A[2] = 0;
  fm_colx<2>(A[2], cw[2], a, b);
#define FM_COLX(K)            \
  A[K] = (uint64_t)cw[K - 2]; \
  fm_colx<K>(A[K], cw[K], a, b);
  FM_COLX(3) FM_COLX(4) FM_COLX(5) FM_COLX(6) FM_COLX(7) FM_COLX(8) FM_COLX(9) FM_COLX(10)
  FM_COLX(11) FM_COLX(12) FM_COLX(13)
#undef FM_COLX
  A[14] = (uint64_t)cw[12];
  A[14] += (uint64_t)a[7] * b[7];
  fm_fold_cols(t, A, cw[13]);
}

// Column K of the cross sum sum_{i<j} a_i a_j 2^(32(i+j)).
template <int K>
FM_DEV void fm_colsq(uint64_t& A, uint32_t& cw, const uint32_t* a) {
  constexpr int lo = K > 7 ? K - 7 : 0, hi = (K - 1) / 2;   // pairs (i, K-i), i < K-i
  A += (uint64_t)a[lo] * a[K - lo];
  if constexpr (hi > lo) {
    fm_madc_first(A, cw, a[lo + 1], a[K - lo - 1]);
#pragma unroll
    for (int i = lo + 2; i <= hi; ++i) fm_madc(A, cw, a[i], a[K - i]);
  }
}

// a^2 = 2*cross + diag: 36 products instead of 64.
FM_DEV void fm_sqr512x(uint32_t t[16], const uint32_t* a) {
  uint64_t A[15];
  uint32_t cw[14];
  A[0] = 0;
  A[1] = 0;
  fm_colsq<1>(A[1], cw[1], a);
  A[2] = 0;
  fm_colsq<2>(A[2], cw[2], a);
  A[3] = 0;
  fm_colsq<3>(A[3], cw[3], a);
  A[4] = 0;
  fm_colsq<4>(A[4], cw[4], a);
#define FM_COLSQ(K)           \
  A[K] = (uint64_t)cw[K - 2]; \
  fm_colsq<K>(A[K], cw[K], a);
  FM_COLSQ(5) FM_COLSQ(6) FM_COLSQ(7) FM_COLSQ(8) FM_COLSQ(9) FM_COLSQ(10) FM_COLSQ(11) FM_COLSQ(12)
  FM_COLSQ(13)
#undef FM_COLSQ
  A[14] = 0;                  // column 14 holds no cross product (7,7 is diagonal)
  // Only columns 3..11 hold two or more cross products, so only cw[3..11] exist; they seed
  // A[5..13].  Columns 1, 2, 12, 13 carry nothing.
  uint32_t c[16];
  fm_fold_cols(c, A, 0u);     // c = cross sum (c[0] = 0)
  uint64_t D[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) D[i] = (uint64_t)a[i] * a[i];
  // t = D + 2c: the doubled cross sum by one funnel shift per word (v_alignbit_b32, no carry flag:
  // (c_k << 1) | (c_k-1 >> 31); c[0] = 0, and 2c < 2^512 since a^2 < 2^512), then one carry chain
  // instead of adding c twice.
  uint32_t c2[16];
  c2[0] = 0u;
  c2[1] = c[1] << 1;
#pragma unroll
  for (int k = 2; k < 16; ++k) c2[k] = __builtin_amdgcn_alignbit(c[k], c[k - 1], 31);
  uint32_t u[16];
  u[0] = (uint32_t)D[0];
  asm("v_add_co_u32_e32 %0, vcc, %15, %30\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %1, vcc, %16, %31, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %2, vcc, %17, %32, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %3, vcc, %18, %33, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %4, vcc, %19, %34, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %5, vcc, %20, %35, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %6, vcc, %21, %36, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %7, vcc, %22, %37, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %8, vcc, %23, %38, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %9, vcc, %24, %39, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %10, vcc, %25, %40, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %11, vcc, %26, %41, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %12, vcc, %27, %42, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %13, vcc, %28, %43, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %14, vcc, %29, %44, vcc"
      : "=&v"(u[1]), "=&v"(u[2]), "=&v"(u[3]), "=&v"(u[4]), "=&v"(u[5]), "=&v"(u[6]), "=&v"(u[7]), "=&v"(u[8]),
        "=&v"(u[9]), "=&v"(u[10]), "=&v"(u[11]), "=&v"(u[12]), "=&v"(u[13]), "=&v"(u[14]), "=&v"(u[15])
      : "v"((uint32_t)(D[0] >> 32)), "v"((uint32_t)D[1]), "v"((uint32_t)(D[1] >> 32)),
        "v"((uint32_t)D[2]), "v"((uint32_t)(D[2] >> 32)), "v"((uint32_t)D[3]), "v"((uint32_t)(D[3] >> 32)),
        "v"((uint32_t)D[4]), "v"((uint32_t)(D[4] >> 32)), "v"((uint32_t)D[5]), "v"((uint32_t)(D[5] >> 32)),
        "v"((uint32_t)D[6]), "v"((uint32_t)(D[6] >> 32)), "v"((uint32_t)D[7]), "v"((uint32_t)(D[7] >> 32)),
        "v"(c2[1]), "v"(c2[2]), "v"(c2[3]), "v"(c2[4]), "v"(c2[5]), "v"(c2[6]), "v"(c2[7]), "v"(c2[8]),
        "v"(c2[9]), "v"(c2[10]), "v"(c2[11]), "v"(c2[12]), "v"(c2[13]), "v"(c2[14]), "v"(c2[15])
      : "vcc");
#pragma unroll
  for (int i = 0; i < 16; ++i) t[i] = u[i];
}

// Second stage of the reduction: T = L + (H << 32) (+ addend) as 10 words with T9:T8 <= 2^32 + 1,
// H = the high half of the product; returns a value < 2^256 congruent to T + 977*H.
FM_DEV void fm_reduce_T(Fe& r, const uint32_t T[10], const uint32_t* H);

// Reduce t (512 bits) mod p to a value < 2^256 (lazy).  2^256 = 2^32 + 977 (mod p).
FM_DEV void fm_reduce(Fe& r, const uint32_t t[16]) {
  const uint32_t* L = t;
  const uint32_t* H = t + 8;
  // T = L + (H << 32): 9 limbs + T9 (both operands near p make L + H*2^32 reach 2^288)
  uint32_t T[10];
  asm("v_mov_b32 %0, %10\n\t"
      "v_add_co_u32_e32 %1, vcc, %11, %18\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %2, vcc, %12, %19, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %3, vcc, %13, %20, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %4, vcc, %14, %21, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %5, vcc, %15, %22, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %6, vcc, %16, %23, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %7, vcc, %17, %24, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %8, vcc, 0, %25, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %9, vcc, 0, %26, vcc"
      : "=&v"(T[0]), "=&v"(T[1]), "=&v"(T[2]), "=&v"(T[3]), "=&v"(T[4]), "=&v"(T[5]), "=&v"(T[6]), "=&v"(T[7]),
        "=&v"(T[8]), "=&v"(T[9])
      : "v"(L[0]), "v"(L[1]), "v"(L[2]), "v"(L[3]), "v"(L[4]), "v"(L[5]), "v"(L[6]), "v"(L[7]),
        "v"(H[0]), "v"(H[1]), "v"(H[2]), "v"(H[3]), "v"(H[4]), "v"(H[5]), "v"(H[6]), "v"(H[7]), "v"(0u)
      : "vcc");
  fm_reduce_T(r, T, H);
}

// (t + w) mod p, lazy (< 2^256), for t a 512-bit product and any w < 2^256: the addend rides in
// the reduction's first carry chain, so a following modular add/sub (x = s^2 - u) costs 9
// instructions instead of 19.  T = (L + w) + (H << 32) < 2^288 + 2^257: T9:T8 <= 2^32 + 1, the
// same bound fm_reduce_T relies on.
FM_DEV void fm_reduce_add(Fe& r, const uint32_t t[16], const Fe& w) {
  const uint32_t* L = t;
  const uint32_t* H = t + 8;
  uint32_t U[9], T[10];
  asm("v_add_co_u32_e32 %0, vcc, %9, %17\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %1, vcc, %10, %18, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %2, vcc, %11, %19, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %3, vcc, %12, %20, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %4, vcc, %13, %21, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %5, vcc, %14, %22, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %6, vcc, %15, %23, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %7, vcc, %16, %24, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %8, vcc, 0, %25, vcc"
      : "=&v"(U[0]), "=&v"(U[1]), "=&v"(U[2]), "=&v"(U[3]), "=&v"(U[4]), "=&v"(U[5]), "=&v"(U[6]), "=&v"(U[7]),
        "=&v"(U[8])
      : "v"(L[0]), "v"(L[1]), "v"(L[2]), "v"(L[3]), "v"(L[4]), "v"(L[5]), "v"(L[6]), "v"(L[7]),
        "v"(w.v[0]), "v"(w.v[1]), "v"(w.v[2]), "v"(w.v[3]), "v"(w.v[4]), "v"(w.v[5]), "v"(w.v[6]), "v"(w.v[7]),
        "v"(0u)
      : "vcc");
  T[0] = U[0];
  asm("v_add_co_u32_e32 %0, vcc, %9, %17\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %1, vcc, %10, %18, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %2, vcc, %11, %19, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %3, vcc, %12, %20, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %4, vcc, %13, %21, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %5, vcc, %14, %22, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %6, vcc, %15, %23, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %7, vcc, %16, %24, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %8, vcc, 0, %25, vcc"
      : "=&v"(T[1]), "=&v"(T[2]), "=&v"(T[3]), "=&v"(T[4]), "=&v"(T[5]), "=&v"(T[6]), "=&v"(T[7]), "=&v"(T[8]),
        "=&v"(T[9])
      : "v"(U[1]), "v"(U[2]), "v"(U[3]), "v"(U[4]), "v"(U[5]), "v"(U[6]), "v"(U[7]), "v"(U[8]),
        "v"(H[0]), "v"(H[1]), "v"(H[2]), "v"(H[3]), "v"(H[4]), "v"(H[5]), "v"(H[6]), "v"(H[7]), "v"(0u)
      : "vcc");
  fm_reduce_T(r, T, H);
}

FM_DEV void fm_reduce_T(Fe& r, const uint32_t T[10], const uint32_t* H) {
  // P_i = 977*H_i + T_i  (< 2^42), independent
  uint64_t P[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) P[i] = (uint64_t)H[i] * 977u + T[i];
  // R = sum P_i 2^(32i) + (T9:T8) 2^256 : one carry chain; top = R9:R8 < 3 * 2^32
  uint32_t R[8], R8, R9;
  asm("v_mov_b32 %0, %10\n\t"
      "v_add_co_u32_e32 %1, vcc, %11, %12\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %2, vcc, %13, %14, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %3, vcc, %15, %16, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %4, vcc, %17, %18, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %5, vcc, %19, %20, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %6, vcc, %21, %22, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %7, vcc, %23, %24, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %8, vcc, %25, %26, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %9, vcc, 0, %27, vcc"
      : "=&v"(R[0]), "=&v"(R[1]), "=&v"(R[2]), "=&v"(R[3]), "=&v"(R[4]), "=&v"(R[5]), "=&v"(R[6]), "=&v"(R[7]),
        "=&v"(R8), "=&v"(R9)
      : "v"((uint32_t)P[0]),
        "v"((uint32_t)P[1]), "v"((uint32_t)(P[0] >> 32)),
        "v"((uint32_t)P[2]), "v"((uint32_t)(P[1] >> 32)),
        "v"((uint32_t)P[3]), "v"((uint32_t)(P[2] >> 32)),
        "v"((uint32_t)P[4]), "v"((uint32_t)(P[3] >> 32)),
        "v"((uint32_t)P[5]), "v"((uint32_t)(P[4] >> 32)),
        "v"((uint32_t)P[6]), "v"((uint32_t)(P[5] >> 32)),
        "v"((uint32_t)P[7]), "v"((uint32_t)(P[6] >> 32)),
        "v"(T[8]), "v"((uint32_t)(P[7] >> 32)), "v"(T[9])
      : "vcc");
  // second fold: top = R9:R8 (< 3 * 2^32); add top*977 at limb 0 and top*2^32 at limb 1
  const uint64_t u = (uint64_t)R8 * 977u + (uint64_t)(R9 * 977u) * 0x100000000ull;   // < 2^44
  const uint64_t w = (uint64_t)(uint32_t)(u >> 32) + R8;                              // limb-1 addend
  const uint32_t w2 = (uint32_t)(w >> 32) + R9;                                       // limb-2 addend (<= 3)
  uint32_t c;
  // limbs 0..2 take the addends; the carry into limb 3 (probability ~2^-30) is propagated, and
  // a wrap past 2^256 (~2^-212) folded, only in the rare branch.
  uint32_t c3;
  asm("v_add_co_u32_e32 %0, vcc, %0, %4\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %1, vcc, %1, %5, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %2, vcc, %2, %6, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %3, vcc, 0, %7, vcc"
      : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "=&v"(c3)
      : "v"((uint32_t)u), "v"((uint32_t)w), "v"(w2), "v"(0u)
      : "vcc");
  if (fm_any(c3)) {
    c = fm_propagate<3>(R, c3);
    const uint32_t k0 = c * 977u;
    uint64_t t = (uint64_t)R[0] + k0;
    R[0] = (uint32_t)t;
    t = (uint64_t)R[1] + c + (t >> 32);
    R[1] = (uint32_t)t;
    fm_propagate<2>(R, (uint32_t)(t >> 32));
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = R[i];
}

// Multiply / square: seeded columns (fm_mul512x / fm_sqr512x), then the reduction.  (The column-shuffle
// and fold-as-completed schedules were measured slower: profiles/r01_fmbench.txt.)
FM_DEV void fm_mul(Fe& r, const Fe& a, const Fe& b) {
  uint32_t t[16];
  fm_mul512x(t, a.v, b.v);
  fm_reduce(r, t);
}

FM_DEV void fm_sqr(Fe& r, const Fe& a) {
  uint32_t t[16];
  fm_sqr512x(t, a.v);
  fm_reduce(r, t);
}

// r = a^2 + w (mod p), lazy; w < 2^256 (fm_reduce_add).
FM_DEV void fm_sqr_add(Fe& r, const Fe& a, const Fe& w) {
  uint32_t t[16];
  fm_sqr512x(t, a.v);
  fm_reduce_add(r, t, w);
}

// a - b mod p for a < 2^256, b < p.
FM_DEV void fm_sub(Fe& r, const Fe& a, const Fe& b) {
  uint32_t d[8], m, k0, k1, b2;
  asm("v_sub_co_u32_e32 %0, vcc, %12, %20\n\t"
      KHB_NOP
      "v_subb_co_u32_e32 %1, vcc, %13, %21, vcc\n\t"
      KHB_NOP
      "v_subb_co_u32_e32 %2, vcc, %14, %22, vcc\n\t"
      KHB_NOP
      "v_subb_co_u32_e32 %3, vcc, %15, %23, vcc\n\t"
      KHB_NOP
      "v_subb_co_u32_e32 %4, vcc, %16, %24, vcc\n\t"
      KHB_NOP
      "v_subb_co_u32_e32 %5, vcc, %17, %25, vcc\n\t"
      KHB_NOP
      "v_subb_co_u32_e32 %6, vcc, %18, %26, vcc\n\t"
      KHB_NOP
      "v_subb_co_u32_e32 %7, vcc, %19, %27, vcc\n\t"
      // m = borrow ? 0xffffffff : 0 ; subtract (0x1000003D1 & m), i.e. add p on borrow
      KHB_NOP
      "v_subb_co_u32_e32 %8, vcc, 0, %28, vcc\n\t"
      "v_and_b32_e32 %9, 0x3d1, %8\n\t"
      "v_and_b32_e32 %10, 1, %8\n\t"
      "v_sub_co_u32_e32 %0, vcc, %0, %9\n\t"
      KHB_NOP
      "v_subb_co_u32_e32 %1, vcc, %1, %10, vcc\n\t"
      KHB_NOP
      // the borrow into limb 2 (probability ~2^-32) is propagated in the rare branch
      "v_subb_co_u32_e32 %11, vcc, 0, %28, vcc"
      : "=&v"(d[0]), "=&v"(d[1]), "=&v"(d[2]), "=&v"(d[3]), "=&v"(d[4]), "=&v"(d[5]), "=&v"(d[6]), "=&v"(d[7]),
        "=&v"(m), "=&v"(k0), "=&v"(k1), "=&v"(b2)
      : "v"(a.v[0]), "v"(a.v[1]), "v"(a.v[2]), "v"(a.v[3]), "v"(a.v[4]), "v"(a.v[5]), "v"(a.v[6]), "v"(a.v[7]),
        "v"(b.v[0]), "v"(b.v[1]), "v"(b.v[2]), "v"(b.v[3]), "v"(b.v[4]), "v"(b.v[5]), "v"(b.v[6]), "v"(b.v[7]),
        "v"(0u)
      : "vcc");
  if (fm_any(b2)) {      // b2 = 0xffffffff where the correction borrowed out of limb 1
    uint32_t bo = b2 & 1u;
#pragma unroll
    for (int i = 2; i < 8; ++i) {
      const uint32_t t = d[i] - bo;
      bo = (bo && d[i] == 0) ? 1u : 0u;
      d[i] = t;
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = d[i];
}

// r = a + 0x1000003D1 (mod 2^256) with carry-out, as a chain (the "subtract p" step).
FM_DEV uint32_t fm_add_k(uint32_t t[8], const uint32_t s[8]) {
  uint32_t c;
  asm("v_add_co_u32_e32 %0, vcc, 0x3d1, %9\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %1, vcc, 1, %10, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %2, vcc, 0, %11, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %3, vcc, 0, %12, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %4, vcc, 0, %13, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %5, vcc, 0, %14, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %6, vcc, 0, %15, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %7, vcc, 0, %16, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %8, vcc, 0, %17, vcc"
      : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]), "=&v"(t[5]), "=&v"(t[6]), "=&v"(t[7]),
        "=&v"(c)
      : "v"(s[0]), "v"(s[1]), "v"(s[2]), "v"(s[3]), "v"(s[4]), "v"(s[5]), "v"(s[6]), "v"(s[7]), "v"(0u)
      : "vcc");
  return c;
}

// canonical a mod p for a < 2^256
FM_DEV void fm_canon(Fe& r, const Fe& a) {
  uint32_t t[8];
  const uint32_t c = fm_add_k(t, a.v);
  const bool sel = c != 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = sel ? t[i] : a.v[i];
}

// a + b mod p, lazy: for a < p and b < 2^256 (so a + b < 2^257 - 0x1000003D1) the sum folds its
// carry back as 2^256 = 0x1000003D1 (mod p) and stays < 2^256.  Feeds a product only.
FM_DEV void fm_add_lazy(Fe& r, const Fe& a, const Fe& b) {
  uint32_t s[8], c;
  asm("v_add_co_u32_e32 %0, vcc, %9, %17\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %1, vcc, %10, %18, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %2, vcc, %11, %19, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %3, vcc, %12, %20, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %4, vcc, %13, %21, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %5, vcc, %14, %22, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %6, vcc, %15, %23, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %7, vcc, %16, %24, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %8, vcc, 0, %25, vcc"       // c = carry (0/1)
      : "=&v"(s[0]), "=&v"(s[1]), "=&v"(s[2]), "=&v"(s[3]), "=&v"(s[4]), "=&v"(s[5]), "=&v"(s[6]), "=&v"(s[7]),
        "=&v"(c)
      : "v"(a.v[0]), "v"(a.v[1]), "v"(a.v[2]), "v"(a.v[3]), "v"(a.v[4]), "v"(a.v[5]), "v"(a.v[6]), "v"(a.v[7]),
        "v"(b.v[0]), "v"(b.v[1]), "v"(b.v[2]), "v"(b.v[3]), "v"(b.v[4]), "v"(b.v[5]), "v"(b.v[6]), "v"(b.v[7]),
        "v"(0u)
      : "vcc");
  // fold the carry as 2^256 = 0x1000003D1: limbs 0..1 always; the carry into limb 2 only behind
  // the rare branch
  uint32_t c2;
  asm("v_mul_u32_u24_e32 %2, 0x3d1, %3\n\t"
      "v_add_co_u32_e32 %0, vcc, %0, %2\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %1, vcc, %1, %3, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %2, vcc, 0, %4, vcc"
      : "+v"(s[0]), "+v"(s[1]), "=&v"(c2)
      : "v"(c), "v"(0u)
      : "vcc");
  if (fm_any(c2)) fm_propagate<2>(s, c2);
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = s[i];
}

// a + b mod p, a, b < p, canonical result
FM_DEV void fm_add(Fe& r, const Fe& a, const Fe& b) {
  uint32_t s[8], c;
  asm("v_add_co_u32_e32 %0, vcc, %9, %17\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %1, vcc, %10, %18, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %2, vcc, %11, %19, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %3, vcc, %12, %20, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %4, vcc, %13, %21, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %5, vcc, %14, %22, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %6, vcc, %15, %23, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %7, vcc, %16, %24, vcc\n\t"
      KHB_NOP
      "v_addc_co_u32_e32 %8, vcc, 0, %25, vcc"
      : "=&v"(s[0]), "=&v"(s[1]), "=&v"(s[2]), "=&v"(s[3]), "=&v"(s[4]), "=&v"(s[5]), "=&v"(s[6]), "=&v"(s[7]),
        "=&v"(c)
      : "v"(a.v[0]), "v"(a.v[1]), "v"(a.v[2]), "v"(a.v[3]), "v"(a.v[4]), "v"(a.v[5]), "v"(a.v[6]), "v"(a.v[7]),
        "v"(b.v[0]), "v"(b.v[1]), "v"(b.v[2]), "v"(b.v[3]), "v"(b.v[4]), "v"(b.v[5]), "v"(b.v[6]), "v"(b.v[7]),
        "v"(0u)
      : "vcc");
  uint32_t t[8];
  const uint32_t ct = fm_add_k(t, s);
  const bool sel = (c | ct) != 0;    // a+b >= p  <=>  carry out of a+b or of (a+b mod 2^256)+K
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = sel ? t[i] : s[i];
}

FM_DEV void fm_sqr_n(Fe& r, const Fe& a, int n) {
  r = a;
  for (int i = 0; i < n; ++i) fm_sqr(r, r);
}

// a^(p-2) (inv(0) = 0); lazy result (congruent, < 2^256).
FM_DEV void fm_inv(Fe& r, const Fe& a) {
  Fe x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223, t;
  fm_sqr(x2, a);            fm_mul(x2, x2, a);
  fm_sqr(x3, x2);           fm_mul(x3, x3, a);
  fm_sqr_n(x6, x3, 3);      fm_mul(x6, x6, x3);
  fm_sqr_n(x9, x6, 3);      fm_mul(x9, x9, x3);
  fm_sqr_n(x11, x9, 2);     fm_mul(x11, x11, x2);
  fm_sqr_n(x22, x11, 11);   fm_mul(x22, x22, x11);
  fm_sqr_n(x44, x22, 22);   fm_mul(x44, x44, x22);
  fm_sqr_n(x88, x44, 44);   fm_mul(x88, x88, x44);
  fm_sqr_n(x176, x88, 88);  fm_mul(x176, x176, x88);
  fm_sqr_n(x220, x176, 44); fm_mul(x220, x220, x44);
  fm_sqr_n(x223, x220, 3);  fm_mul(x223, x223, x3);
  fm_sqr_n(t, x223, 23);    fm_mul(t, t, x22);
  fm_sqr_n(t, t, 5);        fm_mul(t, t, a);
  fm_sqr_n(t, t, 3);        fm_mul(t, t, x2);
  fm_sqr_n(t, t, 2);        fm_mul(r, t, a);
}

}  // namespace khb
