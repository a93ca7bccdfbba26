# Patch for tools/experiments/calib_build.sh: the paired reduction (round 3, measured slower at
# 4 waves/SIMD: profiles/r03_calibration/pair_reduction_ab.txt).  Exact: P_i = 977*H_i + (L_i, H_i)
# as one v_mad_u64_u32 per word; a wave whose mads carried out redoes the reduction via the T chain.
p = 'keyhuntm1cpu_amd/csrc/device/fe_asm.hpp'
s = open(p).read()
a = """// Reduce t (512 bits) mod p to a value < 2^256 (lazy).  2^256 = 2^32 + 977 (mod p).
FM_DEV void fm_reduce(Fe& r, const uint32_t t[16]) {
  const uint32_t* L = t;
  const uint32_t* H = t + 8;
"""
b = """FM_DEV void fm_reduce_top(Fe& r, uint32_t R[8], uint32_t R8, uint32_t R9);

FM_DEV uint64_t fm_reduce_pair(Fe& r, const uint32_t* L, const uint32_t* H, uint32_t top) {
  uint64_t P[8], ovf = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t c;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4"
        : "=v"(P[i]), "=s"(c)
        : "v"(H[i]), "s"(977u), "v"(((uint64_t)H[i] << 32) | L[i]));
    ovf |= c;
  }
  uint32_t R[8], R8, R9;
  asm("v_mov_b32 %0, %10\\n\\t"
      "v_add_co_u32_e32 %1, vcc, %11, %12\\n\\t"
      KHB_NOP
      "v_addc_co_u32_e32 %2, vcc, %13, %14, vcc\\n\\t"
      KHB_NOP
      "v_addc_co_u32_e32 %3, vcc, %15, %16, vcc\\n\\t"
      KHB_NOP
      "v_addc_co_u32_e32 %4, vcc, %17, %18, vcc\\n\\t"
      KHB_NOP
      "v_addc_co_u32_e32 %5, vcc, %19, %20, vcc\\n\\t"
      KHB_NOP
      "v_addc_co_u32_e32 %6, vcc, %21, %22, vcc\\n\\t"
      KHB_NOP
      "v_addc_co_u32_e32 %7, vcc, %23, %24, vcc\\n\\t"
      KHB_NOP
      "v_addc_co_u32_e32 %8, vcc, %25, %26, vcc\\n\\t"
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
        "v"(top), "v"((uint32_t)(P[7] >> 32)), "v"(0u)
      : "vcc");
  fm_reduce_top(r, R, R8, R9);
  return ovf;
}

#if KHB_RARE_FORCE
FM_DEV bool fm_pair_ovf(uint64_t) { return true; }
#else
FM_DEV bool fm_pair_ovf(uint64_t m) { return __builtin_expect(m != 0, 0); }
#endif

// Reduce t (512 bits) mod p to a value < 2^256 (lazy).  2^256 = 2^32 + 977 (mod p).
FM_DEV void fm_reduce(Fe& r, const uint32_t t[16]) {
  const uint32_t* L = t;
  const uint32_t* H = t + 8;
  if (!fm_pair_ovf(fm_reduce_pair(r, L, H, 0u))) return;
"""
assert a in s; s = s.replace(a, b)
a = """        "v"(0u)
      : "vcc");
  T[0] = U[0];"""
b = """        "v"(0u)
      : "vcc");
  if (!fm_pair_ovf(fm_reduce_pair(r, U, H, U[8]))) return;
  T[0] = U[0];"""
assert a in s; s = s.replace(a, b)
a = """      : "vcc");
  // second fold: top = R9:R8 (< 3 * 2^32); add top*977 at limb 0 and top*2^32 at limb 1
"""
b = """      : "vcc");
  fm_reduce_top(r, R, R8, R9);
}

FM_DEV void fm_reduce_top(Fe& r, uint32_t R[8], uint32_t R8, uint32_t R9) {
"""
assert a in s; s = s.replace(a, b)
open(p, 'w').write(s)
