# Timing-only patch for tools/experiments/calib_build.sh (see there); edits fe_asm.hpp in place.
p='keyhuntm1cpu_amd/csrc/device/fe_asm.hpp'
s=open(p).read()
# rmFold: the 15-add fold chain of the product columns -> full-rate xors (timing only)
a="""FM_DEV void fm_fold_cols(uint32_t t[16], const uint64_t A[15], uint32_t cw13) {
#define FM_LO(k) "v"((uint32_t)A[k])"""
b="""FM_DEV void fm_fold_cols(uint32_t t[16], const uint64_t A[15], uint32_t cw13) {
#if KHB_RM_FOLD
  t[0] = (uint32_t)A[0];
#pragma unroll
  for (int k = 1; k < 15; ++k) t[k] = (uint32_t)A[k] ^ (uint32_t)(A[k - 1] >> 32);
  t[15] = cw13 ^ (uint32_t)(A[14] >> 32);
  return;
#endif
#define FM_LO(k) "v"((uint32_t)A[k])"""
assert a in s; s=s.replace(a,b)
a="""  uint64_t P[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) P[i] = (uint64_t)H[i] * 977u + T[i];"""
b="""  uint64_t P[8];
#if KHB_RM_P
#pragma unroll
  for (int i = 0; i < 8; ++i) P[i] = ((uint64_t)(H[i] >> 22) << 32) | (H[i] ^ T[i]);
#else
#pragma unroll
  for (int i = 0; i < 8; ++i) P[i] = (uint64_t)H[i] * 977u + T[i];
#endif"""
assert a in s; s=s.replace(a,b)
a="""  uint32_t T[10];
  asm("v_mov_b32 %0, %10\\n\\t\""""
b="""  uint32_t T[10];
#if KHB_RM_T
  T[0] = L[0];
#pragma unroll
  for (int i = 1; i < 8; ++i) T[i] = L[i] ^ H[i - 1];
  T[8] = H[7] >> 31;
  T[9] = 0;
  fm_reduce_T(r, T, H);
  return;
#endif
  asm("v_mov_b32 %0, %10\\n\\t\""""
assert a in s, 'T'; s=s.replace(a,b)
open(p,'w').write(s)
