# Timing-only patch for tools/experiments/calib_build.sh (see there); edits fe_asm.hpp in place.
p='keyhuntm1cpu_amd/csrc/device/fe_asm.hpp'
s=open(p).read()
a="""FM_DEV void fm_mul(Fe& r, const Fe& a, const Fe& b) {
  uint32_t t[16];
  fm_mul512x(t, a.v, b.v);
  fm_reduce(r, t);
}"""
b="""#ifndef KHB_PAD_N
#define KHB_PAD_N 0
#endif
#ifndef KHB_PAD_OP
#define KHB_PAD_OP 0
#endif
template <int OP>
FM_DEV void fm_pad1(uint64_t& y, uint32_t& x, uint32_t b, uint32_t c) {
  if constexpr (OP == 1) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(b));
  if constexpr (OP == 2) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));
  if constexpr (OP == 3) asm volatile("v_add_co_u32_e32 %0, vcc, %0, %1" : "+v"(x) : "v"(b) : "vcc");
  if constexpr (OP == 4) asm volatile("v_addc_co_u32_e32 %0, vcc, %0, %1, vcc" : "+v"(x) : "v"(b) : "vcc");
  if constexpr (OP == 5) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(y) : "v"(b), "v"(c) : "vcc");
  if constexpr (OP == 6) { uint64_t s; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(y), "=s"(s) : "v"(b), "v"(c)); }
  if constexpr (OP == 7) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));
  if constexpr (OP == 8) asm volatile("s_nop 0");
  if constexpr (OP == 9) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
}
FM_DEV void fm_mul(Fe& r, const Fe& a, const Fe& b) {
  uint32_t t[16];
  fm_mul512x(t, a.v, b.v);
  fm_reduce(r, t);
  uint64_t y[4] = {r.v[7], r.v[6], r.v[5], r.v[4]};
  uint32_t x[4] = {r.v[3], r.v[2], r.v[1], r.v[0]};
#pragma unroll
  for (int i = 0; i < KHB_PAD_N; ++i) fm_pad1<KHB_PAD_OP>(y[i & 3], x[i & 3], a.v[i & 7], b.v[(i + 1) & 7]);
  asm volatile("" :: "v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3]), "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]));
}"""
assert a in s; s=s.replace(a,b); open(p,'w').write(s)
