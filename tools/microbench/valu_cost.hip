// VALU issue cost per instruction class on gfx950, as the field arithmetic uses them.
//
// For each instruction form: CH independent chains per lane (CH = 1: one dependent chain = latency
// bound at one wave per SIMD), W waves per SIMD.  Reported: SIMD cycles per wave-instruction
// (4 SIMDs x 64 lanes / lane-instructions per clock per CU), from HIP events and the shader clock
// (s_memtime vs s_memrealtime at 100 MHz).  Pairs ("mad+addc") count both instructions.
//
// Questions it answers (DESIGN.md §5 issue-slot model): does a VCC-writing VOP2 (v_add_co_u32_e32,
// v_addc_co_u32_e32) issue like v_add_u32 or like a VOP3 (v_mad_u64_u32)?  What does an `s_nop 0`
// between a carry write and its reader cost at 4 waves/SIMD?  How long is a dependent
// v_mad_u64_u32 accumulation chain?
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"

#define ITERS 512
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

enum {
  ADD_U32, MOV_B32, AND_B32, LSHR_B32, ADD_CO_E32, ADDC_E32, ADDC_E32_NOP, ADD_CO_E64, ADDC_E64, MAD64, MAD64_VCC,
  MAD_ADDC_NOP, MAD_ADDC, MUL_LO, MUL_HI, MUL_U24, MULHI_U24, MAD_U24, ADD3, ALIGNBIT, LSHR_B64, LSHL_ADD_U64, CNDMASK,
  BITOP3, BFE, LSHL_OR, AND_OR, PERM, SUB_CO_E32, NOP_ONLY, CND_VCMP, CND_E64, CMP_CND, MAD_ADDU, MAD_2ADDU, ADDC_ADDU, MAD_BANK_SAME, MAD_BANK_DIFF, MAD_BITOP3, N_OPS
};
static const char* kNames[N_OPS] = {
  "v_add_u32", "v_mov_b32", "v_and_b32", "v_lshrrev_b32", "v_add_co_u32_e32(vcc)", "v_addc_co_u32_e32(vcc chain)",
  "v_addc_co_u32_e32+s_nop0", "v_add_co_u32_e64(sgpr)", "v_addc_co_u32_e64(own sgpr)", "v_mad_u64_u32(own sgpr)",
  "v_mad_u64_u32(vcc)", "mad+nop+addc(vcc) pair", "mad+addc(e64 own sgpr) pair", "v_mul_lo_u32", "v_mul_hi_u32",
  "v_mul_u32_u24", "v_mul_hi_u32_u24", "v_mad_u32_u24", "v_add3_u32", "v_alignbit_b32", "v_lshrrev_b64",
  "v_lshl_add_u64", "v_cndmask_b32(vcc)", "v_bitop3_b32", "v_bfe_u32", "v_lshl_or_b32", "v_and_or_b32", "v_perm_b32",
  "v_sub_co_u32_e32(vcc)", "s_nop 0 only", "v_cndmask_b32(vcc from v_cmp)", "v_cndmask_b32_e64(sgpr v_cmp)",
  "v_cmp+v_cndmask pair", "mad + v_add_u32 pair", "mad + 2 v_add_u32", "addc(e64) + v_add_u32 pair",
  "mad srcs same bank (fixed regs)", "mad srcs 4 banks (fixed regs)", "mad + v_bitop3 pair"};
// instructions counted per body (pairs count 2; NOP_ONLY counts the nop)
static int kPer[N_OPS];

template <int OP>
__device__ __forceinline__ void body(uint32_t& x, uint64_t& y, uint64_t& sc, uint32_t b, uint32_t c) {
  if constexpr (OP == ADD_U32) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));
  if constexpr (OP == MOV_B32) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(b));
  if constexpr (OP == AND_B32) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(b));
  if constexpr (OP == LSHR_B32) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(x) : "v"(b));
  if constexpr (OP == ADD_CO_E32) asm volatile("v_add_co_u32_e32 %0, vcc, %0, %1" : "+v"(x) : "v"(b) : "vcc");
  if constexpr (OP == ADDC_E32) asm volatile("v_addc_co_u32_e32 %0, vcc, %0, %1, vcc" : "+v"(x) : "v"(b) : "vcc");
  if constexpr (OP == ADDC_E32_NOP) asm volatile("s_nop 0\n\tv_addc_co_u32_e32 %0, vcc, %0, %1, vcc" : "+v"(x) : "v"(b) : "vcc");
  if constexpr (OP == ADD_CO_E64) { uint64_t s; asm volatile("v_add_co_u32_e64 %0, %1, %0, %2" : "+v"(x), "=s"(s) : "v"(b)); }
  if constexpr (OP == ADDC_E64) { asm volatile("v_addc_co_u32_e64 %0, %1, %0, %2, %1" : "+v"(x), "+s"(sc) : "v"(b)); }
  if constexpr (OP == MAD64) { uint64_t s; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(y), "=s"(s) : "v"(b), "v"(c)); }
  if constexpr (OP == MAD64_VCC) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(y) : "v"(b), "v"(c) : "vcc");
  if constexpr (OP == MAD_ADDC_NOP)
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
                 : "+v"(y), "+v"(x) : "v"(b), "v"(c) : "vcc");
  if constexpr (OP == MAD_ADDC) {
    uint64_t s;
    asm volatile("v_mad_u64_u32 %0, %2, %3, %4, %0\n\tv_addc_co_u32_e64 %1, %2, 0, %1, %2"
                 : "+v"(y), "+v"(x), "=&s"(s) : "v"(b), "v"(c));
  }
  if constexpr (OP == MUL_LO) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));
  if constexpr (OP == MUL_HI) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(b));
  if constexpr (OP == MUL_U24) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(b));
  if constexpr (OP == MULHI_U24) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(x) : "v"(b));
  if constexpr (OP == MAD_U24) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
  if constexpr (OP == ADD3) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
  if constexpr (OP == ALIGNBIT) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x) : "v"(b));
  if constexpr (OP == LSHR_B64) asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(y));
  if constexpr (OP == LSHL_ADD_U64) asm volatile("v_lshl_add_u64 %0, %0, 1, %0" : "+v"(y));
  if constexpr (OP == CNDMASK) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(x) : "v"(b));
  if constexpr (OP == BITOP3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(b), "v"(c));
  if constexpr (OP == BFE) asm volatile("v_bfe_u32 %0, %0, 3, 20" : "+v"(x));
  if constexpr (OP == LSHL_OR) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(x) : "v"(b));
  if constexpr (OP == AND_OR) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
  if constexpr (OP == PERM) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
  if constexpr (OP == SUB_CO_E32) asm volatile("v_sub_co_u32_e32 %0, vcc, %0, %1" : "+v"(x) : "v"(b) : "vcc");
  if constexpr (OP == NOP_ONLY) asm volatile("s_nop 0");
  if constexpr (OP == CND_VCMP) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(x) : "v"(b));
  if constexpr (OP == CND_E64) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x) : "v"(b), "s"(sc));
  if constexpr (OP == MAD_ADDU) {
    uint64_t sg;
    asm volatile("v_mad_u64_u32 %0, %2, %3, %4, %0\n\tv_add_u32 %1, %1, %3" : "+v"(y), "+v"(x), "=s"(sg) : "v"(b), "v"(c));
  }
  if constexpr (OP == MAD_2ADDU) {
    uint64_t sg;
    asm volatile("v_mad_u64_u32 %0, %2, %3, %4, %0\n\tv_add_u32 %1, %1, %3\n\tv_xor_b32 %1, %1, %4"
                 : "+v"(y), "+v"(x), "=s"(sg) : "v"(b), "v"(c));
  }
  if constexpr (OP == ADDC_ADDU)
    asm volatile("v_addc_co_u32_e64 %0, %2, %0, %3, %2\n\tv_add_u32 %1, %1, %3" : "+v"(x), "+v"(c), "+s"(sc) : "v"(b));
  if constexpr (OP == MAD_BANK_SAME)
    asm volatile("v_mad_u64_u32 v[40:41], s[40:41], v44, v48, v[40:41]" ::: "v40", "v41", "v44", "v48", "s40", "s41");
  if constexpr (OP == MAD_BANK_DIFF)
    asm volatile("v_mad_u64_u32 v[40:41], s[40:41], v45, v46, v[40:41]" ::: "v40", "v41", "v45", "v46", "s40", "s41");
  if constexpr (OP == MAD_BITOP3) {
    uint64_t sg;
    asm volatile("v_mad_u64_u32 %0, %2, %3, %4, %0\n\tv_bitop3_b32 %1, %1, %3, %4 bitop3:0x96" : "+v"(y), "+v"(x), "=s"(sg) : "v"(b), "v"(c));
  }
  if constexpr (OP == CMP_CND)
    asm volatile("v_cmp_gt_u32_e32 vcc, %0, %1\n\ts_nop 1\n\tv_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(x) : "v"(b) : "vcc");
}

template <int OP, int CH>
__global__ __launch_bounds__(256) void k(uint64_t* out, uint64_t* clk, uint32_t s) {
  uint32_t b = blockIdx.x * 7 + s, c = threadIdx.x * 5 + s;
  uint32_t x[CH];
  uint64_t y[CH], sc[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) { x[i] = threadIdx.x ^ (s + i); y[i] = (uint64_t)x[i] * 3 + i; sc[i] = 0; }
  if constexpr (OP == CNDMASK) asm volatile("s_mov_b32 vcc_lo, 0x55555555\n\ts_mov_b32 vcc_hi, 0x55555555" ::: "vcc");
  if constexpr (OP == CND_VCMP) asm volatile("v_cmp_gt_u32_e32 vcc, %0, %1\n\ts_nop 4" :: "v"(x[0]), "v"(c) : "vcc");
  if constexpr (OP == CND_E64) {
#pragma unroll
    for (int i = 0; i < CH; ++i) asm volatile("v_cmp_gt_u32_e64 %0, %1, %2\n\ts_nop 4" : "=s"(sc[i]) : "v"(x[0]), "v"(c));
  }
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int u = 0; u < 16 / CH; ++u)
#pragma unroll
      for (int i = 0; i < CH; ++i) body<OP>(x[i], y[i], sc[i], b, c);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint64_t r = 0;
#pragma unroll
  for (int i = 0; i < CH; ++i) r ^= x[i] ^ y[i] ^ sc[i];
  if (r == 0x12345) out[0] = r;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

// cycles per wave-instruction on one SIMD
template <int OP, int CH>
double run(uint64_t* d, uint64_t* clk, int cus, int waves, int per) {
  const int blocks = cus * waves, threads = 256;   // a 256-thread block = one wave on each of a CU's 4 SIMDs
  hipLaunchKernelGGL((k<OP, CH>), dim3(blocks), dim3(threads), 0, 0, d, clk, 1u);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k<OP, CH>), dim3(blocks), dim3(threads), 0, 0, d, clk, 2u + r);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  uint64_t h[2];
  hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
  const double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
  const double wave_inst_per_simd = (double)reps * waves * ITERS * 16 * per;   // per SIMD (blocks spread over CUs)
  const double cycles = ms * 1e-3 * ghz * 1e9;
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return cycles / wave_inst_per_simd;
}

template <int OP>
int row(uint64_t* d, uint64_t* clk, int cus, int per) {
  kPer[OP] = per;
  const double w4 = run<OP, 16>(d, clk, cus, 4, per), w8 = run<OP, 16>(d, clk, cus, 8, per);
  const double w1 = run<OP, 16>(d, clk, cus, 1, per), lat1 = run<OP, 1>(d, clk, cus, 1, per);
  const double lat4 = run<OP, 1>(d, clk, cus, 4, per), ch2w4 = run<OP, 2>(d, clk, cus, 4, per);
  printf("%-32s %7.2f %7.2f %7.2f | %7.2f %7.2f %7.2f\n", kNames[OP], w4, w8, w1, lat1, lat4, ch2w4);
  return 0;
}

int main() {
  uint64_t *d, *clk;
  CHECK(hipMalloc(&d, 64));
  CHECK(hipMalloc(&clk, 64));
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  printf("device %s CUs %d; SIMD cycles per wave-instruction\n", p.gcnArchName, cus);
  printf("%-32s %7s %7s %7s | %7s %7s %7s\n", "instruction", "16ch/w4", "16ch/w8", "16ch/w1", "1ch/w1", "1ch/w4",
         "2ch/w4");
  row<ADD_U32>(d, clk, cus, 1); row<MOV_B32>(d, clk, cus, 1); row<AND_B32>(d, clk, cus, 1);
  row<LSHR_B32>(d, clk, cus, 1); row<ADD_CO_E32>(d, clk, cus, 1); row<SUB_CO_E32>(d, clk, cus, 1);
  row<ADDC_E32>(d, clk, cus, 1); row<ADDC_E32_NOP>(d, clk, cus, 1); row<ADD_CO_E64>(d, clk, cus, 1);
  row<ADDC_E64>(d, clk, cus, 1); row<MAD64>(d, clk, cus, 1); row<MAD64_VCC>(d, clk, cus, 1);
  row<MAD_ADDC_NOP>(d, clk, cus, 2); row<MAD_ADDC>(d, clk, cus, 2); row<MUL_LO>(d, clk, cus, 1);
  row<MUL_HI>(d, clk, cus, 1); row<MUL_U24>(d, clk, cus, 1); row<MULHI_U24>(d, clk, cus, 1);
  row<MAD_U24>(d, clk, cus, 1); row<ADD3>(d, clk, cus, 1); row<ALIGNBIT>(d, clk, cus, 1);
  row<LSHR_B64>(d, clk, cus, 1); row<LSHL_ADD_U64>(d, clk, cus, 1); row<CNDMASK>(d, clk, cus, 1);
  row<BITOP3>(d, clk, cus, 1); row<BFE>(d, clk, cus, 1); row<LSHL_OR>(d, clk, cus, 1);
  row<AND_OR>(d, clk, cus, 1); row<PERM>(d, clk, cus, 1); row<NOP_ONLY>(d, clk, cus, 1);
  row<CND_VCMP>(d, clk, cus, 1); row<CND_E64>(d, clk, cus, 1); row<CMP_CND>(d, clk, cus, 2);
  row<MAD_ADDU>(d, clk, cus, 2); row<MAD_2ADDU>(d, clk, cus, 3); row<ADDC_ADDU>(d, clk, cus, 2);
  row<MAD_BANK_SAME>(d, clk, cus, 1); row<MAD_BANK_DIFF>(d, clk, cus, 1); row<MAD_BITOP3>(d, clk, cus, 2);
  return 0;
}
