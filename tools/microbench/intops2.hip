// VALU issue-rate microbenchmark for gfx950 with in-kernel clock measurement.
// 8 waves/SIMD (2048 threads/CU), 16 independent chains per lane; each kernel reports
// lane-instructions per cycle per CU using s_memtime (shader clock) / s_memrealtime (100 MHz).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 1024
#define CH 16
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int OP>
__global__ __launch_bounds__(256) void k(uint64_t* out, uint64_t* clk, uint32_t s) {
  uint32_t a = threadIdx.x ^ s, b = blockIdx.x * 7 + s;
  uint32_t acc[CH];
  uint64_t acc64[CH];
  for (int i = 0; i < CH; ++i) { acc[i] = a + i; acc64[i] = a * 3 + i; }
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(b));
      if (OP == 1) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(acc[i]) : "v"(b));
      if (OP == 2) { uint64_t cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc64[i]), "=s"(cc) : "v"(a), "v"(b)); }
      if (OP == 3) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(b));
      if (OP == 4) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(b));
      if (OP == 5) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(acc[i]) : "v"(b) : "vcc");
      if (OP == 6) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(acc[i]) : "v"(b) : "vcc");
      if (OP == 7) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(acc[i]) : "v"(b));
      if (OP == 8) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(acc[i]) : "v"(b));
      if (OP == 9) asm volatile("v_lshl_add_u64 %0, %0, 1, %0" : "+v"(acc64[i]));
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint64_t r = 0;
  for (int i = 0; i < CH; ++i) r ^= acc[i] ^ acc64[i];
  if (r == 0x12345) out[0] = r;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

const char* names[] = {"v_add_u32", "v_add3_u32", "v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32",
                       "v_add_co_u32", "v_addc_co_u32", "v_cndmask_b32", "v_alignbit_b32", "v_lshl_add_u64"};

template <int OP>
int run(uint64_t* d, uint64_t* clk, int cus) {
  int blocks = cus * 8, threads = 256;
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(threads), 0, 0, d, clk, 1u);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  const int reps = 10;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(threads), 0, 0, d, clk, 2u + r);
  CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  uint64_t h[2]; CHECK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
  double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
  double lane_inst = (double)reps * blocks * threads * ITERS * CH;
  double per_s = lane_inst / (ms * 1e-3);
  printf("%-16s %8.3f ms  %7.2f T lane-inst/s  clk %.2f GHz  %6.1f lane-inst/clk/CU\n", names[OP], ms, per_s / 1e12, ghz,
         per_s / (ghz * 1e9) / cus);
  return 0;
}
int main() {
  uint64_t *d, *clk; CHECK(hipMalloc(&d, 64)); CHECK(hipMalloc(&clk, 64));
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs %d\n", p.gcnArchName, p.multiProcessorCount);
  int cus = p.multiProcessorCount;
  run<0>(d, clk, cus); run<1>(d, clk, cus); run<2>(d, clk, cus); run<3>(d, clk, cus); run<4>(d, clk, cus);
  run<5>(d, clk, cus); run<6>(d, clk, cus); run<7>(d, clk, cus); run<8>(d, clk, cus); run<9>(d, clk, cus);
  return 0;
}
