// Integer VALU throughput microbenchmark for gfx950 (design input for the Fp kernels).
// Each kernel runs 8 independent chains per lane of one instruction kind (inline asm so the
// compiler cannot substitute), reports lane-ops/s. Results go to DESIGN.md.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <chrono>

#define ITERS 2048
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_mad64(uint64_t* out, uint32_t s) {
  uint32_t a = threadIdx.x ^ s, b = blockIdx.x * 7 + s;
  uint64_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      { uint64_t cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[i]), "=s"(cc) : "v"(a), "v"(b)); }
  }
  uint64_t r = 0; for (int i = 0; i < 8; ++i) r ^= acc[i];
  if (r == 0x12345) out[0] = r;
}
__global__ void k_mullo(uint64_t* out, uint32_t s) {
  uint32_t a = threadIdx.x ^ s, b = blockIdx.x * 7 + s;
  uint32_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(b));
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= acc[i];
  if (r == 0x12345) out[0] = r;
}
__global__ void k_mulhi(uint64_t* out, uint32_t s) {
  uint32_t a = threadIdx.x ^ s, b = blockIdx.x * 7 + s;
  uint32_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(b));
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= acc[i];
  if (r == 0x12345) out[0] = r;
}
__global__ void k_mul24(uint64_t* out, uint32_t s) {
  uint32_t a = threadIdx.x ^ s, b = blockIdx.x * 7 + s;
  uint32_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(acc[i]) : "v"(b));
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= acc[i];
  if (r == 0x12345) out[0] = r;
}
__global__ void k_addc(uint64_t* out, uint32_t s) {
  uint32_t a = threadIdx.x ^ s, b = blockIdx.x * 7 + s;
  uint32_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(acc[i]) : "v"(b) : "vcc");
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= acc[i];
  if (r == 0x12345) out[0] = r;
}
__global__ void k_add3(uint64_t* out, uint32_t s) {
  uint32_t a = threadIdx.x ^ s, b = blockIdx.x * 7 + s;
  uint32_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(acc[i]) : "v"(b));
  }
  uint32_t r = 0; for (int i = 0; i < 8; ++i) r ^= acc[i];
  if (r == 0x12345) out[0] = r;
}
__global__ void k_fma64(uint64_t* out, uint32_t s) {
  double a = threadIdx.x ^ s, b = blockIdx.x * 7 + s;
  double acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(acc[i]) : "v"(b));
  }
  double r = 0; for (int i = 0; i < 8; ++i) r += acc[i];
  if (r == 1.2345) out[0] = 1;
}

typedef void (*kfn)(uint64_t*, uint32_t);
int run(const char* name, kfn k, int insts_per_chain_iter, uint64_t* d) {
  int blocks = 256 * 8, threads = 256;
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 2u + r);
  CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  double ops = 5.0 * blocks * threads * (double)ITERS * 8 * insts_per_chain_iter;
  printf("%-8s %8.3f ms  %8.2f T lane-inst/s  (%.1f lane-inst/clk/CU at 2.4GHz)\n", name, ms, ops / (ms * 1e-3) / 1e12,
         ops / (ms * 1e-3) / 2.4e9 / 256);
  return 0;
}
int main() {
  uint64_t* d; CHECK(hipMalloc(&d, 64));
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs %d clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  run("mad64", k_mad64, 1, d);
  run("mullo", k_mullo, 1, d);
  run("mulhi", k_mulhi, 1, d);
  run("mad24", k_mul24, 1, d);
  run("add+addc", k_addc, 2, d);
  run("add3", k_add3, 1, d);
  run("fma64", k_fma64, 1, d);
  return 0;
}
