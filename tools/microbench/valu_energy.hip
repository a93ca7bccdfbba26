// Energy per instruction class on gfx950 (round 5): each mode keeps the whole chip busy with one instruction form
// (4 waves/SIMD, 16 independent chains per lane, as tools/microbench/valu_cost.hip) or one memory pattern, relaunched
// for `seconds`, and prints its rate; tools/microbench/valu_energy_run.py samples board power around each run and
// turns rate and power into picojoules per lane-instruction (or per byte / per access) above the `sleep` mode (all
// waves resident, `s_sleep`), at the clock the power cap leaves.
//
// Modes: add_u32 mov_b32 alignbit addc_vcc mad64 mad_addc (the field product's pair: v_mad_u64_u32 -> VCC, s_nop 0,
//        v_addc_co_u32) nop fma_f64 sleep | stream (non-temporal 32-B per lane in, 32-B per lane out, [entry][lane]
//        like the prefix scratch) | gather_l2 / gather_mall / gather_hbm (one 8-B load per lane per step from a 2 MiB /
//        32 MiB / 4 GiB table at a hashed index, as the level-0 gate)
// Usage: ./valu_energy <mode> <seconds>
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int ITERS = 4096;
enum { ADD_U32, MOV_B32, ALIGNBIT, ADDC_VCC, MAD64, MAD_ADDC, NOP, FMA_F64, SLEEP, N_ALU };
static const char* kAlu[N_ALU] = {"add_u32", "mov_b32", "alignbit", "addc_vcc", "mad64", "mad_addc", "nop", "fma_f64",
                                  "sleep"};
static const int kPer[N_ALU] = {1, 1, 1, 1, 1, 2, 0, 1, 0};     // VALU instructions per body

template <int OP>
__device__ __forceinline__ void body(uint32_t& x, uint64_t& y, double& f, uint32_t b, uint32_t c) {
  if constexpr (OP == ADD_U32) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));
  if constexpr (OP == MOV_B32) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(b ^ x));
  if constexpr (OP == ALIGNBIT) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x) : "v"(b));
  if constexpr (OP == ADDC_VCC) asm volatile("v_addc_co_u32_e32 %0, vcc, %0, %1, vcc" : "+v"(x) : "v"(b) : "vcc");
  if constexpr (OP == MAD64) { uint64_t s; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(y), "=s"(s) : "v"(b), "v"(c)); }
  if constexpr (OP == MAD_ADDC)
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
                 : "+v"(y), "+v"(x) : "v"(b), "v"(c) : "vcc");
  if constexpr (OP == NOP) asm volatile("s_nop 0");
  if constexpr (OP == FMA_F64) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(f) : "v"((double)b), "v"((double)c));
  if constexpr (OP == SLEEP) asm volatile("s_sleep 1");
}

template <int OP>
__global__ __launch_bounds__(256, 4) void k_alu(uint64_t* out, uint32_t s) {
  const uint32_t b = blockIdx.x * 7 + s, c = threadIdx.x * 5 + s;
  uint32_t x[16];
  uint64_t y[16];
  double f[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) { x[i] = threadIdx.x ^ (s + i); y[i] = (uint64_t)x[i] * 3 + i; f[i] = 1.0 + i; }
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int i = 0; i < 16; ++i) body<OP>(x[i], y[i], f[i], b, c);
  uint64_t r = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) r ^= x[i] ^ y[i] ^ (uint64_t)f[i];
  if (r == 0x12345) out[0] = r;
}

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
// the prefix scratch's pattern: [entry][lane] 32-B entries, non-temporal; per step each lane stores one entry and
// loads one written `lag` entries earlier (streaming, no reuse)
__global__ __launch_bounds__(256, 4) void k_stream(v4u* buf, uint32_t entries, uint32_t lanes, uint64_t* out) {
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  v4u acc = {lane, 1u, 2u, 3u};
  for (uint32_t e = 0; e < entries; ++e) {
    v4u* p = buf + 2 * ((size_t)e * lanes + lane);
    __builtin_nontemporal_store(acc, p);
    __builtin_nontemporal_store(acc + 1u, p + 1);
    const uint32_t r = e >= 512 ? e - 512 : e;
    const v4u* q = buf + 2 * ((size_t)r * lanes + lane);
    acc ^= __builtin_nontemporal_load(q) + __builtin_nontemporal_load(q + 1);
  }
  if (acc.x == 0x12345u) out[0] = acc.y;
}

// the level-0 gate's pattern: one 8-B load per lane per step at a hashed index in a table of (mask + 1) words
__global__ __launch_bounds__(256, 4) void k_gather(const uint2* tab, uint32_t mask, uint32_t steps, uint64_t* out) {
  uint32_t h = (blockIdx.x * blockDim.x + threadIdx.x) * 0x9E3779B9u + 1u, acc = 0;
  for (uint32_t i = 0; i < steps; ++i) {
    h ^= h << 13; h ^= h >> 17; h ^= h << 5;          // xorshift32: the next random block index
    const uint2 w = tab[h & mask];                    // independent loads: the gate's loads do not chain
    acc += w.x ^ w.y;
  }
  if (acc == 0x12345u) out[0] = acc;
}

int main(int argc, char** argv) {
  if (argc < 3) { printf("usage: valu_energy <mode> <seconds>\n"); return 2; }
  const std::string mode = argv[1];
  const double secs = atof(argv[2]);
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const uint32_t cus = prop.multiProcessorCount, blocks = cus * 4, lanes = blocks * 256;
  uint64_t* out;
  CHECK(hipMalloc(&out, 64));
  int alu = -1;
  for (int i = 0; i < N_ALU; ++i) if (mode == kAlu[i]) alu = i;
  void* buf = nullptr;
  uint32_t mask = 0, entries = 0, steps = 0;
  if (mode == "stream") {
    entries = 4096;                                     // 32 B x 4096 x 262,144 lanes = 34 GB, as one prefix slot
    CHECK(hipMalloc(&buf, (size_t)32 * entries * lanes));
  } else if (mode.rfind("gather", 0) == 0) {
    const size_t bytes = mode == "gather_l2" ? (2u << 20) : mode == "gather_mall" ? (32u << 20) : ((size_t)4 << 30);
    mask = (uint32_t)(bytes / 8 - 1);
    steps = 4096;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMemset(buf, 0x5a, bytes));
  } else if (alu < 0) {
    printf("unknown mode %s\n", mode.c_str());
    return 2;
  }
  auto launch = [&](uint32_t s) {
    switch (alu) {
#define L(OP) case OP: hipLaunchKernelGGL(k_alu<OP>, dim3(blocks), dim3(256), 0, 0, out, s); return;
      L(ADD_U32) L(MOV_B32) L(ALIGNBIT) L(ADDC_VCC) L(MAD64) L(MAD_ADDC) L(NOP) L(FMA_F64) L(SLEEP)
#undef L
      default: break;
    }
    if (mode == "stream") hipLaunchKernelGGL(k_stream, dim3(blocks), dim3(256), 0, 0, (v4u*)buf, entries, lanes, out);
    else hipLaunchKernelGGL(k_gather, dim3(blocks), dim3(256), 0, 0, (const uint2*)buf, mask, steps, out);
  };
  launch(1);
  CHECK(hipDeviceSynchronize());
  const auto t0 = std::chrono::steady_clock::now();
  double el = 0;
  uint64_t n = 0;
  while ((el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count()) < secs) {
    launch(2 + (uint32_t)n);
    CHECK(hipDeviceSynchronize());
    ++n;
  }
  // units per launch: lane-instructions (ALU), bytes moved (stream), loads (gather)
  double units = 0;
  const char* unit = "lane_instr";
  if (alu >= 0) units = (double)lanes * ITERS * 16 * kPer[alu];
  else if (mode == "stream") { units = (double)lanes * entries * 64; unit = "byte"; }
  else { units = (double)lanes * steps; unit = "load"; }
  if (alu == NOP || alu == SLEEP) units = (double)lanes * ITERS * 16, unit = "lane_slot";
  printf("{\"mode\": \"%s\", \"launches\": %llu, \"seconds\": %.3f, \"unit\": \"%s\", \"units_per_s\": %.6e}\n",
         mode.c_str(), (unsigned long long)n, el, unit, units * n / el);
  return 0;
}
