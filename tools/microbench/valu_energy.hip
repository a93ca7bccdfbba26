// Energy per instruction class on gfx950 (round 5): each mode keeps the whole chip busy with one instruction form
// (4 waves/SIMD, 16 independent chains per lane, as tools/microbench/valu_cost.hip) or one memory pattern, relaunched
// for `seconds`, and prints its rate; tools/microbench/valu_energy_run.py samples board power around each run and
// turns rate and power into picojoules per lane-instruction (or per byte / per access) above the `sleep` mode (all
// waves resident, `s_sleep`), at the clock the power cap leaves.
//
// Modes: add_u32 mov_b32 alignbit addc_vcc mad64 mad_addc (the field product's pair: v_mad_u64_u32 -> VCC, s_nop 0,
//        v_addc_co_u32) nop fma_f64 sleep | stream (non-temporal 32-B per lane in, 32-B per lane out, [entry][lane]
//        like the prefix scratch) | gather_l2 / gather_mall / gather_hbm (one 8-B load per lane per step from a 2 MiB /
//        32 MiB / 4 GiB table at a hashed index, as the level-0 gate) | salu (s_add_u32 chains, per wave-instruction) |
//        smem (s_load_dwordx8 of 32-B rows of a 64 KiB table, wave-uniform: the GSn rows, per wave-load) | lds (one
//        ds_write_b32 + one ds_read_b32 per lane per step, per lane-access) | scratch (one scratch store + one scratch
//        load of 4 B per lane per step into a 256-B private array at a data-dependent index: 64 MiB over the chip, so
//        mostly MALL, per lane-access) | scratch_l2 (8-B reload + store of 8 fixed slots per lane: the product's
//        spill pattern, L2-resident, per lane-access)
//        (round 6: the classes of VERDICT r5 item 5's energy split)
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

// SALU: 16 independent s_add_u32 chains per wave (one wave-instruction each per body)
__global__ __launch_bounds__(256, 4) void k_salu(uint64_t* out, uint32_t s) {
  uint32_t a0 = s, a1 = s + 1, a2 = s + 2, a3 = s + 3, a4 = s + 4, a5 = s + 5, a6 = s + 6, a7 = s + 7;
  uint32_t b0 = s * 3, b1 = s * 5, b2 = s * 7, b3 = s * 9, b4 = s * 11, b5 = s * 13, b6 = s * 15, b7 = s * 17;
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("s_add_u32 %0, %0, %16\n\ts_add_u32 %1, %1, %16\n\ts_add_u32 %2, %2, %16\n\ts_add_u32 %3, %3, %16\n\t"
                 "s_add_u32 %4, %4, %16\n\ts_add_u32 %5, %5, %16\n\ts_add_u32 %6, %6, %16\n\ts_add_u32 %7, %7, %16\n\t"
                 "s_add_u32 %8, %8, %16\n\ts_add_u32 %9, %9, %16\n\ts_add_u32 %10, %10, %16\n\ts_add_u32 %11, %11, %16\n\t"
                 "s_add_u32 %12, %12, %16\n\ts_add_u32 %13, %13, %16\n\ts_add_u32 %14, %14, %16\n\ts_add_u32 %15, %15, %16"
                 : "+s"(a0), "+s"(a1), "+s"(a2), "+s"(a3), "+s"(a4), "+s"(a5), "+s"(a6), "+s"(a7), "+s"(b0), "+s"(b1),
                   "+s"(b2), "+s"(b3), "+s"(b4), "+s"(b5), "+s"(b6), "+s"(b7)
                 : "s"(s)
                 : "scc");
  }
  const uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ b0 ^ b1 ^ b2 ^ b3 ^ b4 ^ b5 ^ b6 ^ b7;
  if (r == 0x12345u && threadIdx.x == 0) out[0] = r;
}

// SMEM: wave-uniform 32-B rows of a 64 KiB table through the constant address space (s_load_dwordx8), as the walk
// reads GSn[i]; the row index walks the table, 8 loads in flight per body
__global__ __launch_bounds__(256, 4) void k_smem(const __attribute__((address_space(4))) uint32_t* tab, uint64_t* out,
                                                 uint32_t s) {
  uint32_t acc = 0;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t row = (uint32_t)(it * 8 + k + s) & 2047u;      // 2048 rows x 32 B = 64 KiB
      const __attribute__((address_space(4))) uint32_t* p = tab + 8 * row;
      acc += p[0] ^ p[1] ^ p[2] ^ p[3] ^ p[4] ^ p[5] ^ p[6] ^ p[7];
    }
  }
  if (acc == 0x12345u) out[0] = acc + threadIdx.x;
}

// LDS: per lane one 4-B write and one 4-B read per step, 16 steps per body (the survivor queue's accesses)
__global__ __launch_bounds__(256, 4) void k_lds(uint64_t* out, uint32_t s) {
  __shared__ uint32_t buf[256 * 16];
  uint32_t acc = threadIdx.x ^ s;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      volatile __attribute__((address_space(3))) uint32_t* q =
          (volatile __attribute__((address_space(3))) uint32_t*)(buf + k * 256 + threadIdx.x);
      *q = acc + k;
      acc ^= *q;
    }
  }
  if (acc == 0x12345u) out[0] = acc;
}

// scratch: per lane one 4-B store and one 4-B load of a private array indexed by a runtime value (the compiler
// keeps it in scratch memory: the spill pattern, which the product's waves reach through the L1/L2)
__global__ __launch_bounds__(256, 4) void k_scratch(uint64_t* out, uint32_t s) {
  uint32_t arr[64];
  volatile __attribute__((address_space(5))) uint32_t* priv = (volatile __attribute__((address_space(5))) uint32_t*)arr;
  uint32_t acc = threadIdx.x ^ s;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t i = (acc + (uint32_t)k) & 63u;
      priv[i] = acc;
      acc += priv[(i + 7u) & 63u];
    }
  }
  if (acc == 0x12345u) out[0] = acc;
}

// scratch_l2: the product's spill pattern -- a few fixed 8-B slots per lane (8 here, 64 B per lane: 16 MiB over the
// chip, 2 MiB per XCD, L2-resident), stored and reloaded at fixed offsets
__global__ __launch_bounds__(256, 4) void k_scratch_l2(uint64_t* out, uint32_t s) {
  uint64_t arr[8];
  volatile __attribute__((address_space(5))) uint64_t* priv = (volatile __attribute__((address_space(5))) uint64_t*)arr;
  uint64_t acc = threadIdx.x ^ s;
#pragma unroll
  for (int k = 0; k < 8; ++k) priv[k] = acc + k;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      acc += priv[k & 7];
      priv[(k + 3) & 7] = acc;
    }
  }
  if (acc == 0x12345u) out[0] = acc;
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
  } else if (mode == "smem") {
    CHECK(hipMalloc(&buf, 64 * 1024));
    CHECK(hipMemset(buf, 0x3c, 64 * 1024));
  } else if (alu < 0 && mode != "salu" && mode != "lds" && mode != "scratch" && mode != "scratch_l2") {
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
    else if (mode == "salu") hipLaunchKernelGGL(k_salu, dim3(blocks), dim3(256), 0, 0, out, s);
    else if (mode == "smem")
      hipLaunchKernelGGL(k_smem, dim3(blocks), dim3(256), 0, 0,
                         (const __attribute__((address_space(4))) uint32_t*)buf, out, s);
    else if (mode == "lds") hipLaunchKernelGGL(k_lds, dim3(blocks), dim3(256), 0, 0, out, s);
    else if (mode == "scratch") hipLaunchKernelGGL(k_scratch, dim3(blocks), dim3(256), 0, 0, out, s);
    else if (mode == "scratch_l2") hipLaunchKernelGGL(k_scratch_l2, dim3(blocks), dim3(256), 0, 0, out, s);
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
  else if (mode == "salu") { units = (double)(lanes / 64) * ITERS * 16; unit = "wave_instr"; }
  else if (mode == "smem") { units = (double)(lanes / 64) * ITERS * 8; unit = "wave_load_32B"; }
  else if (mode == "lds" || mode == "scratch") { units = (double)lanes * ITERS * 16 * 2; unit = "lane_access_4B"; }
  else if (mode == "scratch_l2") { units = (double)lanes * ITERS * 16 * 2; unit = "lane_access_8B"; }
  else { units = (double)lanes * steps; unit = "load"; }
  if (alu == NOP || alu == SLEEP) units = (double)lanes * ITERS * 16, unit = "lane_slot";
  printf("{\"mode\": \"%s\", \"launches\": %llu, \"seconds\": %.3f, \"unit\": \"%s\", \"units_per_s\": %.6e}\n",
         mode.c_str(), (unsigned long long)n, el, unit, units * n / el);
  return 0;
}
