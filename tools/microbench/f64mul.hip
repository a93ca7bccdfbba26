// Timing-only 256-bit mod-p product on v_fma_f64, against the product's fm_mul.
//
// Representation: five 52-bit limbs held as exact doubles, value < 2^260, congruent mod p = 2^256 - 2^32 - 977.
// Product (IntMod.cpp:855-975 computes the same a*b mod p in 64-bit limbs):
//   * 25 partial products a_i * b_j < 2^104, each split exactly by two FMAs: ph = fma(a, b, 2^104) puts
//     m = round(a*b / 2^52) in ph's mantissa; lo = fma(a, b, -(ph - 2^104)) is the exact remainder,
//     |lo| <= 2^51.  lo + 3*2^51 is a double in [2^52, 2^53) whose mantissa field is lo + 2^51.  Both are
//     accumulated as 64-bit integer bit patterns (the constant offsets removed once per column), so every
//     column sum is exact (< 2^55 in magnitude);
//   * one normalisation pass to ten 52-bit limbs (64-bit add, mask, arithmetic shift);
//   * the fold 2^260 = 16 * (2^32 + 977) = 2^36 + 15632 (mod p): each high limb h times K = 2^36 + 15632 by
//     the same exact two-product, into the low limbs; a second fold of the 37-bit overflow limb; a rare third
//     (wave-uniform branch) when the result still reaches 2^260;
//   * back to doubles by the exponent trick (limb | 0x43300000_00000000) - 2^52.
// fm_mul (device/fe_asm.hpp) is the product's 8 x 32-bit product (64 v_mad_u64_u32 + VCC carry chains + the
// 2^256 = 2^32 + 977 fold).
//
// Modes: ./f64mul verify <n> <out.bin>   one product per lane on seeded inputs; writes x, y, out limbs
//                                        (u64 x 5 each) for tools/microbench/f64mul_check.py (Python big ints)
//        ./f64mul time <f64|u32> <seconds>  full residency (4 waves/SIMD), ITER dependent products per lane in
//                                        CHAINS independent chains, relaunched for `seconds`; prints products/s,
//                                        SIMD cycles per product and the shader clock (s_memtime/s_memrealtime)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "device/fe_asm.hpp"

#pragma clang diagnostic ignored "-Wunused-result"
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace khb;

constexpr int ITER = 256;
constexpr int CHAINS = 2;
constexpr uint64_t M52 = (1ull << 52) - 1;
constexpr double C1 = 20282409603651670423947251286016.0;    // 2^104
constexpr double C2 = 6755399441055744.0;                     // 3 * 2^51
constexpr double KF = 68719492368.0;                          // 2^36 + 15632 = 2^260 mod p
constexpr double TWO52 = 4503599627370496.0;

struct F52 {
  double l[5];
};

__device__ __forceinline__ uint64_t dbits(double d) { return (uint64_t)__double_as_longlong(d); }
__device__ __forceinline__ double from_bits(uint64_t b) { return __longlong_as_double((long long)b); }
// a limb < 2^52 as an exact double: (2^52 + r) - 2^52
__device__ __forceinline__ double limb_to_d(uint64_t r) { return from_bits(r | 0x4330000000000000ull) - TWO52; }

// exact a*b = m * 2^52 + lo for a, b < 2^52: returns the bit patterns of fma(a, b, 2^104) and lo + 3*2^51
__device__ __forceinline__ void two_prod(double a, double b, uint64_t& mb, uint64_t& lb) {
  const double ph = __fma_rn(a, b, C1);
  const double h = ph - C1;
  const double lo = __fma_rn(a, b, -h);
  mb = dbits(ph);
  lb = dbits(lo + C2);
}

__device__ __forceinline__ void normalise(int64_t* t, int n) {
  int64_t c = 0;
#pragma unroll
  for (int k = 0; k < n; ++k) {
    const int64_t v = t[k] + c;
    t[k] = v & (int64_t)M52;
    c = v >> 52;
  }
  t[n] += c;
}

__device__ __forceinline__ void f52_mul(F52& r, const F52& a, const F52& b) {
  const uint64_t B1 = 0x4670000000000000ull, B2 = 0x4338000000000000ull;    // bits(2^104), bits(3 * 2^51)
  uint64_t L[9] = {0}, M[10] = {0};
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      uint64_t mb, lb;
      two_prod(a.l[i], b.l[j], mb, lb);
      L[i + j] += lb;
      M[i + j + 1] += mb;
    }
  int64_t t[11];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    const int nl = k < 9 ? (k < 5 ? k + 1 : 9 - k) : 0;          // lo terms of column k
    const int nm = k >= 1 ? (k - 1 < 5 ? k : 10 - k) : 0;         // hi terms from column k - 1
    t[k] = (int64_t)((k < 9 ? L[k] : 0) - nl * B2) + (int64_t)(M[k] - nm * B1);
  }
  t[10] = 0;
  normalise(t, 10);                                  // ten 52-bit limbs, t[10] = 0 for inputs < 2^260
  // fold limbs 5..9 (x 2^260) by K = 2^36 + 15632
  int64_t u[7] = {t[0], t[1], t[2], t[3], t[4], 0, 0};
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    uint64_t mb, lb;
    two_prod(limb_to_d((uint64_t)t[5 + i]), KF, mb, lb);
    u[i] += (int64_t)(lb - B2);
    u[i + 1] += (int64_t)(mb - B1);
  }
  normalise(u, 6);                                   // u[5] < 2^38, u[6] = 0
  {
    uint64_t mb, lb;
    two_prod(limb_to_d((uint64_t)u[5]), KF, mb, lb);
    u[0] += (int64_t)(lb - B2);
    u[1] += (int64_t)(mb - B1);
    u[5] = 0;
    normalise(u, 5);
  }
  while (__builtin_expect(__ballot(u[5] != 0) != 0, 0)) {   // rare: still >= 2^260
    uint64_t mb, lb;
    two_prod(limb_to_d((uint64_t)u[5]), KF, mb, lb);
    u[0] += (int64_t)(lb - B2);
    u[1] += (int64_t)(mb - B1);
    u[5] = 0;
    normalise(u, 5);
  }
#pragma unroll
  for (int k = 0; k < 5; ++k) r.l[k] = limb_to_d((uint64_t)u[k]);
}

__global__ void k_verify(const uint64_t* x, const uint64_t* y, uint64_t* out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  F52 a, b, r;
  for (int k = 0; k < 5; ++k) {
    a.l[k] = (double)x[5 * i + k];
    b.l[k] = (double)y[5 * i + k];
  }
  f52_mul(r, a, b);
  for (int k = 0; k < 5; ++k) out[5 * i + k] = (uint64_t)r.l[k];
}

__device__ __forceinline__ void clock_probe(uint64_t* clk, int at) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[2 * at] = __builtin_amdgcn_s_memtime();
    clk[2 * at + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

__global__ __launch_bounds__(256, 4) void k_time_f64(double* sink, uint64_t* clk, uint64_t seed) {
  clock_probe(clk, 0);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  F52 x[CHAINS], y;
  uint64_t s = seed ^ (0x9E3779B97F4A7C15ull * (i + 1));
  for (int k = 0; k < 5; ++k) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    y.l[k] = (double)(s >> 12);
    for (int c = 0; c < CHAINS; ++c) x[c].l[k] = (double)((s >> (12 - c)) & M52);
  }
  for (int it = 0; it < ITER; ++it)
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) f52_mul(x[c], x[c], y);
  double acc = 0;
  for (int c = 0; c < CHAINS; ++c)
    for (int k = 0; k < 5; ++k) acc += x[c].l[k];
  sink[i] = acc;
  __syncthreads();
  clock_probe(clk, 1);
}

__global__ __launch_bounds__(256, 4) void k_time_u32(uint32_t* sink, uint64_t* clk, uint64_t seed) {
  clock_probe(clk, 0);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  Fe x[CHAINS], y;
  uint64_t s = seed ^ (0x9E3779B97F4A7C15ull * (i + 1));
  for (int k = 0; k < 8; ++k) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    y.v[k] = (uint32_t)(s >> 32);
    for (int c = 0; c < CHAINS; ++c) x[c].v[k] = (uint32_t)(s >> (16 + c));
  }
  for (int it = 0; it < ITER; ++it)
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) fm_mul(x[c], x[c], y);
  uint32_t acc = 0;
  for (int c = 0; c < CHAINS; ++c)
    for (int k = 0; k < 8; ++k) acc ^= x[c].v[k];
  sink[i] = acc;
  __syncthreads();
  clock_probe(clk, 1);
}

int main(int argc, char** argv) {
  if (argc < 2) { printf("usage: f64mul verify <n> <out.bin> | time <f64|u32> <seconds>\n"); return 2; }
  if (!strcmp(argv[1], "verify")) {
    const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 65536;
    std::vector<uint64_t> hx(5 * n), hy(5 * n), ho(5 * n);
    uint64_t s = 0x6b68756e74663634ull;
    auto next = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
    for (uint32_t i = 0; i < n; ++i)
      for (int k = 0; k < 5; ++k) {
        // limbs < 2^52; the top limb < 2^52 too (values < 2^260), plus all-ones / zero edge lanes
        uint64_t vx = next() & M52, vy = next() & M52;
        if (i % 97 == 0) vx = M52;
        if (i % 89 == 0) vy = M52;
        if (i % 101 == 0) vx = 0;
        hx[5 * i + k] = vx;
        hy[5 * i + k] = vy;
      }
    uint64_t *dx, *dy, *dout;
    CHECK(hipMalloc(&dx, 40 * (size_t)n));
    CHECK(hipMalloc(&dy, 40 * (size_t)n));
    CHECK(hipMalloc(&dout, 40 * (size_t)n));
    CHECK(hipMemcpy(dx, hx.data(), 40 * (size_t)n, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dy, hy.data(), 40 * (size_t)n, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_verify, dim3((n + 255) / 256), dim3(256), 0, 0, dx, dy, dout, n);
    CHECK(hipGetLastError());
    CHECK(hipMemcpy(ho.data(), dout, 40 * (size_t)n, hipMemcpyDeviceToHost));
    FILE* f = fopen(argc > 3 ? argv[3] : "f64mul_verify.bin", "wb");
    fwrite(&n, 4, 1, f);
    fwrite(hx.data(), 8, 5 * (size_t)n, f);
    fwrite(hy.data(), 8, 5 * (size_t)n, f);
    fwrite(ho.data(), 8, 5 * (size_t)n, f);
    fclose(f);
    printf("verify: %u products written\n", n);
    return 0;
  }
  const bool f64 = argc > 2 && !strcmp(argv[2], "f64");
  const double secs = argc > 3 ? atof(argv[3]) : 3.0;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const uint32_t blocks = prop.multiProcessorCount * 4;      // 4 waves/SIMD: 4 blocks of 256 per CU
  const uint64_t lanes = (uint64_t)blocks * 256;
  void* sink;
  uint64_t* clk;
  CHECK(hipMalloc(&sink, 8 * lanes));
  CHECK(hipHostMalloc((void**)&clk, 64, hipHostMallocCoherent));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto launch = [&](uint64_t seed) {
    if (f64) hipLaunchKernelGGL(k_time_f64, dim3(blocks), dim3(256), 0, 0, (double*)sink, clk, seed);
    else hipLaunchKernelGGL(k_time_u32, dim3(blocks), dim3(256), 0, 0, (uint32_t*)sink, clk, seed);
  };
  launch(1);
  CHECK(hipDeviceSynchronize());
  const auto t0 = std::chrono::steady_clock::now();
  double ms_total = 0, mhz_sum = 0;
  int n = 0;
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < secs) {
    CHECK(hipEventRecord(e0, 0));
    launch(n + 2);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms_total += ms;
    mhz_sum += 100.0 * (double)(clk[2] - clk[0]) / (double)(clk[3] - clk[1]);
    ++n;
  }
  const double prods = (double)lanes * ITER * CHAINS * n;
  const double mhz = mhz_sum / n;
  const double simd_cycles = ms_total * 1e-3 * mhz * 1e6 * prop.multiProcessorCount * 4;
  // SIMD cycles per product of one wave (64 lanes): the unit of the walk's issue accounting
  printf("{\"kind\": \"%s\", \"launches\": %d, \"ms_per_launch\": %.3f, \"G_products_per_s\": %.3f, "
         "\"shader_mhz\": %.1f, \"simd_cycles_per_wave_product\": %.1f}\n",
         f64 ? "f64" : "u32", n, ms_total / n, prods / (ms_total * 1e-3) / 1e9, mhz, simd_cycles / (prods / 64.0));
  return 0;
}
