// Field-primitive throughput on gfx950 at the scan kernel's occupancy (4 waves/SIMD), plus an
// exactness check of alternative 512-bit product schedules against the production ones.
// Build: make -C tools/microbench fmbench   Run: tools/microbench/fmbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "device/fe_asm.hpp"
#include "device/bloom_probe.hpp"
using namespace khb;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// ---- exactness: raw products and reduced results of the two schedules ----
__global__ void k_check(const Fe* a, const Fe* b, uint32_t* bad, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t t0[16], t1[16], t2[16], s0[16], s1[16], s2[16];
  fm_mul512(t0, a[i].v, b[i].v);
  fm_mul512x(t1, a[i].v, b[i].v);
  fm_mul512p(t2, a[i].v, b[i].v);
  fm_mul512(s0, a[i].v, a[i].v);
  fm_sqr512x(s1, a[i].v);
  fm_sqr512p(s2, a[i].v);
  uint32_t m = 0;
  for (int k = 0; k < 16; ++k) {
    m |= (t0[k] != t1[k]) ? 1u : 0u;
    m |= (t0[k] != t2[k]) ? 16u : 0u;
    m |= (s0[k] != s2[k]) ? 32u : 0u;
    m |= (s0[k] != s1[k]) ? 2u : 0u;
  }
  Fe r0, r1, q0, q1;
  fm_mul_shuffle(r0, a[i], b[i]); fm_canon(r0, r0);
  fm_mul(r1, a[i], b[i]); fm_canon(r1, r1);
  fm_sqr_generic(q0, a[i]); fm_canon(q0, q0);
  fm_sqr(q1, a[i]); fm_canon(q1, q1);
  for (int k = 0; k < 8; ++k) {
    m |= (r0.v[k] != r1.v[k]) ? 4u : 0u;
    m |= (q0.v[k] != q1.v[k]) ? 8u : 0u;
  }
  if (m) atomicOr(bad, m);
}

// ---- throughput ----
#define ITERS 256
template <int OP>
__global__ __launch_bounds__(256) void k_tp(const Fe* seed, Fe* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  Fe x = seed[i & 1023], y = seed[(i + 7) & 1023];
  uint64_t h = x.v[0];
  for (int it = 0; it < ITERS; ++it) {
    if (OP == 0) fm_mul_shuffle(x, x, y);
    if (OP == 1) fm_mul(x, x, y);
    if (OP == 2) fm_sqr_generic(x, x);
    if (OP == 3) fm_sqr(x, x);
    if (OP == 4) { uint64_t w[4]; x_words(w, x); h = xxh64_32(w, h); x.v[0] ^= (uint32_t)h; }
    if (OP == 5) { fm_sub(x, x, y); fm_canon(x, x); }
    if (OP == 6) { fm_add(x, x, y); }
  }
  if (x.v[0] == 0x12345678u && x.v[1] == 0x9abcdef0u) out[i] = x;
}

const char* names[] = {"fm_mul_shuffle (old)", "fm_mul (seeded columns)", "fm_sqr_generic (old)", "fm_sqr (36 products)",
                       "xxh64_32", "fm_sub+fm_canon", "fm_add"};

template <int OP>
int run(const Fe* seed, Fe* out, int cus) {
  const int blocks = cus * 4, threads = 256;   // 16 waves per CU = 4 per SIMD
  hipLaunchKernelGGL(k_tp<OP>, dim3(blocks), dim3(threads), 0, 0, seed, out);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  const int reps = 20;
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_tp<OP>, dim3(blocks), dim3(threads), 0, 0, seed, out);
  CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double ops = (double)reps * blocks * threads * ITERS;
  printf("%-26s %9.2f G ops/s   %7.3f ns/op/CU\n", names[OP], ops / (ms * 1e-3) / 1e9,
         (ms * 1e6) / ops * cus);
  return 0;
}

static uint64_t sm = 11;
static uint32_t rnd() { uint64_t z = (sm += 0x9E3779B97F4A7C15ull); z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; return (uint32_t)(z ^ (z >> 31)); }

int main() {
  hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  // exactness: random values, values with all-ones / all-zero limbs, and values near 2^256 and p
  const int n = 1 << 20;
  std::vector<Fe> a(n), b(n);
  const uint32_t pat[6] = {0u, 1u, 0xffffffffu, 0xfffffffeu, 0x80000000u, 0xfffffc2fu};
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < 8; ++k) {
      const uint32_t r = rnd();
      const int mode = i & 3;
      a[i].v[k] = mode == 0 ? rnd() : mode == 1 ? pat[r % 6] : mode == 2 ? (r & 7 ? 0xffffffffu : rnd()) : rnd() | 0xffff0000u;
      b[i].v[k] = mode == 0 ? rnd() : mode == 1 ? pat[(r >> 8) % 6] : mode == 2 ? ((r >> 4) & 7 ? 0xffffffffu : rnd()) : rnd();
    }
  Fe *da, *db; uint32_t* dbad;
  CHECK(hipMalloc(&da, n * sizeof(Fe))); CHECK(hipMalloc(&db, n * sizeof(Fe))); CHECK(hipMalloc(&dbad, 4));
  CHECK(hipMemcpy(da, a.data(), n * sizeof(Fe), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(db, b.data(), n * sizeof(Fe), hipMemcpyHostToDevice));
  CHECK(hipMemset(dbad, 0, 4));
  hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, da, db, dbad, n);
  uint32_t bad = 0; CHECK(hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost));
  printf("exactness over %d inputs: %s (mask 0x%x: 1 mul512x 2 sqr512x 4 fm_mul 8 fm_sqr 16 mul512p 32 sqr512p)\n", n, bad ? "MISMATCH" : "ok", bad);
  Fe* dout; CHECK(hipMalloc(&dout, (size_t)cus * 1024 * sizeof(Fe)));
  if (run<0>(da, dout, cus) || run<1>(da, dout, cus) || run<2>(da, dout, cus) || run<3>(da, dout, cus) ||
      run<4>(da, dout, cus) || run<5>(da, dout, cus) || run<6>(da, dout, cus))
    return 1;
  return bad ? 2 : 0;
}
