// Throughput of the 9 x 29-bit field (device/fe29.hpp) against the 8 x 32 asm field (fe_asm.hpp) on
// gfx950 at the scan kernel's occupancy (4 waves/SIMD), plus a GPU exactness check of f9_mul /
// f9_sqr / f9_to_fe against fm_mul / fm_sqr + fm_canon.
// Build: make -C tools/microbench fe29bench   Run: tools/microbench/fe29bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "device/fe_asm.hpp"
#include "device/fe29.hpp"
using namespace khb;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_check(const Fe* a, const Fe* b, uint32_t* bad, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fe r0, q0, r1, q1;
  fm_mul(r0, a[i], b[i]); fm_canon(r0, r0);
  fm_sqr(q0, a[i]); fm_canon(q0, q0);
  F9 fa, fb, fr, fq;
  f9_from_fe(fa, a[i]); f9_from_fe(fb, b[i]);
  f9_mul(fr, fa, fb); f9_to_fe(r1, fr);
  f9_sqr(fq, fa); f9_to_fe(q1, fq);
  uint32_t m = 0;
  for (int k = 0; k < 8; ++k) { m |= r0.v[k] != r1.v[k] ? 1u : 0u; m |= q0.v[k] != q1.v[k] ? 2u : 0u; }
  uint32_t w0, w1; bool rare;
  F9 s; f9_add(s, fr, fq);             // a lazy sum, as x = s^2 + nu in the walk
  Fe sc; f9_to_fe(sc, s);
  f9_gate_words(w0, w1, rare, s);
  if (!rare && (w0 != sc.v[0] || w1 != sc.v[1])) m |= 4u;
  if (m) atomicOr(bad, m);
}

#define ITERS 256
template <int OP>
__global__ __launch_bounds__(256) void k_tp(const Fe* seed, Fe* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  Fe x = seed[i & 1023], y = seed[(i + 7) & 1023];
  F9 u, v, u2;
  f9_from_fe(u, x); f9_from_fe(v, y);
  const Fe x2 = seed[(i + 3) & 1023];
  f9_from_fe(u2, x2);
  for (int it = 0; it < ITERS; ++it) {
    if (OP == 0) fm_mul(x, x, y);
    if (OP == 1) fm_sqr(x, x);
    if (OP == 2) f9_mul(u, u, v);
    if (OP == 3) f9_sqr(u, u);
    if (OP == 4) { uint32_t w0, w1; bool r; f9_gate_words(w0, w1, r, u); u.v[0] ^= w0 ^ w1 ^ (r ? 1u : 0u); }
    if (OP == 6) { fm_mul(x, x, y); fm_mul(y, y, x2); }
    if (OP == 7) { f9_mul(u, u, v); f9_mul(v, v, u2); }
    if (OP == 5) {   // raw v_lshrrev_b64 rate, 8 independent chains
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        uint64_t t = ((uint64_t)u.v[k] << 32) | u.v[k + 1];
        asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(t));
        u.v[k] = (uint32_t)t ^ (uint32_t)(t >> 32);
      }
    }
  }
  if (OP >= 2 && OP != 6) for (int k = 0; k < 8; ++k) x.v[k] = (u.v[k] * 0x9E3779B1u) ^ u.v[8] ^ v.v[k];
  if (OP == 6) for (int k = 0; k < 8; ++k) x.v[k] ^= y.v[k];
  if (x.v[0] == 0x12345678u && x.v[1] == 0x9abcdef0u) out[i] = x;
}

const char* names[] = {"fm_mul (8x32 asm)", "fm_sqr (8x32 asm)", "f9_mul (9x29)", "f9_sqr (9x29)", "f9_gate_words",
                       "8x (v_lshrrev_b64+xor)", "2 fm_mul chains (x2 ops)", "2 f9_mul chains (x2 ops)"};

template <int OP>
int run(const Fe* seed, Fe* out, int cus) {
  const int blocks = cus * 4, threads = 256;
  hipLaunchKernelGGL(k_tp<OP>, dim3(blocks), dim3(threads), 0, 0, seed, out);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  const int reps = 20;
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_tp<OP>, dim3(blocks), dim3(threads), 0, 0, seed, out);
  CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double ops = (double)reps * blocks * threads * ITERS;
  printf("%-22s %9.2f G ops/s   %7.3f ns/op/CU\n", names[OP], ops / (ms * 1e-3) / 1e9, (ms * 1e6) / ops * cus);
  return 0;
}

static uint64_t sm = 11;
static uint32_t rnd() { uint64_t z = (sm += 0x9E3779B97F4A7C15ull); z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; return (uint32_t)(z ^ (z >> 31)); }

int main() {
  hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int n = 1 << 20;
  std::vector<Fe> a(n), b(n);
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < 8; ++k) {
      a[i].v[k] = (i & 3) == 1 ? 0xFFFFFFFFu : rnd();
      b[i].v[k] = (i & 7) == 2 ? 0xFFFFFFFFu : rnd();
    }
  Fe *da, *db; uint32_t* dbad;
  CHECK(hipMalloc(&da, n * sizeof(Fe))); CHECK(hipMalloc(&db, n * sizeof(Fe))); CHECK(hipMalloc(&dbad, 4));
  CHECK(hipMemcpy(da, a.data(), n * sizeof(Fe), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(db, b.data(), n * sizeof(Fe), hipMemcpyHostToDevice));
  CHECK(hipMemset(dbad, 0, 4));
  hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, da, db, dbad, n);
  uint32_t bad = 0; CHECK(hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost));
  printf("exactness over %d inputs: %s (mask 0x%x: 1 mul 2 sqr 4 gate words)\n", n, bad ? "MISMATCH" : "ok", bad);
  Fe* dout; CHECK(hipMalloc(&dout, (size_t)cus * 1024 * sizeof(Fe)));
  if (run<0>(da, dout, cus) || run<1>(da, dout, cus) || run<2>(da, dout, cus) || run<3>(da, dout, cus) ||
      run<4>(da, dout, cus) || run<5>(da, dout, cus) || run<6>(da, dout, cus) || run<7>(da, dout, cus))
    return 1;
  return bad ? 2 : 0;
}
