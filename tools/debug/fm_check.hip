// Debug: check each fe_asm.hpp primitive on the GPU against the portable fe.hpp on the host.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include "../../keyhuntm1cpu_amd/csrc/device/fe_asm.hpp"
using namespace khb;

__global__ void k(const Fe* a, const Fe* b, uint32_t* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t t[16];
  fm_mul512(t, a[i].v, b[i].v);
  uint32_t* o = out + (size_t)i * 56;
  for (int k = 0; k < 16; ++k) o[k] = t[k];
  Fe r; fm_reduce(r, t);
  for (int k = 0; k < 8; ++k) o[16 + k] = r.v[k];
  Fe s; fm_sub(s, a[i], b[i]);
  for (int k = 0; k < 8; ++k) o[24 + k] = s.v[k];
  Fe ad; fm_add(ad, a[i], b[i]);
  for (int k = 0; k < 8; ++k) o[32 + k] = ad.v[k];
  Fe c; fm_canon(c, r);
  for (int k = 0; k < 8; ++k) o[40 + k] = c.v[k];
  Fe m; fm_mul(m, a[i], b[i]); fm_canon(m, m);
  for (int k = 0; k < 8; ++k) o[48 + k] = m.v[k];
}
static uint64_t sm = 7;
static uint32_t rnd() { uint64_t z = (sm += 0x9E3779B97F4A7C15ull); z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; return (uint32_t)(z ^ (z >> 31)); }
int main() {
  const int n = 4096;
  std::vector<Fe> a(n), b(n);
  for (int i = 0; i < n; ++i) {
    for (int k = 0; k < 8; ++k) { a[i].v[k] = rnd(); b[i].v[k] = rnd(); }
    if (i % 4 == 1) for (int k = 2; k < 8; ++k) a[i].v[k] = 0xFFFFFFFFu;       // near p
    if (i % 4 == 2) { for (int k = 0; k < 8; ++k) a[i].v[k] = b[i].v[k] = 0xFFFFFFFFu; a[i].v[0] = rnd(); b[i].v[1] = rnd(); }
    if (i % 4 == 3) for (int k = 3; k < 8; ++k) { a[i].v[k] = 0xFFFFFFFFu; b[i].v[k] = 0xFFFFFFFFu; }
    // canonical inputs (< p): p = FFFFFFFF x6, FFFFFFFE, FFFFFC2F
    bool ge = true;
    for (int k = 7; k >= 2; --k) if (a[i].v[k] != 0xFFFFFFFFu) ge = false;
    if (ge && (a[i].v[1] > 0xFFFFFFFEu || (a[i].v[1] == 0xFFFFFFFEu && a[i].v[0] >= 0xFFFFFC2Fu))) a[i].v[1] = 0x12345678;
    ge = true;
    for (int k = 7; k >= 2; --k) if (b[i].v[k] != 0xFFFFFFFFu) ge = false;
    if (ge && (b[i].v[1] > 0xFFFFFFFEu || (b[i].v[1] == 0xFFFFFFFEu && b[i].v[0] >= 0xFFFFFC2Fu))) b[i].v[1] = 0x12345678;
    if (i < 8) { memset(&a[i], 0, 32); a[i].v[0] = i; }
  }
  Fe *da, *db; uint32_t* dout;
  hipMalloc(&da, n * 32); hipMalloc(&db, n * 32); hipMalloc(&dout, (size_t)n * 56 * 4);
  hipMemcpy(da, a.data(), n * 32, hipMemcpyHostToDevice); hipMemcpy(db, b.data(), n * 32, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, da, db, dout, n);
  std::vector<uint32_t> out((size_t)n * 56);
  hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost);
  int bad[6] = {0};
  for (int i = 0; i < n; ++i) {
    const uint32_t* o = &out[(size_t)i * 56];
    // host 512-bit product
    uint32_t t[16] = {0};
    for (int x = 0; x < 8; ++x) { uint64_t c = 0; for (int y = 0; y < 8; ++y) { c = (uint64_t)a[i].v[x] * b[i].v[y] + t[x + y] + (c >> 32); t[x + y] = (uint32_t)c; } t[x + 8] = (uint32_t)(c >> 32); }
    if (memcmp(t, o, 64)) { if (bad[0]++ < 3) { printf("mul512 mismatch i=%d\n  got ", i); for (int k = 15; k >= 0; --k) printf("%08x", o[k]); printf("\n  exp "); for (int k = 15; k >= 0; --k) printf("%08x", t[k]); printf("\n"); } }
    Fe ref; fe_mul(ref, a[i], b[i]);
    Fe rr; memcpy(rr.v, o + 16, 32); Fe rc; memcpy(rc.v, o + 40, 32);
    if (memcmp(rc.v, ref.v, 32)) { if (bad[1]++ < 3) { printf("reduce mismatch i=%d\n", i); } }
    Fe sref; fe_sub(sref, a[i], b[i]);
    if (memcmp(sref.v, o + 24, 32)) { if (bad[2]++ < 3) { printf("sub mismatch i=%d\n  got ", i); for (int k = 7; k >= 0; --k) printf("%08x", o[24 + k]); printf("\n  exp "); for (int k = 7; k >= 0; --k) printf("%08x", sref.v[k]); printf("\n"); } }
    Fe aref; fe_add(aref, a[i], b[i]);
    if (memcmp(aref.v, o + 32, 32)) { if (bad[3]++ < 3) printf("add mismatch i=%d\n", i); }
    if (memcmp(ref.v, o + 48, 32)) { if (bad[4]++ < 3) printf("fm_mul mismatch i=%d\n", i); }
  }
  printf("mismatches: mul512 %d reduce %d sub %d add %d mul %d (of %d)\n", bad[0], bad[1], bad[2], bad[3], bad[4], n);
  return 0;
}
