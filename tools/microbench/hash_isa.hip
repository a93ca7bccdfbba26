// Static VALU counts of the hash building blocks as compiled for gfx950 (no GPU needed):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I keyhuntm1cpu_amd/csrc --cuda-device-only -S \
//     -o /tmp/hash_isa.s tools/microbench/hash_isa.hip && python tools/debug/hash_isa_count.py /tmp/hash_isa.s
// Each kernel is straight-line code (every loop unrolled), so the static count is the executed count
// per thread, loads/stores of the operands included (≈ 25 instructions).
#include <hip/hip_runtime.h>
#include "device/hash160.hpp"
using namespace khb;

// hash160 of both compressed keys 02 || x and 03 || x in one scope: the two messages differ only in
// word 0, so their SHA-256 schedules share W17, W19, W21 and the partial sums of words 18..30 (round-2
// experiment KHB_ADDR_PAIR: 4401 VALU for the pair vs 2 x 2249, no faster in the kernel).
__device__ __forceinline__ void hash160_compressed_pair(uint32_t out2[5], uint32_t out3[5], const Fe& x) {
  hash160_compressed(out2, 2u, x);
  hash160_compressed(out3, 3u, x);
}

__global__ void k_sha_block(const uint32_t* in, uint32_t* out) {       // one SHA-256 compression
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  uint32_t w[16], s[8];
  for (int k = 0; k < 16; ++k) w[k] = in[i * 16 + k];
  sha256_init(s);
  sha256_block(s, w);
  for (int k = 0; k < 8; ++k) out[i * 8 + k] = s[k];
}
__global__ void k_rmd_block(const uint32_t* in, uint32_t* out) {       // RIPEMD-160 of a 32-byte digest
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  uint32_t d[8], o[5];
  for (int k = 0; k < 8; ++k) d[k] = in[i * 8 + k];
  ripemd160_of_sha(o, d);
  for (int k = 0; k < 5; ++k) out[i * 5 + k] = o[k];
}
__global__ void k_hash160_compressed(const uint32_t* in, uint32_t* out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  Fe x;
  for (int k = 0; k < 8; ++k) x.v[k] = in[i * 8 + k];
  uint32_t o[5];
  hash160_compressed(o, 2, x);
  for (int k = 0; k < 5; ++k) out[i * 5 + k] = o[k];
}
__global__ void k_hash160_pair(const uint32_t* in, uint32_t* out) {     // 02 and 03 in one scope
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  Fe x;
  for (int k = 0; k < 8; ++k) x.v[k] = in[i * 8 + k];
  uint32_t o[5], p[5];
  hash160_compressed_pair(o, p, x);
  for (int k = 0; k < 5; ++k) out[i * 5 + k] = o[k] ^ p[k];
}
__global__ void k_hash160_uncompressed(const uint32_t* in, uint32_t* out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  Fe x, y;
  for (int k = 0; k < 8; ++k) {
    x.v[k] = in[i * 16 + k];
    y.v[k] = in[i * 16 + 8 + k];
  }
  uint32_t o[5];
  hash160_uncompressed(o, x, y);
  for (int k = 0; k < 5; ++k) out[i * 5 + k] = o[k];
}
__global__ void k_xxh64_pair(const uint32_t* in, uint64_t* out) {       // the bloom's two XXH64
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  uint32_t h[5];
  for (int k = 0; k < 5; ++k) h[k] = in[i * 5 + k];
  const uint64_t a = xxh64_20(h, KHB_BLOOM_SEED);
  out[i] = a ^ xxh64_20(h, a);
}
