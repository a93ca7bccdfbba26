// Host-side check of the 9 x 29-bit field (device/fe29.hpp, compiled for the CPU) against the
// oracle's exact arithmetic, over canonical inputs and over limbs at the bounds the header states
// (strict < 2^29 + 2^20, lazy sums < 2^30.4, gate / to_fe inputs < 2^30.6).
// Test infrastructure: links oracle/liboracle (the checker).
#include "../../keyhuntm1cpu_amd/csrc/device/fe29.hpp"
extern "C" {
#include "../../oracle/ora.h"
}
#include <cstdio>
#include <cstring>
using namespace khb;

static uint64_t sm = 29;
static uint64_t splitmix() { uint64_t z = (sm += 0x9E3779B97F4A7C15ull); z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; return z ^ (z >> 31); }

// value of an F9 mod p, by Horner over the oracle field (every limb < 2^31 is a canonical element)
static void f9_value(ora_u256* r, const F9& a) {
  ora_u256 acc, t, sh;
  memset(&acc, 0, sizeof acc);
  memset(&sh, 0, sizeof sh);
  uint8_t b[32] = {0};
  b[28] = 0x20;                       // 2^29 big-endian
  ora_u256_from_be(&sh, b);
  for (int i = 8; i >= 0; --i) {
    ora_fe_mul_exact(&acc, &acc, &sh);
    uint8_t lb[32] = {0};
    lb[28] = (uint8_t)(a.v[i] >> 24); lb[29] = (uint8_t)(a.v[i] >> 16); lb[30] = (uint8_t)(a.v[i] >> 8); lb[31] = (uint8_t)a.v[i];
    ora_u256_from_be(&t, lb);
    ora_fe_add(&acc, &acc, &t);
  }
  *r = acc;
}

// limbs < bound (bound as a fraction of 2^30 scaled by 1000), adversarial at the top of the range
static F9 rnd_f9(int mode, double hi) {
  F9 a;
  const uint64_t lim = (uint64_t)(hi * 1073741824.0);
  for (int i = 0; i < 9; ++i) {
    const uint64_t r = splitmix();
    if (mode == 0) a.v[i] = (uint32_t)(r % lim);
    else if (mode == 1) a.v[i] = (uint32_t)(lim - 1 - (r & 0xFF));      // all limbs at the bound
    else a.v[i] = (r & 1) ? (uint32_t)(lim - 1) : (uint32_t)(r % 4);
  }
  return a;
}

static F9 rnd_canon(int mode) {
  uint8_t b[32];
  for (int i = 0; i < 32; ++i) b[i] = (uint8_t)splitmix();
  if (mode == 1) memset(b, 0xFF, 28);
  if (mode == 2) memset(b, 0, 24);
  ora_u256 v; ora_u256_from_be(&v, b);
  while (ora_u256_cmp(&v, ora_prime()) >= 0) ora_u256_sub(&v, &v, ora_prime());
  ora_u256_to_be(&v, b);
  Fe f; fe_from_be(f, b);
  F9 r; f9_from_fe(r, f);
  return r;
}

static bool same(const ora_u256& x, const ora_u256& y) { return ora_u256_cmp(&x, &y) == 0; }

int main() {
  int fails = 0;
  const double kLazy = 1.3195;        // 2^30.4 / 2^30
  const double kGate = 1.5157;        // 2^30.6 / 2^30
  for (int it = 0; it < 200000; ++it) {
    const int mode = it % 3;
    const F9 a = (it & 8) ? rnd_canon(it % 5 == 1 ? 1 : it % 5 == 2 ? 2 : 0) : rnd_f9(mode, kLazy);
    const F9 b = (it & 16) ? rnd_canon(0) : rnd_f9((mode + 1) % 3, kLazy);
    ora_u256 va, vb, ve, vg;
    f9_value(&va, a);
    f9_value(&vb, b);
    F9 r;
    f9_mul(r, a, b);
    ora_fe_mul_exact(&ve, &va, &vb);
    f9_value(&vg, r);
    if (!same(ve, vg)) { if (fails++ < 10) printf("FAIL mul it %d\n", it); }
    for (int i = 0; i < 9; ++i)
      if (r.v[i] >= (1u << 29) + (1u << 20)) { if (fails++ < 10) printf("FAIL mul limb %d bound it %d\n", i, it); }
    f9_sqr(r, a);
    ora_fe_mul_exact(&ve, &va, &va);
    f9_value(&vg, r);
    if (!same(ve, vg)) { if (fails++ < 10) printf("FAIL sqr it %d\n", it); }
    for (int i = 0; i < 9; ++i)
      if (r.v[i] >= (1u << 29) + (1u << 20)) { if (fails++ < 10) printf("FAIL sqr limb %d bound it %d\n", i, it); }
    // to_fe (canonical) and the gate words, on limbs up to 2^30.6
    const F9 g = (it & 32) ? rnd_f9(mode, kGate) : a;
    ora_u256 vgate;
    f9_value(&vgate, g);
    Fe fc;
    f9_to_fe(fc, g);
    uint8_t be[32], be2[32];
    fe_to_be(be, fc);
    ora_u256_to_be(&vgate, be2);
    if (memcmp(be, be2, 32)) { if (fails++ < 10) printf("FAIL to_fe it %d\n", it); }
    uint32_t w0, w1;
    bool rare;
    f9_gate_words(w0, w1, rare, g);
    if (!rare && (w0 != fc.v[0] || w1 != fc.v[1])) { if (fails++ < 10) printf("FAIL gate words it %d\n", it); }
    if (it < 2000) {
      f9_inv(r, a);
      ora_fe_inv(&ve, &va);
      f9_value(&vg, r);
      if (!same(ve, vg)) { if (fails++ < 10) printf("FAIL inv it %d\n", it); }
    }
  }
  // a + 2p - b (f9_add_neg) for canonical b, and its product with a strict value
  for (int it = 0; it < 50000; ++it) {
    const F9 a = (it & 1) ? rnd_canon(it % 3) : rnd_f9(1, 1.0);      // strict or limbs at 2^30 - 256
    const F9 b = rnd_canon(it % 3 == 1 ? 1 : 0);
    F9 d, m, q;
    f9_add_neg(d, a, b);
    ora_u256 va, vb, vd, ve, vm;
    f9_value(&va, a); f9_value(&vb, b); f9_value(&vd, d);
    ora_fe_sub(&ve, &va, &vb);
    if (!same(ve, vd)) { if (fails++ < 10) printf("FAIL add_neg it %d\n", it); }
    f9_mul(q, rnd_canon(0), rnd_canon(2));                            // a strict product result
    f9_mul(m, d, q);
    ora_u256 vq; f9_value(&vq, q);
    ora_fe_mul_exact(&ve, &vd, &vq);
    f9_value(&vm, m);
    if (!same(ve, vm)) { if (fails++ < 10) printf("FAIL add_neg product it %d\n", it); }
  }
  // the gate's rare flag: limb 8 within 4 of a multiple of 2^24 (and its exact neighbours)
  for (int it = 0; it < 20000; ++it) {
    F9 g = rnd_f9(0, 1.0);
    g.v[8] = (uint32_t)((splitmix() % 64) << 24) | (0xFFFFFFu - (uint32_t)(splitmix() % 8));
    Fe fc;
    f9_to_fe(fc, g);
    uint32_t w0, w1;
    bool rare;
    f9_gate_words(w0, w1, rare, g);
    if (!rare && (w0 != fc.v[0] || w1 != fc.v[1])) { if (fails++ < 10) printf("FAIL gate edge it %d\n", it); }
  }
  printf("%s (%d failures)\n", fails ? "FAIL" : "ok", fails);
  return fails ? 1 : 0;
}
