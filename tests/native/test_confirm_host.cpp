// Host-compiled check of device/confirm.hpp (the GPU's bsgs_secondcheck / bsgs_thirdcheck, khb_check)
// against the oracle's restatement (oracle/ora_bsgs.c secondcheck, keyhunt.cpp:4271-4368).  Test
// infrastructure: the oracle is the checker.
//   1. real tables of a small geometry: planted keys around each candidate's window (found / not found,
//      both signs of the third check's +-(j+1)), the AddDirect(P, -P) special case of the third check,
//      and random candidates;
//   2. the same candidates with every level-2 and level-3 bloom bit set in both implementations, so each
//      candidate runs 32 third checks, 1024 level-3 probes and bPtable searches.
#include "../../keyhuntm1cpu_amd/csrc/device/confirm.hpp"
extern "C" {
#include "../../oracle/ora.h"
}
#include <cstdio>
#include <cstring>
#include <vector>
using namespace khb;

static uint64_t sm = 0x636f6e6669726dull;
static uint64_t splitmix() {
  uint64_t z = (sm += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static Fe fe_of(const ora_u256& a) {
  Fe f;
  for (int k = 0; k < 4; ++k) {
    f.v[2 * k] = (uint32_t)a.w[k];
    f.v[2 * k + 1] = (uint32_t)(a.w[k] >> 32);
  }
  return f;
}
static U8 u8_of(const ora_u256& a) {
  Fe f = fe_of(a);
  U8 r;
  memcpy(r.v, f.v, sizeof r.v);
  return r;
}
static ora_u256 ora_of(const U8& a) {
  ora_u256 r;
  for (int k = 0; k < 4; ++k) r.w[k] = a.v[2 * k] | ((uint64_t)a.v[2 * k + 1] << 32);
  return r;
}
static CPt cpt_of(const ora_point& p) { return CPt{fe_of(p.x), fe_of(p.y)}; }
static CPt cpt_be(const uint8_t* b) {
  CPt p;
  fe_from_be(p.x, b);
  fe_from_be(p.y, b + 32);
  return p;
}
static ora_u256 u64v(uint64_t v) {
  ora_u256 r;
  ora_u256_set64(&r, v);
  return r;
}
static ora_u256 add(ora_u256 a, const ora_u256& b) {
  ora_u256 r;
  ora_u256_add(&r, &a, &b);
  return r;
}
static ora_u256 mul(ora_u256 a, uint64_t m) {
  ora_u256 r;
  ora_u256_mul64(&r, &a, m);
  return r;
}

struct Case {
  ora_u256 base;
  uint32_t a;
  ora_point target;
  const char* kind;
};

int main() {
  ora_secp_init();
  char err[256];
  ora_bsgs* B = ora_bsgs_new("0x1000000000", 1, 8, err, sizeof err);   // N = 2^36: m = 2^18, m2 = 2^13, m3 = 2^8
  if (!B) {
    printf("FAIL oracle tables: %s\n", err);
    return 1;
  }
  uint64_t par[10];
  ora_bsgs_params(B, par);
  const uint64_t m = par[0], m2 = par[1], m3 = par[2];
  // tables in the device layout
  std::vector<CPt> gtab(32 * 256);
  for (int i = 0; i < 32; ++i)
    for (int b = 1; b < 256; ++b) {
      ora_u256 k = {{0, 0, 0, 0}};
      k.w[i / 8] = (uint64_t)b << (8 * (i % 8));
      ora_point P;
      ora_compute_pubkey(&P, &k);
      gtab[256 * i + b - 1] = cpt_of(P);
    }
  uint8_t a2b[32 * 64], a3b[32 * 64];
  ora_bsgs_amp_table(B, 2, a2b);
  ora_bsgs_amp_table(B, 3, a3b);
  std::vector<CPt> amp2(32), amp3(32);
  for (int i = 0; i < 32; ++i) {
    amp2[i] = cpt_be(a2b + 64 * i);
    amp3[i] = cpt_be(a3b + 64 * i);
  }
  std::vector<uint8_t> l2, l3, bp(16 * m3);
  const ora_bloom* b2 = ora_bsgs_bloom(B, 2, 0);
  const ora_bloom* b3 = ora_bsgs_bloom(B, 3, 0);
  for (int s = 0; s < 256; ++s) {
    const ora_bloom* x = ora_bsgs_bloom(B, 2, s);
    l2.insert(l2.end(), x->bf, x->bf + x->bytes);
    x = ora_bsgs_bloom(B, 3, s);
    l3.insert(l3.end(), x->bf, x->bf + x->bytes);
  }
  memcpy(bp.data(), ora_bsgs_bptable(B), 16 * m3);
  auto geom = [](const ora_bloom* b) {
    BloomGeom g;
    g.bytes_per_sub = b->bytes;
    g.bits = b->bits;
    g.magic = (uint64_t)(((unsigned __int128)1 << 64) / b->bits);
    g.wrap = (uint64_t)(((unsigned __int128)1 << 64) % b->bits);
    g.hashes = b->hashes;
    return g;
  };
  CheckTables T;
  T.gtab = gtab.data();
  T.amp2 = amp2.data();
  T.amp3 = amp3.data();
  T.l2 = l2.data();
  T.l3 = l3.data();
  T.bp = bp.data();
  T.g2 = geom(b2);
  T.g3 = geom(b3);
  T.n_bp = m3;
  T.m_double = u8_of(u64v(2 * m));
  T.m2_double = u8_of(u64v(2 * m2));
  T.m3 = u8_of(u64v(m3));
  T.m3_double = u8_of(u64v(2 * m3));

  // candidates
  std::vector<Case> cases;
  for (int c = 0; c < 48; ++c) {             // planted: key = base + a*2m + off, off across the window
    Case x;
    x.base = {{splitmix(), splitmix() & 0xffff, 0, 0}};
    x.a = (uint32_t)(splitmix() % 4096);
    const uint64_t off = splitmix() % (2 * m + 64);
    ora_u256 key = add(add(x.base, mul(u64v(2 * m), x.a)), u64v(off));
    ora_compute_pubkey(&x.target, &key);
    x.kind = "planted";
    cases.push_back(x);
  }
  for (int c = 0; c < 16; ++c) {             // the third check's AddDirect(P, -P) special case
    Case x;
    x.base = {{splitmix(), 0, 0, 0}};
    x.a = (uint32_t)(splitmix() % 4096);
    const uint32_t i2 = (uint32_t)(splitmix() % 32), i = (uint32_t)(splitmix() % 32);
    ora_u256 key = add(add(x.base, mul(u64v(2 * m), x.a)), mul(u64v(2 * m2), i2));
    key = add(key, add(mul(u64v(2 * m3), i), u64v(m3)));
    ora_compute_pubkey(&x.target, &key);
    x.kind = "special";
    cases.push_back(x);
  }
  for (int c = 0; c < 32; ++c) {             // random: nothing to find
    Case x;
    x.base = {{splitmix(), splitmix(), splitmix() >> 8, 0}};
    x.a = (uint32_t)splitmix();
    ora_u256 key = {{splitmix(), splitmix(), splitmix(), splitmix() >> 4}};
    ora_compute_pubkey(&x.target, &key);
    x.kind = "random";
    cases.push_back(x);
  }

  int fails = 0, found = 0, l2h = 0, l3h = 0, bph = 0, special_found = 0;
  auto run = [&](const char* phase, size_t ncases) {
    for (size_t c = 0; c < ncases; ++c) {
      const Case& x = cases[c];
      ora_u256 okey = {{0, 0, 0, 0}};
      const int ofound = ora_bsgs_secondcheck(B, &x.base, x.a, &x.target, &okey);
      CheckResult r{};
      const bool gfound = second_check(T, u8_of(x.base), x.a, cpt_of(x.target), r);
      found += gfound;
      l2h += r.l2_hits;
      l3h += r.l3_hits;
      bph += r.bp_hits;
      if (gfound && !strcmp(x.kind, "special")) special_found++;
      const ora_u256 gk = ora_of(r.key);
      if (ofound != (int)gfound || (ofound && ora_u256_cmp(&okey, &gk) != 0)) {
        char h1[65], h2[65];
        ora_u256_to_hex(&okey, h1);
        ora_u256_to_hex(&gk, h2);
        printf("FAIL %s case %zu (%s): oracle %d %s, device code %d %s\n", phase, c, x.kind, ofound, h1, (int)gfound, h2);
        fails++;
      }
    }
  };
  run("real", cases.size());
  printf("real tables: %zu candidates, %d found (%d special), l2 hits %d, l3 hits %d, bPtable hits %d\n", cases.size(),
         found, special_found, l2h, l3h, bph);
  if (found < 16 || special_found < 8 || bph == 0) {
    printf("FAIL too few paths exercised\n");
    fails++;
  }
  // dense blooms: every level-2/3 bit set in both implementations
  for (int s = 0; s < 256; ++s) {
    ora_bloom* x = const_cast<ora_bloom*>(ora_bsgs_bloom(B, 2, s));
    memset(x->bf, 0xff, x->bytes);
    x = const_cast<ora_bloom*>(ora_bsgs_bloom(B, 3, s));
    memset(x->bf, 0xff, x->bytes);
  }
  memset(l2.data(), 0xff, l2.size());
  memset(l3.data(), 0xff, l3.size());
  found = l2h = l3h = bph = special_found = 0;
  run("dense", 24);
  printf("dense blooms: 24 candidates, %d found, l2 hits %d, l3 hits %d, bPtable hits %d\n", found, l2h, l3h, bph);
  ora_bsgs_free(B);
  printf(fails ? "FAIL %d\n" : "ok\n", fails);
  return fails ? 1 : 0;
}
