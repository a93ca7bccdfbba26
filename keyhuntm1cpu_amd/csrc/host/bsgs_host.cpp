#include "bsgs_host.hpp"

#include "../../../include/khbsgs.h"

#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>

namespace khb {

namespace {

constexpr int kGrp = 1024;      // CPU_GRP_SIZE, keyhunt.cpp:127
constexpr int kHalf = kGrp / 2;
constexpr uint64_t kJobKeys = 1048576;    // THREADBPWORKLOAD, keyhunt.cpp:63
constexpr long double kBloomErr = 0.000001;   // keyhunt.cpp:1238, 1267, 1296

uint64_t items_for(uint64_t m, uint64_t limit) {   // keyhunt.cpp:1185-1213
  if (m / 256 > limit) return m / 256 + ((m % 256) ? 1 : 0);
  return 1000;
}

// One 1024-point group centred on c over stride table tab/tab2 (keyhunt.cpp:4438-4578):
// xs[t] = x(c + (t - 512) * stride) for t in [0, 1024), then c += 1024 * stride.
void group_x(Pt& c, const Pt* tab, const Pt& tab2, Fh* xs, Fh* dx, Fh* pre) {
  for (int i = 0; i < kHalf; ++i) fe_sub(dx[i], tab[i].x, c.x);
  fe_sub(dx[kHalf], tab2.x, c.x);
  // Montgomery batch inverse over 513 values (IntGroup.cpp:36-58); a zero product gives 0s.
  pre[0] = dx[0];
  for (int i = 1; i <= kHalf; ++i) fe_mul(pre[i], pre[i - 1], dx[i]);
  Fh inv;
  fe_inv(inv, pre[kHalf]);
  for (int i = kHalf; i > 0; --i) {
    Fh nv;
    fe_mul(nv, pre[i - 1], inv);
    fe_mul(inv, inv, dx[i]);
    dx[i] = nv;
  }
  dx[0] = inv;
  xs[kHalf] = c.x;
  for (int i = 0; i < kHalf; ++i) {
    Fh u, s, x;
    fe_add(u, c.x, tab[i].x);
    fe_add(s, tab[i].y, c.y);         // c - tab[i]: s^2 = ((tab.y + c.y)/dx)^2
    fe_mul(s, s, dx[i]);
    fe_sqr(x, s);
    fe_sub(xs[kHalf - 1 - i], x, u);
    if (i < kHalf - 1) {
      fe_sub(s, tab[i].y, c.y);
      fe_mul(s, s, dx[i]);
      fe_sqr(x, s);
      fe_sub(xs[kHalf + 1 + i], x, u);
    }
  }
  Fh s, nx, ny;
  fe_sub(s, tab2.y, c.y);
  fe_mul(s, s, dx[kHalf]);
  fe_sqr(nx, s);
  fe_sub(nx, nx, c.x);
  fe_sub(nx, nx, tab2.x);
  fe_sub(ny, tab2.x, nx);
  fe_mul(ny, ny, s);
  fe_sub(ny, ny, tab2.y);
  c.x = nx;
  c.y = ny;
}

}  // namespace

bool make_geometry(const char* n_str, int kfactor, Geometry& g, std::string& err) {
  g = Geometry();
  if (n_str) {
    bool ok = (n_str[0] == '0' && n_str[1] == 'x') ? U256::from_hex(n_str + 2, g.N) : U256::from_dec(n_str, g.N);
    if (!ok) { err = "[E] invalid -n value"; return false; }
  } else {
    g.N = U256(0x100000000000ull);                      // keyhunt.cpp:1066
  }
  // keyhunt.cpp:1069-1076: "exact root" = Euler's criterion mod p; root = ModSqrt mod p.
  if (g.N >= secp_prime()) { err = "[E] -n param doesn't have exact square root"; return false; }
  Fh nf = fe_of(g.N), mf;
  if (!fe_has_sqrt(nf)) { err = "[E] -n param doesn't have exact square root"; return false; }
  fe_sqrt(mf, nf);
  g.M = u256_of(mf);
  U256 r;
  U256::divmod(g.M, U256(kGrp), nullptr, &r);
  if (!r.is_zero()) { err = "[E] M value is not divisible by 1024"; return false; }
  // keyhunt.cpp:1129-1179
  g.M = g.M * (uint64_t)(kfactor <= 0 ? 1 : kfactor);
  U256::divmod(g.M, U256(32), &g.M2, &r);
  if (!r.is_zero()) g.M2 = g.M2 + U256(1);
  g.M_double = g.M * 2ull;
  g.M2_double = g.M2 * 2ull;
  U256::divmod(g.M2, U256(32), &g.M3, &r);
  if (!r.is_zero()) g.M3 = g.M3 + U256(1);
  g.M3_double = g.M3 * 2ull;
  U256 aux;
  U256::divmod(g.N, g.M, &aux, &r);
  if (!r.is_zero()) g.N = g.M * aux;
  g.N_double = g.N * 2ull;
  if (!g.M.fits64() || g.M.w[0] > (1ull << 40) || !aux.fits64()) {
    err = "[E] baby-step table too large";
    return false;
  }
  g.m = g.M.w[0];
  g.m2 = g.M2.w[0];
  g.m3 = g.M3.w[0];
  g.aux = aux.w[0];
  g.items1 = items_for(g.m, 10000);
  g.items2 = items_for(g.m2, 1000);
  g.items3 = items_for(g.m3, 1000);
  g.cycles = g.aux / kGrp + ((g.aux % kGrp) ? 1 : 0);     // keyhunt.cpp:3810-3813
  g.intaux = g.M_double * (uint64_t)kHalf + g.M;           // keyhunt.cpp:3815-3817
  // L1 extent: the last 2^20-key build job's `to` overshoots m by one job when m is not a
  // multiple of the job size (keyhunt.cpp:1739-1793 with thread_bPload's "i_counter < to").
  uint64_t W = kJobKeys >= g.m ? g.m : kJobKeys;
  uint64_t R = g.m % W;
  g.l1ext = R ? (g.m / W) * W + W + R : g.m;
  return true;
}

// Baby-step walk on the GPU (khb_build_baby): jobs of 2^20 keys, centre key k*2^20 + 513.
static bool build_baby_gpu(Tables& T, const Geometry& g, const std::vector<Pt>& gn, const Pt& g2n, uint64_t extent,
                           bool need_l1, bool need_l2, bool need_l3, bool need_bp, uint32_t gate_log2, int device,
                           int nthreads, double& kernel_ms, std::string& err) {
  const uint32_t gpj = 1024, gpl = 4;
  const uint64_t job_keys = (uint64_t)gpj * kGrp;
  const uint32_t n_jobs = (uint32_t)((extent + job_keys - 1) / job_keys);
  std::vector<uint8_t> centres(64 * (size_t)n_jobs), tab(513 * 64), offs(64 * (gpj / gpl));
  {
    std::atomic<uint32_t> next{0};
    auto work = [&] {
      for (uint32_t k; (k = next.fetch_add(1)) < n_jobs;)
        pt_to_be(centres.data() + 64 * (size_t)k, mul_g(U256((uint64_t)k * job_keys + 1 + kHalf)));
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
  }
  for (int i = 0; i < kHalf; ++i) pt_to_be(tab.data() + 64 * i, gn[i]);
  pt_to_be(tab.data() + 64 * kHalf, g2n);
  for (uint32_t m = 1; m < gpj / gpl; ++m) pt_to_be(offs.data() + 64 * m, mul_g(U256((uint64_t)m * gpl * kGrp)));
  khb_ctx* ctx = nullptr;
  int rc = khb_open(device, 0, &ctx);
  if (rc) {
    err = std::string("[E] GPU table build: ") + khb_strerror(rc);
    return false;
  }
  const uint64_t bytes[3] = {T.l1[0].bytes, T.l2[0].bytes, T.l3[0].bytes};
  const uint64_t bits[3] = {T.l1[0].bits, T.l2[0].bits, T.l3[0].bits};
  const uint32_t hashes[3] = {T.l1[0].hashes, T.l2[0].hashes, T.l3[0].hashes};
  std::vector<uint8_t> cat[3];
  if (need_l1) cat[0].assign(256 * bytes[0], 0);
  if (need_l2) cat[1].assign(256 * bytes[1], 0);
  if (need_l3) cat[2].assign(256 * bytes[2], 0);
  float ms = 0;
  if (!(rc = khb_load_giant_table(ctx, tab.data())) &&
      !(rc = khb_load_lane_offsets(ctx, offs.data(), gpj / gpl, gpl)))
    rc = khb_build_baby(ctx, centres.data(), n_jobs, gpj, g.l1ext, g.m2, g.m3, bytes, bits, hashes,
                        need_l1 ? cat[0].data() : nullptr, need_l2 ? cat[1].data() : nullptr,
                        need_l3 ? cat[2].data() : nullptr, need_bp ? (uint8_t*)T.bp.data() : nullptr,
                        gate_log2 ? T.gate.data() : nullptr, gate_log2, T.gate_probes, &ms);
  khb_close(ctx);
  if (rc) {
    err = std::string("[E] GPU table build: ") + khb_strerror(rc);
    return false;
  }
  kernel_ms = ms;
  std::vector<BloomFilter>* lv[3] = {&T.l1, &T.l2, &T.l3};
  for (int l = 0; l < 3; ++l)
    if (!cat[l].empty())
      for (int i = 0; i < 256; ++i) memcpy((*lv[l])[i].bf.data(), cat[l].data() + i * bytes[l], bytes[l]);
  return true;
}

uint32_t Tables::gate_probes_for() {
  uint32_t p = 3;
  if (const char* e = getenv("KHB_GATE_PROBES")) p = (uint32_t)atoi(e);
  return p < 1 ? 1 : (p > KHB_GATE_MAX_PROBES ? KHB_GATE_MAX_PROBES : p);
}

uint32_t Tables::gate_log2_for(const Geometry& g) {
  uint32_t cap = 30, sparsity = 6;
  if (const char* e = getenv("KHB_GATE_LOG2")) cap = (uint32_t)atoi(e);
  if (const char* e = getenv("KHB_GATE_SPARSITY")) sparsity = (uint32_t)atoi(e);
  if (cap == 0 || g.l1ext == 0) return 0;
  if (cap < 13) cap = 13;
  if (cap > 32) cap = 32;
  if (sparsity > 8) sparsity = 8;
  uint32_t lg = 13;
  while (lg < cap && (1ull << lg) < (g.l1ext << sparsity)) ++lg;
  return (1ull << lg) < 4 * g.l1ext ? 0 : lg;   // more than ~22 % full: not worth a load
}

void Tables::prepare(const Geometry& g) {
  geo = g;
  l1.assign(256, BloomFilter());
  l2.assign(256, BloomFilter());
  l3.assign(256, BloomFilter());
  bp.assign(g.m3, XValue());
}

bool Tables::build(const Geometry& g, int nthreads, uint32_t groups_per_lane, std::string& err,
                   const std::function<void(uint64_t, uint64_t)>& progress, uint32_t have, int gpu_device) {
  if (!have) prepare(g);
  geo = g;
  for (int i = 0; i < 256; ++i) {
    if ((!(have & kFileL1) && l1[i].init2(g.items1, kBloomErr)) || (!(have & kFileL2) && l2[i].init2(g.items2, kBloomErr)) ||
        (!(have & kFileL3) && l3[i].init2(g.items3, kBloomErr))) {
      err = "[E] error bloom_init";
      return false;
    }
  }
  if (!(have & kFileBp)) bp.assign(g.m3, XValue());
  const bool need_l1 = !(have & kFileL1), need_l2 = !(have & kFileL2), need_l3 = !(have & kFileL3),
             need_bp = !(have & kFileBp);
  // level-0 gate: built wherever the whole L1 set is walked (the GPU walks it for the gate alone)
  gate_log2 = (need_l1 || gpu_device >= 0) ? gate_log2_for(g) : 0;
  gate_probes = gate_log2 ? gate_probes_for() : 0;
  gate.assign(gate_log2 ? (size_t)1 << (gate_log2 - 3) : 0, 0);
  // baby steps to walk: all of the L1 extent, or only the first m2 when L1 came from a file
  const uint64_t extent = (need_l1 || (gate_log2 && gpu_device >= 0)) ? g.l1ext
                          : ((need_l2 || need_l3 || need_bp) ? g.m2 : 0);
  // giant tables (keyhunt.cpp:1309-1364)
  {
    Pt bsP = negation(mul_g(g.M_double));
    Pt q = bsP;
    gsn[0] = q;
    q = double_direct(q);
    gsn[1] = q;
    for (int i = 2; i < kHalf; ++i) { q = add_direct(q, bsP); gsn[i] = q; }
    g2sn = double_direct(gsn[kHalf - 1]);
    Pt t;
    amp2[0] = negation(mul_g(g.M2));
    t = negation(mul_g(g.M2_double));
    for (int i = 1; i < 32; ++i) amp2[i] = add_direct(amp2[i - 1], t);
    amp3[0] = negation(mul_g(g.M3));
    t = negation(mul_g(g.M3_double));
    for (int i = 1; i < 32; ++i) amp3[i] = add_direct(amp3[i - 1], t);
  }
  // lane offsets for the GPU: offs[m] = (m * gpl) * _2GSn = -(m * gpl * 2048 * M) * G
  gpl = groups_per_lane ? groups_per_lane : 1;
  const uint64_t n_off = (g.cycles + gpl - 1) / gpl;
  lane_offs.assign(n_off, Pt());
  // baby-step stride table Gn (init_generator, keyhunt.cpp:4386-4399)
  std::vector<Pt> gn(kHalf);
  Pt g2n;
  {
    Pt q = secp_g();
    gn[0] = q;
    q = double_direct(q);
    gn[1] = q;
    for (int i = 2; i < kHalf; ++i) { q = add_direct(q, secp_g()); gn[i] = q; }
    g2n = double_direct(gn[kHalf - 1]);
  }
  // build jobs (keyhunt.cpp:1739-1807): [from, to) of 2^20 keys, last job overshooting (quirk vi)
  struct Job { uint64_t from, to; };
  std::vector<Job> jobs;
  if (extent) {
    const uint64_t span = need_l1 ? g.m : extent;   // with L1 from a file: the m2 rebuild jobs
    uint64_t W = kJobKeys >= span ? span : kJobKeys;
    uint64_t cyc = span / W, R = span % W;
    if (R) cyc++;
    uint64_t base = 0;
    for (uint64_t j = 0; j < cyc; ++j) {
      jobs.push_back({base, j < cyc - 1 ? base + W : base + W + R});
      base += W;
    }
  }
  if (nthreads < 1) nthreads = 1;
  if (gpu_device >= 0 && extent) {
    if (!build_baby_gpu(*this, g, gn, g2n, extent, need_l1, need_l2, need_l3, need_bp, gate_log2, gpu_device,
                        nthreads, build_gpu_ms, err))
      return false;
    jobs.clear();   // the CPU workers below only compute the lane offsets
    if (progress) progress(extent, extent);
  }
  std::atomic<uint64_t> next_job{0}, next_off{1}, done{0};
  std::atomic<int> finished{0};
  auto worker = [&]() {
    std::vector<Fh> xs(kGrp), dx(kHalf + 1), pre(kHalf + 1);
    uint8_t xb[32];
    for (;;) {
      const uint64_t j = next_job.fetch_add(1);
      if (j >= jobs.size()) break;
      const uint64_t from = jobs[j].from, to = jobs[j].to;
      const uint64_t nb = (to - from) / kGrp + (((to - from) % kGrp) ? 1 : 0);
      Pt c = mul_g(U256(from + 1 + kHalf));
      uint64_t ic = from;
      for (uint64_t s = 0; s < nb; ++s) {
        group_x(c, gn.data(), g2n, xs.data(), dx.data(), pre.data());
        for (int t = 0; t < kGrp; ++t, ++ic) {
          fe_to_be(xb, xs[t]);
          const int idx = xb[0];
          if (ic < g.m3) {
            if (need_bp) {
              memcpy(bp[ic].value, xb + 16, 6);
              bp[ic].index = ic;
            }
            if (need_l3) l3[idx].add32_atomic(xb);
          }
          if (need_l2 && ic < g.m2) l2[idx].add32_atomic(xb);
          if (need_l1 && ic < to) {
            l1[idx].add32_atomic(xb);
            // blocked gate (khb_load_gate): block w0 mod 2^(gate_log2-6), bit (w1 >> 5p) mod 32 of word p mod 2;
            // w0 = x mod 2^32 is big-endian bytes 28..31, w1 = (x >> 32) mod 2^32 bytes 24..27
            if (gate_probes) {
              const uint32_t w0 = ((uint32_t)xb[28] << 24) | ((uint32_t)xb[29] << 16) | ((uint32_t)xb[30] << 8) | xb[31];
              const uint32_t w1 = ((uint32_t)xb[24] << 24) | ((uint32_t)xb[25] << 16) | ((uint32_t)xb[26] << 8) | xb[27];
              const uint64_t blk = w0 & (uint32_t)((1ull << (gate_log2 - 6)) - 1);
              for (uint32_t p = 0; p < gate_probes; ++p) {
                const uint32_t b = 32u * (p & 1u) + ((w1 >> (5 * p)) & 31u);
                __atomic_fetch_or(&gate[8 * blk + (b >> 3)], (uint8_t)(1u << (b & 7)), __ATOMIC_RELAXED);
              }
            }
          }
        }
        done.fetch_add(kGrp);
      }
    }
    // lane offsets share the pool
    for (;;) {
      const uint64_t m = next_off.fetch_add(1);
      if (m >= n_off) break;
      lane_offs[m] = negation(mul_g(g.M_double * (uint64_t)(m * gpl * kHalf * 2)));
    }
    finished.fetch_add(1);
  };
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) th.emplace_back(worker);
  while (progress && finished.load() < nthreads) {
    progress(done.load(), extent);
    std::this_thread::sleep_for(std::chrono::milliseconds(250));
  }
  for (auto& x : th) x.join();
  if (progress) progress(extent, extent);
  // bsgs_sort (keyhunt.cpp:3657-3746): for distinct 6-byte keys any correct sort gives the same
  // array; equal keys (SURVEY §8a quirk v) are ordered by index here.
  if (need_bp)
    std::sort(bp.begin(), bp.end(), [](const XValue& a, const XValue& b) {
      int r = memcmp(a.value, b.value, 6);
      return r ? r < 0 : a.index < b.index;
    });
  return true;
}

std::vector<uint8_t> Tables::l1_concat() const {
  std::vector<uint8_t> out(256 * l1[0].bytes);
  for (int i = 0; i < 256; ++i) memcpy(out.data() + i * l1[0].bytes, l1[i].bf.data(), l1[0].bytes);
  return out;
}

std::vector<uint8_t> Tables::bloom_concat(int level) const {
  const std::vector<BloomFilter>& L = level == 1 ? l1 : level == 2 ? l2 : l3;
  std::vector<uint8_t> out(256 * L[0].bytes);
  for (int i = 0; i < 256; ++i) memcpy(out.data() + i * L[0].bytes, L[i].bf.data(), L[0].bytes);
  return out;
}

std::vector<uint8_t> Tables::amp_table_be(int level) const {
  std::vector<uint8_t> out(32 * 64);
  for (int i = 0; i < 32; ++i) pt_to_be(out.data() + 64 * i, level == 2 ? amp2[i] : amp3[i]);
  return out;
}

std::vector<uint8_t> Tables::giant_table_be() const {
  std::vector<uint8_t> out(513 * 64);
  for (int i = 0; i < kHalf; ++i) pt_to_be(out.data() + 64 * i, gsn[i]);
  pt_to_be(out.data() + 64 * kHalf, g2sn);
  return out;
}

std::vector<uint8_t> Tables::lane_offsets_be() const {
  std::vector<uint8_t> out(64 * lane_offs.size());
  for (size_t i = 0; i < lane_offs.size(); ++i) pt_to_be(out.data() + 64 * i, lane_offs[i]);
  return out;
}

Pt Tables::chunk_aux(const U256& base) const {
  U256 km = secp_order() - base - geo.intaux;
  return mul_g(km);
}

void batch_add_direct(const Pt* targets, const Pt& aux, size_t n, Pt* out) {
  std::vector<Fh> dx(n), pre(n);
  for (size_t k = 0; k < n; ++k) fe_sub(dx[k], aux.x, targets[k].x);
  fe_batch_inv(dx.data(), n, pre.data());
  for (size_t k = 0; k < n; ++k) {
    Fh dy, s, p;
    Pt r;
    fe_sub(dy, aux.y, targets[k].y);
    fe_mul(s, dy, dx[k]);
    fe_sqr(p, s);
    fe_sub(r.x, p, targets[k].x);
    fe_sub(r.x, r.x, aux.x);
    fe_sub(r.y, aux.x, r.x);
    fe_mul(r.y, r.y, s);
    fe_sub(r.y, r.y, aux.y);
    out[k] = r;
  }
}

// out[i] = AddDirect(a[i], b[i]) for i < n with one shared inversion (SECP256K1.cpp:242-265
// semantics per element: a zero x-difference gets inverse 0, as batch_add_direct).
void batch_add_pairs(const Pt* a, const Pt* b, size_t n, Pt* out) {
  std::vector<Fh> dx(n), pre(n);
  for (size_t k = 0; k < n; ++k) fe_sub(dx[k], b[k].x, a[k].x);
  fe_batch_inv(dx.data(), n, pre.data());
  for (size_t k = 0; k < n; ++k) {
    Fh dy, s, p;
    Pt r;
    fe_sub(dy, b[k].y, a[k].y);
    fe_mul(s, dy, dx[k]);
    fe_sqr(p, s);
    fe_sub(r.x, p, a[k].x);
    fe_sub(r.x, r.x, b[k].x);
    fe_sub(r.y, b[k].x, r.x);
    fe_mul(r.y, r.y, s);
    fe_sub(r.y, r.y, b[k].y);
    out[k] = r;
  }
}

// Chunk auxiliaries aux(base_c) = (order - base_c - intaux) G (keyhunt.cpp:3861-3866) for
// base_c = base0 + c * 2N, c < n: one scalar multiplication per block of kAuxBlock chunks, the rest
// aux(block start) - j * 2N G by batched affine additions (one inversion per block).  A degenerate
// addition (aux(block start) = +-j * 2N G) falls back to the scalar multiplication.
void Tables::chunk_aux_run(const U256& base0, size_t n, Pt* aux, int threads) const {
  constexpr size_t kAuxBlock = 64;
  if (n == 0) return;
  const Pt D = mul_g(secp_order() - geo.N_double);          // -(2N) G
  std::vector<Pt> jd(kAuxBlock);                             // jd[j] = j * D, j >= 1
  jd[1] = D;
  jd[2] = mul_g(secp_order() - geo.N_double * 2ull);         // not D + D: AddDirect cannot double
  for (size_t j = 3; j < kAuxBlock; ++j) jd[j] = add_direct(jd[j - 1], D);
  const size_t blocks = (n + kAuxBlock - 1) / kAuxBlock;
  const U256 lim = secp_order() - geo.intaux;                // chunk_aux's km = lim - base wraps at base > lim
  auto body = [&](size_t blk) {
    const size_t s = blk * kAuxBlock, m = std::min(kAuxBlock, n - s);
    const U256 bs = base0 + geo.N_double * (uint64_t)s;
    if (bs >= lim || lim - bs <= geo.N_double * (uint64_t)(m - 1)) {
      // the block reaches the group order: km of a later chunk is 0 (the identity) or wraps mod 2^256
      // (not mod n) in chunk_aux, which the walk from the block start would not reproduce
      for (size_t j = 0; j < m; ++j) aux[s + j] = chunk_aux(bs + geo.N_double * (uint64_t)j);
      return;
    }
    aux[s] = chunk_aux(bs);
    if (m < 2) return;
    std::vector<Pt> a(m - 1, aux[s]);
    batch_add_pairs(a.data(), jd.data() + 1, m - 1, aux + s + 1);
    for (size_t j = 1; j < m; ++j)
      if (fe_eq(aux[s].x, jd[j].x)) aux[s + j] = chunk_aux(bs + geo.N_double * (uint64_t)j);
  };
  if (threads <= 1 || blocks < 2) {
    for (size_t b = 0; b < blocks; ++b) body(b);
    return;
  }
  std::atomic<size_t> next{0};
  auto worker = [&]() {
    for (size_t b; (b = next.fetch_add(1)) < blocks;) body(b);
  };
  std::vector<std::thread> th;
  for (int t = 1; t < threads && (size_t)t < blocks; ++t) th.emplace_back(worker);
  worker();
  for (auto& t : th) t.join();
}

bool Tables::searchbinary(const uint8_t* x, uint64_t& idx) const {
  // bsgs_searchbinary (keyhunt.cpp:3748-3773), its own probe sequence (bytes 16..21 of x): with equal
  // 6-byte keys in bPtable the entry it lands on, and so the key the third check tries, is the reference's
  int64_t min = 0, max = (int64_t)bp.size(), half = max, current = 0;
  while (half >= 1) {
    half = (max - min) / 2;
    const int r = memcmp(x + 16, bp[(size_t)(current + half)].value, 6);
    if (r == 0) { idx = bp[(size_t)(current + half)].index; return true; }
    if (r < 0) max = max - half;
    else min = min + half;
    current = min;
  }
  return false;
}

static U256 calc_index(const Geometry& g, uint32_t i) {   // calcualteindex, keyhunt.cpp:6680-6689
  return g.M3_double * (uint64_t)i + g.M3;
}

// AddDirect(q, tab[i]) for i < 32 with one shared inversion (same values as 32 separate
// AddDirects, incl. dx == 0 -> inverse 0).
static void add_direct_32(const Pt& q, const Pt* tab, Pt* out) {
  Fh dx[32], pre[32];
  for (int i = 0; i < 32; ++i) fe_sub(dx[i], tab[i].x, q.x);
  fe_batch_inv(dx, 32, pre);
  for (int i = 0; i < 32; ++i) {
    Fh dy, s, p;
    fe_sub(dy, tab[i].y, q.y);
    fe_mul(s, dy, dx[i]);
    fe_sqr(p, s);
    fe_sub(out[i].x, p, q.x);
    fe_sub(out[i].x, out[i].x, tab[i].x);
    fe_sub(out[i].y, tab[i].x, out[i].x);
    fe_mul(out[i].y, out[i].y, s);
    fe_sub(out[i].y, out[i].y, tab[i].y);
  }
}

bool Tables::thirdcheck(const U256& start, uint32_t a, const Pt& target, U256& key) const {
  U256 base = geo.M2_double * (uint64_t)a + start;
  const Pt Q = add_direct(target, negation(mul_g(base)));
  Pt S32[32];
  add_direct_32(Q, amp3, S32);
  uint8_t xb[32];
  for (int i = 0; i < 32; ++i) {
    const Pt& S = S32[i];
    fe_to_be(xb, S.x);
    if (l3[xb[0]].check32(xb)) {
      uint64_t j = 0;
      if (searchbinary(xb, j)) {
        const U256 ci = calc_index(geo, (uint32_t)i);
        key = ci + U256(j + 1) + base;
        if (fe_eq(mul_g(key).x, target.x)) return true;
        key = ci - U256(j + 1) + base;
        if (fe_eq(mul_g(key).x, target.x)) return true;
      }
    } else if (fe_eq(Q.x, amp3[i].x)) {        // AddDirect(P,-P) special case, keyhunt.cpp:4352-4364
      key = calc_index(geo, (uint32_t)i) + base;
      return true;
    }
  }
  return false;
}

bool Tables::secondcheck(const U256& start, uint32_t a, const Pt& target, U256& key) const {
  U256 base = geo.M_double * (uint64_t)a + start;
  const Pt Q = add_direct(target, negation(mul_g(base)));
  Pt S32[32];
  add_direct_32(Q, amp2, S32);
  uint8_t xb[32];
  for (int i = 0; i < 32; ++i) {
    fe_to_be(xb, S32[i].x);
    if (l2[xb[0]].check32(xb)) {
      if (thirdcheck(base, (uint32_t)i, target, key)) return true;
    }
  }
  return false;
}

}  // namespace khb
