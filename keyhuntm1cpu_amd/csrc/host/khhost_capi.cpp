// libkhhost.so: C ABI over the host engine (include/khhost.h).
#include <string.h>

#include <string>
#include <thread>
#include <vector>

#include "../../../include/khbsgs.h"
#include "../../../include/khhost.h"
#include "address_host.hpp"
#include "bsgs_host.hpp"
#include "engine.hpp"

using namespace khb;

struct khh_tables {
  Tables t;
};

struct khh_addr {
  AddrTargets T;
  AddrGen G;
  uint64_t n_seq = 0;
  uint32_t hit_cap = 0;      // tests: bloom-hit ring capacity per launch (0 = library default)
};

static void set_err(char* err, size_t n, const std::string& m) {
  if (err && n) {
    strncpy(err, m.c_str(), n - 1);
    err[n - 1] = 0;
  }
}

extern "C" {

int khh_abi_version(void) { return KHH_ABI_VERSION; }

khh_tables* khh_tables_new(const char* n_str, int k, int threads, uint32_t gpl, char* err, size_t errlen) {
  Geometry g;
  std::string e;
  if (!make_geometry(n_str, k, g, e)) { set_err(err, errlen, e); return nullptr; }
  khh_tables* t = new khh_tables();
  if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
  if (!t->t.build(g, threads, gpl ? gpl : 4, e)) {
    set_err(err, errlen, e);
    delete t;
    return nullptr;
  }
  return t;
}

khh_tables* khh_tables_new_files(const char* n_str, int k, int threads, uint32_t gpl, const char* dir,
                                 int skip_checksum, int save, uint32_t* have, char* err, size_t errlen) {
  Geometry g;
  std::string e;
  if (!make_geometry(n_str, k, g, e)) { set_err(err, errlen, e); return nullptr; }
  khh_tables* t = new khh_tables();
  if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
  uint32_t h = 0;
  t->t.prepare(g);
  if (!t->t.load_files(dir ? dir : ".", skip_checksum != 0, h, e, nullptr) ||
      !t->t.build(g, threads, gpl ? gpl : 4, e, nullptr, h) ||
      (save && h != kFileAll && !t->t.save_files(dir ? dir : ".", h, e, nullptr))) {
    set_err(err, errlen, e);
    delete t;
    return nullptr;
  }
  if (have) *have = h;
  return t;
}

khh_tables* khh_tables_new_gpu(const char* n_str, int k, int threads, uint32_t gpl, int device, double* kernel_ms,
                               char* err, size_t errlen) {
  Geometry g;
  std::string e;
  if (!make_geometry(n_str, k, g, e)) { set_err(err, errlen, e); return nullptr; }
  khh_tables* t = new khh_tables();
  if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
  if (!t->t.build(g, threads, gpl ? gpl : 4, e, nullptr, 0, device)) {
    set_err(err, errlen, e);
    delete t;
    return nullptr;
  }
  if (kernel_ms) *kernel_ms = t->t.build_gpu_ms;
  return t;
}

int khh_tables_save(const khh_tables* t, const char* dir, char* err, size_t errlen) {
  std::string e;
  if (!t->t.save_files(dir ? dir : ".", 0, e, nullptr)) {
    set_err(err, errlen, e);
    return -100;
  }
  return 0;
}

void khh_tables_free(khh_tables* t) { delete t; }

void khh_params(const khh_tables* t, uint64_t out[10]) {
  const Geometry& g = t->t.geo;
  out[0] = g.m; out[1] = g.m2; out[2] = g.m3; out[3] = g.aux; out[4] = g.cycles;
  out[5] = g.N.w[0]; out[6] = g.l1ext; out[7] = g.items1; out[8] = g.items2; out[9] = g.items3;
}

const uint8_t* khh_bloom(const khh_tables* t, int level, int idx, uint64_t* bytes, uint64_t* bits, uint32_t* hashes) {
  if (idx < 0 || idx > 255 || level < 1 || level > 3) return nullptr;
  const BloomFilter& b = level == 1 ? t->t.l1[idx] : level == 2 ? t->t.l2[idx] : t->t.l3[idx];
  if (bytes) *bytes = b.bytes;
  if (bits) *bits = b.bits;
  if (hashes) *hashes = b.hashes;
  return b.bf.data();
}

void khh_giant_table(const khh_tables* t, uint8_t out[513 * 64]) {
  std::vector<uint8_t> v = t->t.giant_table_be();
  memcpy(out, v.data(), v.size());
}

void khh_amp_table(const khh_tables* t, int level, uint8_t out[32 * 64]) {
  const Pt* a = level == 2 ? t->t.amp2 : t->t.amp3;
  for (int i = 0; i < 32; ++i) pt_to_be(out + 64 * i, a[i]);
}

uint32_t khh_lane_offsets(const khh_tables* t, uint8_t* out, uint32_t* gpl) {
  if (gpl) *gpl = t->t.gpl;
  if (out) {
    std::vector<uint8_t> v = t->t.lane_offsets_be();
    memcpy(out, v.data(), v.size());
  }
  return (uint32_t)t->t.lane_offs.size();
}

uint32_t khh_gate_probes(const khh_tables* t) { return t->t.gate_probes; }

const uint8_t* khh_gate(const khh_tables* t, uint32_t* log2) {
  if (log2) *log2 = t->t.gate_log2;
  return t->t.gate_log2 ? t->t.gate.data() : nullptr;
}

const uint8_t* khh_bptable(const khh_tables* t, uint64_t* n) {
  static_assert(sizeof(XValue) == 16, "bsgs_xvalue is 16 bytes");
  if (n) *n = t->t.bp.size();
  return reinterpret_cast<const uint8_t*>(t->t.bp.data());
}

int khh_chunk_centre(const khh_tables* t, const uint8_t base_be[32], const uint8_t target_xy[64], uint8_t out_xy[64]) {
  const U256 base = U256::from_be(base_be);
  const Pt tg = pt_from_be(target_xy);
  const Pt aux = t->t.chunk_aux(base);
  Pt c;
  batch_add_direct(&tg, aux, 1, &c);
  pt_to_be(out_xy, c);
  return 0;
}

int khh_job_centres(const khh_tables* t, const uint8_t* bases_be, uint32_t n_chunks, const uint8_t* targets_xy,
                    uint32_t n_targets, uint8_t* out_xy, int threads) {
  if (!t || !bases_be || !targets_xy || !out_xy) return -1;
  std::vector<U256> bases(n_chunks);
  for (uint32_t c = 0; c < n_chunks; ++c) bases[c] = U256::from_be(bases_be + 32 * (size_t)c);
  std::vector<Pt> tp(n_targets);
  for (uint32_t j = 0; j < n_targets; ++j) tp[j] = pt_from_be(targets_xy + 64 * (size_t)j);
  job_centres(t->t, bases, tp, out_xy, threads);
  return 0;
}

int khh_secondcheck(const khh_tables* t, const uint8_t base_be[32], uint32_t a, const uint8_t target_xy[64],
                    uint8_t key_be[32]) {
  U256 key;
  if (!t->t.secondcheck(U256::from_be(base_be), a, pt_from_be(target_xy), key)) return 0;
  key.to_be(key_be);
  return 1;
}

struct khh_session {
  Session s;
  bool record = false;                 // tests: keep every level-1 candidate of the last run
  struct Rec {
    U256 base;
    uint32_t target, a;
  };
  std::vector<Rec> recorded;
};

khh_session* khh_session_open(const khh_tables* t, const int* devices, int n_devices, uint32_t lanes,
                              uint32_t chunks_per_batch, int check_threads, char* err, size_t errlen) {
  if (!t || !devices || n_devices <= 0) { set_err(err, errlen, "[E] bad arguments"); return nullptr; }
  SearchConfig cfg;
  cfg.devices.assign(devices, devices + n_devices);
  cfg.lanes = lanes;
  cfg.chunks_per_batch = chunks_per_batch;
  cfg.check_threads = check_threads;
  khh_session* s = new khh_session();
  std::string e;
  if (s->s.open(t->t, cfg, e)) {
    set_err(err, errlen, e);
    delete s;
    return nullptr;
  }
  return s;
}

void khh_session_close(khh_session* s) { delete s; }

int khh_session_run(khh_session* s, const uint8_t* targets_xy, int n_targets, const uint8_t start_be[32],
                    const uint8_t end_be[32], uint64_t max_chunks, int random_chunks, int* found, uint8_t* keys_be,
                    uint64_t* stats_out, char* err, size_t errlen) {
  return khh_session_run_ex(s, targets_xy, n_targets, start_be, end_be, max_chunks, random_chunks, found, keys_be,
                            stats_out, stats_out ? 6 : 0, err, errlen);
}

int khh_session_run_ex(khh_session* s, const uint8_t* targets_xy, int n_targets, const uint8_t start_be[32],
                       const uint8_t end_be[32], uint64_t max_chunks, int random_chunks, int* found, uint8_t* keys_be,
                       uint64_t* stats_out, uint32_t stats_len, char* err, size_t errlen) {
  if (!s || !targets_xy || n_targets <= 0) return KHB_EINVAL;
  std::vector<Target> tg((size_t)n_targets);
  for (int k = 0; k < n_targets; ++k) tg[k].p = pt_from_be(targets_xy + 64 * k);
  SearchCallbacks cb;
  s->recorded.clear();
  if (s->record)
    cb.on_candidate = [s](const U256& base, int k, uint32_t a) { s->recorded.push_back({base, (uint32_t)k, a}); };
  std::vector<int> f;
  std::vector<U256> keys;
  SearchStats st;
  std::string e;
  int rc = s->s.run(tg, U256::from_be(start_be), U256::from_be(end_be), cb, f, keys, st, e, max_chunks,
                    random_chunks != 0);
  for (int k = 0; k < n_targets; ++k) {
    if (found) found[k] = f.empty() ? 0 : f[k];
    if (keys_be) (f.empty() ? U256() : keys[k]).to_be(keys_be + 32 * k);
  }
  if (stats_out) {
    const uint64_t v[KHH_SESSION_STATS] = {
        st.chunks, st.giant_steps, st.candidates, st.degenerate, (uint64_t)(st.kernel_seconds * 1e6), st.launches,
        st.rescans, (uint64_t)(st.busy_seconds * 1e6),
        st.shader_mhz_n ? (uint64_t)(1e3 * st.shader_mhz_sum / st.shader_mhz_n) : 0, st.device_checked,
        (uint64_t)(st.device_check_seconds * 1e6), (uint64_t)(st.event_seconds * 1e6)};
    memcpy(stats_out, v, sizeof(uint64_t) * (stats_len < KHH_SESSION_STATS ? stats_len : KHH_SESSION_STATS));
  }
  if (rc) set_err(err, errlen, e);
  return rc;
}

int khh_session_set_test_hooks(khh_session* s, uint32_t cand_cap, int use_gate, int record, const uint8_t* l1_concat) {
  if (!s) return KHB_EINVAL;
  s->s.config().record_candidates = record != 0;
  s->record = record != 0;
  return s->s.set_test_hooks(cand_cap, use_gate != 0, l1_concat);
}

int khh_session_set_check_mode(khh_session* s, int mode) {
  if (!s) return KHB_EINVAL;
  return s->s.set_check_mode(mode);
}

int khh_session_set_chunk_mode(khh_session* s, int mode) {
  if (!s || mode < kChunkSequential || mode > kChunkDance) return KHB_EINVAL;
  s->s.config().chunk_mode = mode;
  return 0;
}

uint64_t khh_chunk_sequence(int mode, const uint8_t start_be[32], const uint8_t end_be[32], const uint8_t two_n_be[32],
                            uint64_t seed, uint8_t* out_be, uint64_t cap) {
  if (mode < kChunkSequential || mode > kChunkDance) return 0;
  const U256 two_n = U256::from_be(two_n_be);
  if (two_n == U256()) return 0;
  ChunkCursor c(mode, U256::from_be(start_be), U256::from_be(end_be), two_n, seed);
  uint64_t n = 0;
  U256 base;
  while (n < cap && c.next(base)) {
    if (out_be) base.to_be(out_be + 32 * n);
    n++;
  }
  return n;
}

void khh_gtable(uint8_t out[32 * 256 * 64]) {
  const std::vector<uint8_t>& g = gtable_be();
  memcpy(out, g.data(), g.size());
}

uint64_t khh_session_recorded(const khh_session* s, uint8_t* bases_be, uint32_t* targets, uint32_t* a, uint64_t cap) {
  if (!s) return 0;
  for (uint64_t i = 0; i < s->recorded.size() && i < cap; ++i) {
    if (bases_be) s->recorded[i].base.to_be(bases_be + 32 * i);
    if (targets) targets[i] = s->recorded[i].target;
    if (a) a[i] = s->recorded[i].a;
  }
  return s->recorded.size();
}

int khh_search(const khh_tables* t, const uint8_t* targets_xy, int n_targets, const uint8_t start_be[32],
               const uint8_t end_be[32], const int* devices, int n_devices, uint32_t lanes,
               uint32_t chunks_per_batch, uint64_t max_chunks, int* found, uint8_t* keys_be, uint64_t* stats_out,
               char* err, size_t errlen) {
  khh_session* s = khh_session_open(t, devices, n_devices, lanes, chunks_per_batch, 0, err, errlen);
  if (!s) return KHB_ENODEV;
  int rc = khh_session_run(s, targets_xy, n_targets, start_be, end_be, max_chunks, 0, found, keys_be, stats_out, err,
                           errlen);                                 // khh_search's stats hold 6
  khh_session_close(s);
  return rc;
}

int khh_pubkey(const uint8_t key_be[32], uint8_t out_xy[64]) {
  const U256 k = U256::from_be(key_be);
  if (k.is_zero() || k >= secp_order()) return KHB_EINVAL;
  pt_to_be(out_xy, mul_g(k));
  return 0;
}

int khh_parse_pubkey(const char* hex, uint8_t out_xy[64], int* compressed) {
  Pt p;
  bool c = true;
  if (!parse_pubkey_hex(hex, p, c, nullptr)) return KHB_EINVAL;
  pt_to_be(out_xy, p);
  if (compressed) *compressed = c ? 1 : 0;
  return 0;
}

khh_addr* khh_addr_new(const char* text, int bloom_multiplier, const uint8_t stride_be[32], uint64_t n_seq,
                       uint32_t gpl, int threads, char* err, size_t errlen) {
  if (!text || n_seq < 1024 || n_seq % 1024) {
    set_err(err, errlen, "n must be a positive multiple of 1024");
    return nullptr;
  }
  khh_addr* a = new khh_addr();
  std::string e;
  if (!AddrTargets::load_text(text, bloom_multiplier, a->T, &e)) {
    set_err(err, errlen, e);
    delete a;
    return nullptr;
  }
  const U256 stride = stride_be ? U256::from_be(stride_be) : U256(1);
  if (stride.is_zero()) {
    set_err(err, errlen, "stride must be positive");
    delete a;
    return nullptr;
  }
  if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
  a->n_seq = n_seq;
  a->G.build(stride, (uint32_t)(n_seq / 1024), gpl ? gpl : 16, threads);
  return a;
}

void khh_addr_free(khh_addr* a) { delete a; }

const uint8_t* khh_addr_table(const khh_addr* a, uint64_t* n) {
  if (n) *n = a->T.table.size();
  return a->T.table.empty() ? nullptr : a->T.table[0].data();
}

const uint8_t* khh_addr_bloom(const khh_addr* a, uint64_t* bytes, uint64_t* bits, uint32_t* hashes) {
  if (bytes) *bytes = a->T.bloom.bytes;
  if (bits) *bits = a->T.bloom.bits;
  if (hashes) *hashes = a->T.bloom.hashes;
  return a->T.bloom.bf.data();
}

void khh_addr_giant_table(const khh_addr* a, uint8_t out[513 * 64]) {
  const std::vector<uint8_t> v = a->G.table_be();
  memcpy(out, v.data(), v.size());
}

uint32_t khh_addr_lane_offsets(const khh_addr* a, uint8_t* out, uint32_t* gpl) {
  if (gpl) *gpl = a->G.gpl;
  if (out) {
    const std::vector<uint8_t> v = a->G.offs_be();
    memcpy(out, v.data(), v.size());
  }
  return (uint32_t)a->G.offs.size();
}

int khh_addr_search(const khh_addr* a, const uint8_t start_be[32], const uint8_t end_be[32], int search,
                    int random_chunks, const int* devices, int n_devices, uint32_t lanes, uint64_t max_chunks,
                    uint8_t* keys_be, uint8_t* compressed, uint8_t* rmd, uint32_t cap, uint32_t* n_found,
                    uint64_t* stats_out, char* err, size_t errlen) {
  return khh_addr_search_ex(a, start_be, end_be, search, random_chunks, devices, n_devices, lanes, max_chunks, keys_be,
                            compressed, rmd, cap, n_found, stats_out, stats_out ? 6 : 0, err, errlen);
}

int khh_addr_search_ex(const khh_addr* a, const uint8_t start_be[32], const uint8_t end_be[32], int search,
                       int random_chunks, const int* devices, int n_devices, uint32_t lanes, uint64_t max_chunks,
                       uint8_t* keys_be, uint8_t* compressed, uint8_t* rmd, uint32_t cap, uint32_t* n_found,
                       uint64_t* stats_out, uint32_t stats_len, char* err, size_t errlen) {
  const bool endo = search >= 0 && (search & KHB_SEARCH_ENDOMORPHISM);
  if (endo) search &= ~KHB_SEARCH_ENDOMORPHISM;
  if (!a || !start_be || !end_be || search < 0 || search > 2) return KHB_EINVAL;
  AddrConfig cfg;
  cfg.search = search;
  cfg.endomorphism = endo;
  cfg.start = U256::from_be(start_be);
  cfg.end = U256::from_be(end_be);
  cfg.n_seq = a->n_seq;
  cfg.random = random_chunks != 0;
  cfg.lanes = lanes;
  cfg.gpl = a->G.gpl;
  cfg.max_chunks = max_chunks;
  cfg.hit_cap = a->hit_cap;
  cfg.devices.clear();
  for (int i = 0; i < n_devices; ++i) cfg.devices.push_back(devices[i]);
  if (cfg.devices.empty()) cfg.devices.push_back(0);
  uint32_t nf = 0;
  AddrCallbacks cb;
  cb.on_found = [&](const AddrFound& f) {
    if (nf < cap) {
      if (keys_be) f.key.to_be(keys_be + 32 * (size_t)nf);
      if (compressed) compressed[nf] = f.compressed ? 1 : 0;
      if (rmd) memcpy(rmd + 20 * (size_t)nf, f.rmd.data(), 20);
    }
    ++nf;
  };
  AddrStats st;
  std::string e;
  const int rc = addr_search(a->T, a->G, cfg, cb, &st, &e);
  if (n_found) *n_found = nf;
  if (stats_out) {
    const uint64_t v[KHH_ADDR_STATS] = {
        st.chunks, st.keys, st.hits, st.degenerate, (uint64_t)(st.kernel_seconds * 1e6), st.launches,
        st.shader_mhz_n ? (uint64_t)(1e3 * st.shader_mhz_sum / st.shader_mhz_n) : 0, st.rescans};
    memcpy(stats_out, v, sizeof(uint64_t) * (stats_len < KHH_ADDR_STATS ? stats_len : KHH_ADDR_STATS));
  }
  if (rc) set_err(err, errlen, e);
  return rc;
}

int khh_addr_set_hit_capacity(khh_addr* a, uint32_t cap) {
  if (!a) return KHB_EINVAL;
  a->hit_cap = cap;
  return KHB_OK;
}

int khh_addr_confirm(const khh_addr* a, const uint8_t key_be[32], uint32_t kind, uint8_t out_key_be[32],
                     int* compressed) {
  if (!a || !key_be) return KHB_EINVAL;
  AddrFound f;
  if (!confirm_hit(a->T, U256::from_be(key_be), kind, &f)) return 0;
  if (out_key_be) f.key.to_be(out_key_be);
  if (compressed) *compressed = f.compressed ? 1 : 0;
  return 1;
}

void khh_hash160(const uint8_t xy[64], int compressed, uint8_t out[20]) {
  hash160_pub(pt_from_be(xy), compressed != 0, out);
}

void khh_rmd_to_address(const uint8_t rmd[20], char* out_addr) {
  const std::string s = rmd_to_address(rmd);
  memcpy(out_addr, s.c_str(), s.size() + 1);
}

}  // extern "C"
