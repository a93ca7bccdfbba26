#include "address_host.hpp"

#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <deque>
#include <thread>

#include "../../../include/khbsgs.h"
#include "../device/hash160.hpp"

namespace khb {

// ------------------------------------------------------------------------------- hashing
void sha256(const uint8_t* msg, size_t len, uint8_t out[32]) {
  uint32_t s[8], w[16];
  sha256_init(s);
  uint8_t blk[128];
  size_t i = 0;
  auto load = [&](const uint8_t* b) {
    for (int k = 0; k < 16; ++k)
      w[k] = ((uint32_t)b[4 * k] << 24) | ((uint32_t)b[4 * k + 1] << 16) | ((uint32_t)b[4 * k + 2] << 8) | b[4 * k + 3];
  };
  for (; i + 64 <= len; i += 64) {
    load(msg + i);
    sha256_block(s, w);
  }
  const size_t rem = len - i;
  memset(blk, 0, sizeof blk);
  memcpy(blk, msg + i, rem);
  blk[rem] = 0x80;
  const size_t total = rem >= 56 ? 128 : 64;
  const uint64_t bits = (uint64_t)len * 8;
  for (int k = 0; k < 8; ++k) blk[total - 1 - k] = (uint8_t)(bits >> (8 * k));
  for (size_t o = 0; o < total; o += 64) {
    load(blk + o);
    sha256_block(s, w);
  }
  for (int k = 0; k < 8; ++k) {
    out[4 * k] = (uint8_t)(s[k] >> 24); out[4 * k + 1] = (uint8_t)(s[k] >> 16);
    out[4 * k + 2] = (uint8_t)(s[k] >> 8); out[4 * k + 3] = (uint8_t)s[k];
  }
}

static void fe_of_pt(Fe& x, Fe& y, const Pt& p) {
  uint8_t b[64];
  pt_to_be(b, p);
  fe_from_be(x, b);
  fe_from_be(y, b + 32);
}

static void bytes_of_words(uint8_t out[20], const uint32_t h[5]) {
  for (int k = 0; k < 5; ++k)
    for (int b = 0; b < 4; ++b) out[4 * k + b] = (uint8_t)(h[k] >> (8 * b));
}

void hash160_pub(const Pt& p, bool compressed, uint8_t out[20]) {
  Fe x, y;
  fe_of_pt(x, y, p);
  uint32_t h[5];
  if (compressed)
    hash160_compressed(h, (y.v[0] & 1) ? 3u : 2u, x);
  else
    hash160_uncompressed(h, x, y);
  bytes_of_words(out, h);
}

void hash160_x(uint8_t prefix, const Pt& p, uint8_t out[20]) {
  Fe x, y;
  fe_of_pt(x, y, p);
  uint32_t h[5];
  hash160_compressed(h, prefix, x);
  bytes_of_words(out, h);
}

// -------------------------------------------------------------------------------- base58
static const char kB58[] = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";

static int b58_digit(unsigned char c) {
  if (!c || (c & 0x80)) return -1;
  const char* p = strchr(kB58, c);
  return p ? (int)(p - kB58) : -1;
}

bool b58decode25(const char* s, uint8_t out[25]) {
  const size_t n = strlen(s);
  size_t i = 0, zeros = 0;
  memset(out, 0, 25);
  for (; i < n && s[i] == '1'; ++i) ++zeros;
  for (; i < n; ++i) {
    const int v = b58_digit((unsigned char)s[i]);
    if (v < 0) return false;
    uint32_t carry = (uint32_t)v;
    for (int k = 24; k >= 0; --k) {
      const uint32_t t = (uint32_t)out[k] * 58u + carry;
      out[k] = (uint8_t)t;
      carry = t >> 8;
    }
    if (carry) return false;   // "Output number too big"
  }
  size_t lz = 0;
  while (lz < 25 && out[lz] == 0) ++lz;
  return 25 - lz + zeros == 25;  // keyhunt.cpp:6338: raw_value_length == 25
}

std::string rmd_to_address(const uint8_t rmd[20]) {
  uint8_t d[25], h1[32], h2[32];
  d[0] = 0x00;   // byte_encode_crypto (P2PKH)
  memcpy(d + 1, rmd, 20);
  sha256(d, 21, h1);
  sha256(h1, 32, h2);
  memcpy(d + 21, h2, 4);
  size_t zc = 0;
  while (zc < 25 && !d[zc]) ++zc;
  const size_t size = (25 - zc) * 138 / 100 + 1;   // b58enc (base58.c:145-189)
  std::vector<uint8_t> buf(size, 0);
  size_t high = size - 1, j = 0;
  for (size_t i = zc; i < 25; ++i, high = j) {
    int carry = d[i];
    for (j = size - 1; (j > high) || carry; --j) {
      carry += 256 * buf[j];
      buf[j] = (uint8_t)(carry % 58);
      carry /= 58;
      if (!j) break;
    }
  }
  for (j = 0; j < size && !buf[j]; ++j) {}
  std::string out(zc, '1');
  for (; j < size; ++j) out += kB58[buf[j]];
  return out;
}

// ------------------------------------------------------------------------------- targets
static void trim(char* s) {
  const char* seps = " \t\n\r";
  size_t n = strlen(s);
  while (n && strchr(seps, s[n - 1])) s[--n] = 0;
  const size_t k = strspn(s, seps);
  if (k) memmove(s, s + k, n + 1 - k);
}

static bool all_b58(const char* s) {
  for (; *s; ++s)
    if (b58_digit((unsigned char)*s) < 0) return false;
  return true;
}

static bool all_hex(const char* s) {
  for (; *s; ++s) {
    const char c = *s;
    if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'))) return false;
  }
  return true;
}

static int hexv(char c) { return c <= '9' ? c - '0' : (c | 32) - 'a' + 10; }

// Split like fgets(aux, 100, f): a line longer than 99 characters continues in the next read.
static std::vector<std::string> fgets_lines(const std::string& text) {
  std::vector<std::string> out;
  size_t p = 0;
  while (p < text.size()) {
    size_t e = text.find('\n', p);
    size_t len = (e == std::string::npos ? text.size() : e + 1) - p;
    if (len > 99) len = 99;
    out.push_back(text.substr(p, len));
    p += len;
  }
  return out;
}

bool AddrTargets::load_text(const std::string& text, int bloom_multiplier, AddrTargets& T, std::string* err) {
  T = AddrTargets();
  const std::vector<std::string> lines = fgets_lines(text);
  char aux[128];
  for (const std::string& l : lines) {
    snprintf(aux, sizeof aux, "%s", l.c_str());
    trim(aux);
    if (strlen(aux) > 20) ++T.counted;
  }
  // initBloomFilter (keyhunt.cpp:6559-6576)
  const uint64_t entries = T.counted <= 10000 ? 10000 : (uint64_t)(bloom_multiplier > 0 ? bloom_multiplier : 1) * T.counted;
  if (T.bloom.init2(entries, 0.000001L) != 0) {
    if (err) *err = "bloom_init failed";
    return false;
  }
  uint64_t items = T.counted, i = 0;
  size_t li = 0;
  while (i < items && li < lines.size()) {
    snprintf(aux, sizeof aux, "%s", lines[li++].c_str());
    trim(aux);
    const size_t r = strlen(aux);
    bool valid = false;
    if (r > 0 && r <= 40) {
      if (r < 40 && all_b58(aux)) {
        uint8_t raw[25];
        if (b58decode25(aux, raw)) {
          H160 h;
          memcpy(h.data(), raw + 1, 20);
          T.bloom.add20(h.data());
          T.table.push_back(h);
          ++i;
          valid = true;
        }
      }
      if (r == 40 && all_hex(aux)) {
        H160 h;
        for (int k = 0; k < 20; ++k) h[k] = (uint8_t)(hexv(aux[2 * k]) * 16 + hexv(aux[2 * k + 1]));
        T.bloom.add20(h.data());
        T.table.push_back(h);
        ++i;
        valid = true;
      }
    }
    if (!valid) {
      T.skipped.push_back(aux);
      --items;
    }
  }
  std::sort(T.table.begin(), T.table.end(),
            [](const H160& a, const H160& b) { return memcmp(a.data(), b.data(), 20) < 0; });
  return true;
}

bool AddrTargets::load_file(const char* path, int bloom_multiplier, AddrTargets& T, std::string* err) {
  FILE* f = fopen(path, "r");
  if (!f) {
    if (err) *err = std::string("Error opening the file ") + path;
    return false;
  }
  std::string text;
  char buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) text.append(buf, n);
  fclose(f);
  return load_text(text, bloom_multiplier, T, err);
}

bool AddrTargets::searchbinary(const uint8_t data[20]) const {
  int64_t half, min = 0, max = (int64_t)table.size(), current = 0;
  bool r = false;
  half = max;
  while (!r && half >= 1) {
    half = (max - min) / 2;
    const int rcmp = memcmp(data, table[(size_t)(current + half)].data(), 20);
    if (rcmp == 0) {
      r = true;
    } else {
      if (rcmp < 0) max = max - half;
      else min = min + half;
      current = min;
    }
  }
  return r;
}

// ----------------------------------------------------------------------------- generator
void AddrGen::build(const U256& s, uint32_t groups_per_chunk, uint32_t g_per_lane, int threads) {
  stride = s;
  gpl = g_per_lane;
  gn.assign(513, Pt());
  const Pt G = mul_g(stride);
  gn[0] = G;
  gn[1] = double_direct(G);
  for (int i = 2; i < 512; ++i) gn[i] = add_direct(gn[i - 1], G);
  gn[512] = double_direct(gn[511]);
  const uint32_t n_off = (groups_per_chunk + gpl - 1) / gpl;
  offs.assign(n_off ? n_off : 1, Pt());
  std::atomic<uint32_t> next{1};
  auto work = [&] {
    for (;;) {
      const uint32_t m = next.fetch_add(1);
      if (m >= n_off) break;
      U256 k = stride * ((uint64_t)m * gpl * 1024u), r;
      U256::divmod(k, secp_order(), nullptr, &r);
      offs[m] = r.is_zero() ? Pt() : mul_g(r);
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < threads; ++t) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
}

std::vector<uint8_t> AddrGen::table_be() const {
  std::vector<uint8_t> out(64 * gn.size());
  for (size_t i = 0; i < gn.size(); ++i) pt_to_be(out.data() + 64 * i, gn[i]);
  return out;
}

std::vector<uint8_t> AddrGen::offs_be() const {
  std::vector<uint8_t> out(64 * offs.size());
  for (size_t i = 0; i < offs.size(); ++i) pt_to_be(out.data() + 64 * i, offs[i]);
  return out;
}

// -------------------------------------------------------------------------------- search
const U256& endo_lambda(int e) {
  static const U256 L[2] = {[] { U256 v; U256::from_hex("5363ad4cc05c30e0a5261c028812645a122e22ea20816678df02967c1b23bd72", v); return v; }(),
                            [] { U256 v; U256::from_hex("ac9c52b33fa3cf1f5ad9e3fd77ed9ba4a880b9fc8ec739c2e0cfc810b51283ce", v); return v; }()};
  return L[e - 1];
}

// The hash is recomputed from the key (independently of the GPU's): P = (lambda^e * k)*G has x = beta^e * x(k*G)
// and the same y.  Compressed forms 0/1: the x-only hit belongs to k' or to n - k' (keyhunt.cpp:2811-2822; with -e
// the reference decides by the parity of y, 2800-2860, which gives the same key).  Uncompressed form 2 is k' itself,
// form 3 (-e only) the negated point, n - k' (keyhunt.cpp:2876-2920).
bool confirm_hit(const AddrTargets& T, const U256& key, uint32_t kind, AddrFound* out) {
  const uint32_t form = kind & 3u, e = kind >> 2;
  if (e > 2) return false;
  U256 k;
  U256::divmod(key, secp_order(), nullptr, &k);
  if (e) k = mulmod(k, endo_lambda((int)e), secp_order());
  if (k.is_zero()) return false;
  const Pt P = mul_g(k);
  uint8_t h[20];
  if (form < 2) {
    hash160_x((uint8_t)(2 + form), P, h);
    if (!T.searchbinary(h)) return false;
    uint8_t hc[20];
    hash160_pub(P, true, hc);
    out->key = memcmp(h, hc, 20) != 0 ? secp_order() - k : k;
    out->compressed = true;
  } else {
    hash160_pub(form == 2 ? P : negation(P), false, h);
    if (!T.searchbinary(h)) return false;
    out->key = form == 2 ? k : secp_order() - k;
    out->compressed = false;
  }
  // without -e the reported key is the scanned key itself (key, not key mod n), as the reference's keyfound
  if (!e && form == 2) out->key = key;
  else if (!e && form < 2 && out->key == k) out->key = key;
  memcpy(out->rmd.data(), h, 20);
  return true;
}

namespace {

struct AddrShared {
  const AddrTargets& T;
  const AddrGen& G;
  const AddrConfig& cfg;
  const AddrCallbacks& cb;
  U256 cursor;
  uint64_t claimed = 0;
  std::mutex mu;
  AddrStats& stats;
  std::string err;
  int rc = 0;
};


void device_loop(AddrShared& S, int device) {
  khb_ctx* ctx = nullptr;
  int rc = khb_open(device, S.cfg.lanes, &ctx);
  auto fail = [&](int code, const char* what) {
    std::lock_guard<std::mutex> lk(S.mu);
    if (!S.rc) {
      S.rc = code;
      S.err = std::string(what) + ": " + khb_strerror(code);
    }
  };
  if (rc) return fail(rc, "khb_open");
  const uint32_t groups = (uint32_t)(S.cfg.n_seq / 1024);
  const std::vector<uint8_t> gtab = S.G.table_be(), offs = S.G.offs_be();
  const BloomGeom bg = S.T.bloom.geom();
  if ((S.cfg.hit_cap && (rc = khb_set_candidate_capacity(ctx, S.cfg.hit_cap))) ||
      (rc = khb_load_giant_table(ctx, gtab.data())) ||
      (rc = khb_load_lane_offsets(ctx, offs.data(), (uint32_t)S.G.offs.size(), S.G.gpl)) ||
      (rc = khb_load_addr_bloom(ctx, S.T.bloom.bf.data(), bg.bytes_per_sub, bg.bits, bg.hashes))) {
    khb_close(ctx);
    return fail(rc, "table upload");
  }
  const uint64_t lanes_per_job = (groups + S.G.gpl - 1) / S.G.gpl;
  const uint64_t lanes = khb_lanes(ctx);
  // about eight work items per lane (the kernel's waves take items dynamically, so a deep launch
  // keeps every SIMD full until its last items), and two launches queued (the context's two
  // submission slots): the next launch fills the CUs the current one's tail leaves idle
  uint64_t per_batch = (8 * lanes + lanes_per_job - 1) / lanes_per_job;
  if (per_batch < 1) per_batch = 1;
  if (per_batch > 4096) per_batch = 4096;
  struct ABatch {
    std::vector<U256> bases;
    std::vector<uint8_t> centres;
    uint32_t group_begin = 0, group_count = 0;   // group range of every chunk (0 = the whole chunk)
    bool part = false;                           // a rescan part of a batch whose hits overflowed
  };
  ABatch ring[3];
  int next = 0;
  auto take = [&]() { const int i = next; next = (next + 1) % 3; return i; };
  const U256 half = S.G.stride * 512u;
  // A batch whose bloom hits overflowed the ring is rescanned in two parts (by chunks, or one chunk by
  // a gpl-aligned group range), queued ahead of new chunks: every hit reaches confirm_hit, as every
  // hit reaches searchbinary in the reference (keyhunt.cpp:2716-2937).
  std::deque<ABatch> parts;
  auto split = [&](const ABatch& b, ABatch& lo, ABatch& hi) {
    const size_t n = b.bases.size();
    const uint32_t g0 = b.group_begin, gc = b.group_count ? b.group_count : groups;
    auto part = [&](ABatch& o, size_t j0, size_t j1, uint32_t pb, uint32_t pc) {
      o.bases.assign(b.bases.begin() + j0, b.bases.begin() + j1);
      o.centres.assign(b.centres.begin() + 64 * j0, b.centres.begin() + 64 * j1);
      o.group_begin = pb;
      o.group_count = pc;
      o.part = true;
    };
    if (n > 1) {
      part(lo, 0, n / 2, g0, gc);
      part(hi, n / 2, n, g0, gc);
      return true;
    }
    if (n == 0 || gc <= S.G.gpl) return false;
    const uint32_t h = (gc / 2 + S.G.gpl - 1) / S.G.gpl * S.G.gpl;
    part(lo, 0, 1, g0, h);
    part(hi, 0, 1, g0 + h, gc - h);
    return true;
  };
  auto prepare = [&](ABatch& b) {
    b.bases.clear();
    if (S.cb.stop && S.cb.stop()) return false;
    if (!parts.empty()) {
      b = std::move(parts.front());
      parts.pop_front();
      return true;
    }
    b.group_begin = b.group_count = 0;
    b.part = false;
    {
      std::lock_guard<std::mutex> lk(S.mu);
      if (S.rc) return false;
      while (b.bases.size() < per_batch) {
        if (S.cfg.max_chunks && S.claimed >= S.cfg.max_chunks) break;
        if (S.cfg.random) {
          b.bases.push_back(random_in(S.cfg.start, S.cfg.end));
        } else {
          if (!(S.cursor < S.cfg.end)) break;
          b.bases.push_back(S.cursor);
          S.cursor = S.cursor + U256(S.cfg.n_seq);
        }
        ++S.claimed;
      }
    }
    if (b.bases.empty()) return false;
    if (S.cb.on_chunk)
      for (const U256& c : b.bases) S.cb.on_chunk(c, device);
    b.centres.resize(64 * b.bases.size());
    for (size_t k = 0; k < b.bases.size(); ++k) {
      U256 c = b.bases[k] + half, r;   // startP = ComputePublicKey(key_mpz + 512*stride)
      U256::divmod(c, secp_order(), nullptr, &r);
      pt_to_be(b.centres.data() + 64 * k, mul_g(r));
    }
    return true;
  };
  auto submit = [&](ABatch& b) {
    return khb_addr_submit(ctx, b.centres.data(), (uint32_t)b.bases.size(), b.group_begin,
                           b.group_count ? b.group_count : groups,
                           S.cfg.search | (S.cfg.endomorphism ? KHB_SEARCH_ENDOMORPHISM : 0));
  };
  // both submission slots up front; on KHB_ENOMEM (large targets or many devices' worth of scratch)
  // one launch at a time instead of failing (advisor r2)
  size_t depth = 2;
  if ((rc = khb_reserve_slots(ctx, 2)) == KHB_ENOMEM) {
    depth = 1;
    rc = 0;
    std::lock_guard<std::mutex> lk(S.mu);
    if (S.cb.on_warning) S.cb.on_warning("[W] no device memory for a second submission slot: one batch in flight");
  } else if (rc) {
    khb_close(ctx);
    return fail(rc, "khb_reserve_slots");
  }
  std::vector<khb_addr_hit> hits(1u << 18);
  std::deque<int> q;
  while (q.size() < depth) {
    const int i = take();
    if (!prepare(ring[i])) break;
    if ((rc = submit(ring[i]))) { fail(rc, "khb_addr_submit"); break; }
    q.push_back(i);
  }
  const uint32_t acap = std::min<uint32_t>(khb_addr_hit_capacity(ctx), (uint32_t)(1u << 18));
  int pre = -1;
  while (!q.empty()) {
    if (pre < 0 && !rc && prepare(ring[next])) pre = take();   // overlaps the GPU scan
    const int i = q.front();
    q.pop_front();
    khb_stats st{};
    const int crc = khb_addr_collect(ctx, hits.data(), (uint32_t)hits.size(), &st);
    if (crc) { fail(crc, "khb_addr_collect"); rc = crc; continue; }   // keep draining the queue
    // after a stop (every target found, or the caller's stop) the prepared batch is dropped instead of
    // queued, so the exit waits for at most the one launch still in flight (advisor r2)
    if (pre >= 0 && !rc && !(S.cb.stop && S.cb.stop())) {
      if ((rc = submit(ring[pre]))) fail(rc, "khb_addr_submit");
      else q.push_back(pre);
    }
    pre = -1;
    if (rc) continue;
    const ABatch& b = ring[i];
    if (st.n_cand > acap) {              // the ring kept only acap hits: rescan the batch in parts
      ABatch lo, hi;
      if (!split(b, lo, hi)) {
        fail(-100, "bloom hit ring overflow on a single work item (target bloom too full)");
        rc = -100;
        continue;
      }
      parts.push_front(std::move(hi));
      parts.push_front(std::move(lo));
      {
        std::lock_guard<std::mutex> lk(S.mu);
        S.stats.launches++;
        S.stats.rescans++;
        S.stats.kernel_seconds += st.kernel_ms * 1e-3;
        if (!b.part) S.stats.chunks += b.bases.size();
      }
      if (q.empty() && pre < 0 && prepare(ring[next])) {    // keep the device busy with the parts
        const int k = take();
        if ((rc = submit(ring[k]))) fail(rc, "khb_addr_submit");
        else q.push_back(k);
      }
      continue;
    }
    const uint32_t nh = st.n_cand;
    std::sort(hits.begin(), hits.begin() + nh, [](const khb_addr_hit& x, const khb_addr_hit& y) {
      if (x.job != y.job) return x.job < y.job;
      if (x.group != y.group) return x.group < y.group;
      if (x.t != y.t) return x.t < y.t;
      return x.kind < y.kind;
    });
    std::vector<AddrFound> found;
    for (uint32_t h = 0; h < nh; ++h) {
      const khb_addr_hit& ht = hits[h];
      const U256 key = b.bases[ht.job] + S.G.stride * ((uint64_t)ht.group * 1024u + ht.t);
      AddrFound f;
      if (confirm_hit(S.T, key, ht.kind, &f)) found.push_back(f);
    }
    std::lock_guard<std::mutex> lk(S.mu);
    S.stats.launches++;
    if (!b.part) S.stats.chunks += b.bases.size();
    S.stats.keys += st.giant_steps;
    S.stats.hits += st.n_cand;
    S.stats.degenerate += st.n_degenerate;
    S.stats.kernel_seconds += st.kernel_ms * 1e-3;
    if (st.shader_mhz > 0) {
      S.stats.shader_mhz_sum += st.shader_mhz;
      S.stats.shader_mhz_n++;
    }
    S.stats.found += found.size();
    if (S.cb.on_found)
      for (const AddrFound& f : found) S.cb.on_found(f);
  }
  khb_close(ctx);
}

}  // namespace

int addr_search(const AddrTargets& T, const AddrGen& G, const AddrConfig& cfg, const AddrCallbacks& cb,
                AddrStats* stats, std::string* err) {
  AddrStats local;
  AddrStats& st = stats ? *stats : local;
  st = AddrStats();
  if (cfg.n_seq < 1024 || cfg.n_seq % 1024 || cfg.n_seq / 1024 > 0xFFFFFFFFull) {
    if (err) *err = "n must be a positive multiple of 1024";
    return -100;
  }
  if ((cfg.n_seq / 1024 + G.gpl - 1) / G.gpl > G.offs.size()) {
    if (err) *err = "generator lane offsets do not cover a chunk";
    return -100;
  }
  AddrShared S{T, G, cfg, cb, cfg.start, 0, {}, st, {}, 0};
  std::vector<std::thread> th;
  for (int d : cfg.devices) th.emplace_back(device_loop, std::ref(S), d);
  for (auto& t : th) t.join();
  if (S.rc && err) *err = S.err;
  return S.rc;
}

}  // namespace khb
