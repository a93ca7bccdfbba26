#include "engine.hpp"

#include <stdlib.h>
#include <string.h>
#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <deque>
#include <mutex>
#include <random>
#include <thread>

#include "../../../include/khbsgs.h"

namespace khb {

ChunkCursor::ChunkCursor(int mode, const U256& start, const U256& end, const U256& two_n, uint64_t seed)
    : mode_(mode), start_(start), end_(end), two_n_(two_n), cursor_(start), top_(end), rng_(seed) {}

// The next chunk from the top: keyhunt's `n_range_end -= 2N; base = max(n_range_end, lower)` while
// n_range_end > lower (keyhunt.cpp:5122-5133 backward with lower = the range start; 5383-5400 both and
// 4837-4854 dance with lower = BSGS_CURRENT).  Unsigned: a step to or below `lower` clamps to it and ends
// the side, as the reference's next `n_range_end > lower` test does.
bool ChunkCursor::top(const U256& lower, U256& base) {
  if (!(top_ > lower)) return false;
  if (top_ - lower <= two_n_) {
    base = lower;
    top_ = lower;
  } else {
    top_ = top_ - two_n_;
    base = top_;
  }
  return true;
}

// The next chunk from the bottom (keyhunt.cpp:3843-3844; 5401-5414 both and 4855-4868 dance, n_range_end
// moving).
bool ChunkCursor::bottom(const U256& upper, U256& base) {
  if (!(cursor_ < upper)) return false;
  base = cursor_;
  cursor_ = cursor_ + two_n_;
  return true;
}

bool ChunkCursor::next(U256& base) {
  switch (mode_) {
    case kChunkRandom: base = random_in(start_, end_); return true;        // keyhunt.cpp:4069
    case kChunkBackward: return top(start_, base);
    case kChunkBoth: return rng_() % 2 ? bottom(top_, base) : top(cursor_, base);
    case kChunkDance:
      switch (rng_() % 3) {
        case 0: return top(cursor_, base);
        case 1: return bottom(top_, base);
        default:                                   // base_key.Rand(&BSGS_CURRENT, &n_range_end), 4869-4870
          if (!(cursor_ < top_)) return false;
          base = random_in(cursor_, top_);
          return true;
      }
    default: return bottom(end_, base);            // sequential, keyhunt.cpp:3843-3844
  }
}

namespace {

template <class F>
void parallel_for(size_t n, int threads, F&& fn) {
  if (n == 0) return;
  if (threads <= 1 || n < 2) {
    for (size_t i = 0; i < n; ++i) fn(i);
    return;
  }
  std::atomic<size_t> next{0};
  auto body = [&]() {
    for (;;) {
      size_t i = next.fetch_add(1);
      if (i >= n) break;
      fn(i);
    }
  };
  std::vector<std::thread> th;
  const int nt = (int)std::min<size_t>((size_t)threads, n);
  for (int t = 1; t < nt; ++t) th.emplace_back(body);
  body();
  for (auto& t : th) t.join();
}

struct Shared {
  const Tables& T;
  const std::vector<Target>& targets;
  const SearchConfig& cfg;
  const SearchCallbacks& cb;
  U256 start, end;
  ChunkCursor chunks;       // the shared chunk cursor (keyhunt's BSGS_CURRENT / n_range_end)
  std::mutex mu;            // cursor, found, keys, stats, callbacks
  std::vector<int>& found;
  std::vector<U256>& keys;
  SearchStats& stats;
  std::vector<uint8_t> targets_xy;   // the targets x||y BE, for khb_check
  uint64_t claimed = 0;
  int n_found = 0;
  bool stop = false;
  int error = 0;
  std::string err;

  Shared(const Tables& t, const std::vector<Target>& tg, const SearchConfig& c, const SearchCallbacks& b,
         std::vector<int>& f, std::vector<U256>& k, SearchStats& s)
      : T(t), targets(tg), cfg(c), cb(b), found(f), keys(k), stats(s), targets_xy(64 * tg.size()) {
    for (size_t i = 0; i < tg.size(); ++i) pt_to_be(targets_xy.data() + 64 * i, tg[i].p);
  }
};

struct Batch {
  std::vector<U256> bases;        // chunk bases, in claim order
  std::vector<uint32_t> job_chunk, job_target;
  std::vector<uint8_t> centres;   // 64 B per job
  uint32_t group_begin = 0;       // groups [group_begin, group_begin + group_count) of every job;
  uint32_t group_count = 0;       // 0 = the whole chunk
  bool part = false;              // a rescan part of a batch whose candidate ring overflowed
};

// The two halves of a batch whose candidates overflowed the ring (the caller rescans):
// by jobs, or a single job by its group range, cut at a multiple of gpl (khb_submit's alignment).
// false: a single job of at most gpl groups (cannot be split further).
bool split_batch(const Batch& b, uint32_t cycles, uint32_t gpl, Batch& lo, Batch& hi) {
  const size_t nj = b.job_chunk.size();
  const uint32_t g0 = b.group_begin, gc = b.group_count ? b.group_count : cycles;
  auto part = [&](Batch& o, size_t j0, size_t j1, uint32_t pb, uint32_t pc) {
    o.bases = b.bases;
    o.job_chunk.assign(b.job_chunk.begin() + j0, b.job_chunk.begin() + j1);
    o.job_target.assign(b.job_target.begin() + j0, b.job_target.begin() + j1);
    o.centres.assign(b.centres.begin() + 64 * j0, b.centres.begin() + 64 * j1);
    o.group_begin = pb;
    o.group_count = pc;
    o.part = true;
  };
  if (nj > 1) {
    part(lo, 0, nj / 2, g0, gc);
    part(hi, nj / 2, nj, g0, gc);
    return true;
  }
  if (nj == 0 || gc <= gpl) return false;
  const uint32_t half = (gc / 2 + gpl - 1) / gpl * gpl;     // gpl <= half < gc
  part(lo, 0, 1, g0, half);
  part(hi, 0, 1, g0 + half, gc - half);
  return true;
}

// Device-busy time of one context's launches: the length of the union of their [begin, end) intervals
// (ms on the context's epoch).  Launches are collected in submission order and at most two overlap, so
// intervals are merged as they arrive and only the open one is kept (a long CLI run stays O(1)); an
// interval that starts before the open one (never seen) is merged into it.
struct BusyUnion {
  double total = 0, b = 0, e = -1;
  void add(double lo, double hi) {
    if (lo < 0 || hi < lo) return;                  // no timing for this launch
    if (lo > e) {
      if (e > b) total += e - b;
      b = lo;
      e = hi;
    } else {
      b = std::min(b, lo);
      e = std::max(e, hi);
    }
  }
  double ms() const { return total + (e > b ? e - b : 0); }
};

bool claim(Shared& S, uint32_t want, Batch& b) {
  std::lock_guard<std::mutex> lk(S.mu);
  b.bases.clear();
  for (uint32_t i = 0; i < want && !S.stop; ++i) {
    if (S.cfg.max_chunks && S.claimed >= S.cfg.max_chunks) break;
    U256 base;
    if (!S.chunks.next(base)) break;
    b.bases.push_back(base);
    S.claimed++;
    if (S.cb.on_chunk) S.cb.on_chunk(base);
  }
  return !b.bases.empty();
}

// Centres of every (chunk, live target) job: target + (order - base - intaux)*G
// (keyhunt.cpp:3861-3869).  Sequential chunks (bases 2N apart) take their auxiliary points from a
// batched walk (Tables::chunk_aux_run: one scalar multiplication per 64 chunks) instead of one
// scalar multiplication each, and the job additions share one inversion per block of 256 jobs
// across chunks: at small -n (few groups per chunk) the host would otherwise set the pace.
void make_jobs(Shared& S, Batch& b, int threads) {
  std::vector<int> live;
  {
    std::lock_guard<std::mutex> lk(S.mu);
    for (size_t k = 0; k < S.targets.size(); ++k)
      if (!S.found[k]) live.push_back((int)k);
  }
  const size_t nc = b.bases.size(), nt = live.size();
  b.job_chunk.resize(nc * nt);
  b.job_target.resize(nc * nt);
  b.centres.resize(64 * nc * nt);
  if (nc == 0 || nt == 0) return;
  std::vector<Pt> tp(nt);
  for (size_t j = 0; j < nt; ++j) tp[j] = S.targets[live[j]].p;
  for (size_t job = 0; job < nc * nt; ++job) {
    b.job_chunk[job] = (uint32_t)(job / nt);
    b.job_target[job] = (uint32_t)live[job % nt];
  }
  job_centres(S.T, b.bases, tp, b.centres.data(), threads);
}

}  // namespace

void job_centres(const Tables& T, const std::vector<U256>& bases, const std::vector<Pt>& tp, uint8_t* out,
                 int threads) {
  const size_t nc = bases.size(), nt = tp.size();
  if (nc == 0 || nt == 0) return;
  std::vector<Pt> aux(nc);
  bool up = nc > 1, down = nc > 1;
  for (size_t c = 1; c < nc && (up || down); ++c) {
    up = up && bases[c] == bases[c - 1] + T.geo.N_double;
    down = down && bases[c - 1] == bases[c] + T.geo.N_double;     // -B backward claims descend
  }
  if (up) {
    T.chunk_aux_run(bases[0], nc, aux.data(), threads);
  } else if (down) {
    T.chunk_aux_run(bases[nc - 1], nc, aux.data(), threads);
    std::reverse(aux.begin(), aux.end());
  } else
    parallel_for(nc, threads, [&](size_t c) { aux[c] = T.chunk_aux(bases[c]); });
  constexpr size_t kJobBlock = 256;
  const size_t nj = nc * nt;
  parallel_for((nj + kJobBlock - 1) / kJobBlock, threads, [&](size_t blk) {
    const size_t s0 = blk * kJobBlock, m = std::min(kJobBlock, nj - s0);
    std::vector<Pt> ta(m), xa(m), res(m);
    for (size_t i = 0; i < m; ++i) {
      ta[i] = tp[(s0 + i) % nt];
      xa[i] = aux[(s0 + i) / nt];
    }
    batch_add_pairs(ta.data(), xa.data(), m, res.data());
    for (size_t i = 0; i < m; ++i) pt_to_be(out + 64 * (s0 + i), res[i]);
  });
}

namespace {

// The device check of a batch's candidates (khb_check): ok / key per candidate, as Tables::secondcheck.
int confirm_device(Shared& S, khb_ctx* ctx, const Batch& b, const std::vector<khb_cand>& cands,
                   const std::vector<int>& found_snapshot, std::vector<int>& ok, std::vector<U256>& key) {
  std::vector<khb_check_in> in;
  std::vector<size_t> idx;
  in.reserve(cands.size());
  for (size_t i = 0; i < cands.size(); ++i) {
    const uint32_t job = cands[i].job;
    const uint32_t k = b.job_target[job];
    if (found_snapshot[k]) continue;
    khb_check_in c{};
    b.bases[b.job_chunk[job]].to_be(c.start_be);
    c.a = cands[i].a;
    c.target = k;
    in.push_back(c);
    idx.push_back(i);
  }
  if (in.empty()) return KHB_OK;
  std::vector<khb_check_out> out(in.size());
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = khb_check(ctx, S.targets_xy.data(), (uint32_t)S.targets.size(), in.data(), (uint32_t)in.size(),
                           out.data());
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (rc) return rc;
  for (size_t m = 0; m < in.size(); ++m) {
    ok[idx[m]] = out[m].found ? 1 : 0;
    if (out[m].found) key[idx[m]] = U256::from_be(out[m].key_be);
  }
  std::lock_guard<std::mutex> lk(S.mu);
  S.stats.device_checked += in.size();
  S.stats.device_check_seconds += dt;
  return KHB_OK;
}

// Confirm level-1 candidates (bsgs_secondcheck, keyhunt.cpp:3947-3982): speculative parallel
// checks (the CPU pool, or the device: SearchConfig::check_mode), then in-order resolution.
// A failed device check is confirmed on the host pool instead (the same keys); `device_off` then stays
// set for the calling device thread, which warns once and confirms every later batch on the host.
void confirm(Shared& S, khb_ctx* ctx, const Batch& b, std::vector<khb_cand>& cands, int threads, bool& device_off) {
  std::sort(cands.begin(), cands.end(), [](const khb_cand& x, const khb_cand& y) {
    return x.job != y.job ? x.job < y.job : x.a < y.a;
  });
  std::vector<int> ok(cands.size(), 0);
  std::vector<U256> key(cands.size());
  std::vector<int> found_snapshot;
  {
    std::lock_guard<std::mutex> lk(S.mu);
    found_snapshot = S.found;
  }
  bool dev = !device_off &&
             (S.cfg.check_mode == kCheckDevice || (S.cfg.check_mode == kCheckAuto && cands.size() > kCheckAutoMin));
  if (dev) {
    const int rc = confirm_device(S, ctx, b, cands, found_snapshot, ok, key);
    if (rc) {      // the host pool confirms this batch and every later one of this device (the same keys)
      device_off = true;
      std::lock_guard<std::mutex> lk(S.mu);
      if (S.cb.on_warning)
        S.cb.on_warning(std::string("[W] device check failed (") + khb_strerror(rc) +
                        "): candidates of this device are confirmed on the host from now on");
      std::fill(ok.begin(), ok.end(), 0);
      dev = false;
    }
  }
  if (!dev) {
    parallel_for(cands.size(), threads, [&](size_t i) {
      const uint32_t job = cands[i].job;
      const uint32_t k = b.job_target[job];
      if (found_snapshot[k]) return;
      ok[i] = S.T.secondcheck(b.bases[b.job_chunk[job]], cands[i].a, S.targets[k].p, key[i]) ? 1 : 0;
    });
  }
  std::lock_guard<std::mutex> lk(S.mu);
  for (size_t i = 0; i < cands.size(); ++i) {
    if (!ok[i]) continue;
    const uint32_t k = b.job_target[cands[i].job];
    if (S.found[k]) continue;
    S.found[k] = 1;
    S.keys[k] = key[i];
    S.n_found++;
    if (S.cb.on_found) S.cb.on_found((int)k, key[i]);
  }
  if (S.n_found == (int)S.targets.size()) S.stop = true;   // "All points were found"
}

uint32_t batch_chunks(const Tables& T, const SearchConfig& cfg, size_t ntargets, uint32_t ctx_lanes) {
  if (cfg.chunks_per_batch) return cfg.chunks_per_batch;
  const uint64_t per_item = khb_groups_per_item();
  const uint64_t lanes_per_job = (T.geo.cycles + per_item - 1) / per_item;
  const uint64_t lanes = ctx_lanes ? ctx_lanes : 256u * 16u * 64u;
  // ~8 work items per lane: the kernel's waves take items dynamically (KHB_DYN), so a deep queue
  // keeps the device full until the batch's last items
  const uint64_t jobs = (8ull * lanes + lanes_per_job - 1) / lanes_per_job;
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(jobs / std::max<size_t>(1, ntargets), 65536));
}

// One device: up to `queue_depth` batches queued on the GPU (khb_submit fills the context's next
// slot, each on its own stream, so a queued batch takes over the CUs the running one's last waves
// free); the next batch is claimed and centred while the GPU scans, and each collected batch is
// confirmed after its successor has been submitted.  A batch whose candidates overflowed the ring
// is rescanned in two parts (split_batch, recursively), queued ahead of new chunks.
void device_thread(Shared& S, khb_ctx* ctx) {
  auto fail = [&](int rc, const char* what) {
    std::lock_guard<std::mutex> lk(S.mu);
    if (!S.error) {
      S.error = rc;
      S.err = std::string("[E] ") + what + ": " + khb_strerror(rc);
    }
    S.stop = true;
  };
  auto warn = [&](const std::string& m) {
    std::lock_guard<std::mutex> lk(S.mu);
    if (S.cb.on_warning) S.cb.on_warning(m);
  };
  const Tables& T = S.T;
  const uint32_t cycles = (uint32_t)T.geo.cycles;
  const uint32_t want = batch_chunks(T, S.cfg, S.targets.size(), khb_lanes(ctx));
  const int threads = S.cfg.check_threads > 0 ? S.cfg.check_threads
                                               : (int)std::max(2u, std::min(16u, std::thread::hardware_concurrency()));
  int depth = std::max(1, std::min(S.cfg.queue_depth, 2));
  if (depth > 1) {
    // the second slot's scratch (~35 GB at the default lanes) up front; without it the device runs one
    // batch at a time
    const int rrc = khb_reserve_slots(ctx, depth);
    if (rrc == KHB_ENOMEM) {
      depth = 1;
      warn("[W] no device memory for a second submission slot: one batch in flight");
    } else if (rrc) {
      fail(rrc, "khb_reserve_slots");
      return;
    }
  }
  std::vector<khb_cand> cbuf(1u << 20);
  std::vector<khb_degenerate> dbuf(4096);
  const uint32_t cap = std::min<uint32_t>(khb_candidate_capacity(ctx), (uint32_t)cbuf.size());
  std::vector<Batch> ring(depth + 1);
  std::deque<Batch> parts;    // rescan parts of overflowed batches, submitted before new chunks
  BusyUnion busy;
  int next = 0;               // ring slots are used and released in FIFO order
  auto take = [&]() { const int i = next; next = (next + 1) % (int)ring.size(); return i; };
  auto stopped = [&]() { std::lock_guard<std::mutex> lk(S.mu); return S.stop; };
  auto prepare = [&](Batch& b) {
    if (stopped()) return false;
    if (!parts.empty()) {
      b = std::move(parts.front());
      parts.pop_front();
      return true;
    }
    if (!claim(S, want, b)) return false;
    b.group_begin = b.group_count = 0;
    b.part = false;
    make_jobs(S, b, threads);
    return !b.job_chunk.empty();
  };
  auto submit = [&](Batch& b) {
    return khb_submit(ctx, b.centres.data(), (uint32_t)b.job_chunk.size(), b.group_begin,
                      b.group_count ? b.group_count : cycles);
  };
  int rc = khb_reset_epoch(ctx);
  if (rc) { fail(rc, "khb_reset_epoch"); return; }
  std::deque<int> q;          // batches on the GPU, oldest first
  auto fill = [&]() {         // queue up to `depth` batches (start, and after a rescan drained the queue)
    while (!rc && (int)q.size() < depth) {
      if (!prepare(ring[next])) break;
      const int i = take();
      if ((rc = submit(ring[i]))) { fail(rc, "khb_submit"); break; }
      q.push_back(i);
    }
  };
  fill();
  int pre = -1;               // claimed and centred, not yet submitted
  std::vector<khb_cand> cands;
  bool device_check_off = false;       // a failed khb_check moves this device's confirmations to the host
  while (!q.empty()) {
    if (pre < 0 && !rc && prepare(ring[next])) pre = take();   // overlaps the GPU scan
    const int i = q.front();
    q.pop_front();
    khb_stats st{};
    const int crc = khb_collect(ctx, cbuf.data(), (uint32_t)cbuf.size(), dbuf.data(), (uint32_t)dbuf.size(), &st);
    if (crc) { fail(crc, "khb_collect"); rc = crc; continue; }  // keep draining the queue
    if (pre >= 0 && !rc) {
      if ((rc = submit(ring[pre]))) fail(rc, "khb_submit");
      else q.push_back(pre);
    }
    pre = -1;
    if (rc) continue;
    const Batch& b = ring[i];
    busy.add(st.launch_begin_ms, st.launch_end_ms);
    const bool overflow = st.n_cand > cap;
    if (overflow) {
      Batch lo, hi;
      if (!split_batch(b, cycles, T.gpl, lo, hi)) {
        fail(KHB_ENOMEM, "candidate ring overflow on a single work item");
        rc = KHB_ENOMEM;
        continue;
      }
      parts.push_front(std::move(hi));
      parts.push_front(std::move(lo));
    }
    {
      std::lock_guard<std::mutex> lk(S.mu);
      S.stats.launches += 1;
      S.stats.kernel_seconds += st.kernel_ms * 1e-3;
      if (st.event_ms > 0) S.stats.event_seconds += st.event_ms * 1e-3;
      if (st.shader_mhz > 0) {
        S.stats.shader_mhz_sum += st.shader_mhz;
        S.stats.shader_mhz_n += 1;
      }
      if (!b.part) S.stats.chunks += b.bases.size();
      if (overflow) {
        S.stats.rescans += 1;
      } else {
        S.stats.giant_steps += st.giant_steps;
        S.stats.candidates += st.n_cand;
        S.stats.degenerate += st.n_degenerate;
        for (uint32_t d = 0; d < st.n_degenerate && d < dbuf.size(); ++d) {
          if (!S.cb.on_warning) break;
          const uint32_t job = dbuf[d].job;
          S.cb.on_warning("[W] collapsed batch inverse (target on a window centre): chunk 0x" +
                          b.bases[b.job_chunk[job]].hex() + " group " + std::to_string(dbuf[d].group & 0x7fffffffu));
        }
        if (S.cfg.record_candidates && S.cb.on_candidate)
          for (uint32_t c = 0; c < st.n_cand; ++c)
            S.cb.on_candidate(b.bases[b.job_chunk[cbuf[c].job]], (int)b.job_target[cbuf[c].job], cbuf[c].a);
      }
    }
    if (!overflow) {
      cands.assign(cbuf.begin(), cbuf.begin() + st.n_cand);
      confirm(S, ctx, b, cands, threads, device_check_off);    // overlaps the GPU scan of the queue
    }
    if (q.empty()) fill();     // rescan parts left after the last batch
  }
  std::lock_guard<std::mutex> lk(S.mu);
  S.stats.busy_seconds += busy.ms() * 1e-3;
}

}  // namespace

int parse_check_mode(const char* s) {
  if (!strcmp(s, "host")) return kCheckHost;
  if (!strcmp(s, "gpu")) return kCheckDevice;
  if (!strcmp(s, "auto")) return kCheckAuto;
  return -1;
}

int load_check_tables(khb_ctx* c, const Tables& T) {
  const std::vector<uint8_t> l2 = T.bloom_concat(2), l3 = T.bloom_concat(3);
  const std::vector<uint8_t> a2 = T.amp_table_be(2), a3 = T.amp_table_be(3);
  khb_check_tables ct{};
  ct.gtable = gtable_be().data();
  ct.amp2 = a2.data();
  ct.amp3 = a3.data();
  ct.l2 = l2.data();
  ct.l2_bytes_per_sub = T.l2[0].bytes;
  ct.l2_bits_per_sub = T.l2[0].bits;
  ct.l2_hashes = T.l2[0].hashes;
  ct.l3 = l3.data();
  ct.l3_bytes_per_sub = T.l3[0].bytes;
  ct.l3_bits_per_sub = T.l3[0].bits;
  ct.l3_hashes = T.l3[0].hashes;
  ct.bptable = reinterpret_cast<const uint8_t*>(T.bp.data());
  ct.m3 = T.bp.size();
  T.geo.M_double.to_be(ct.m_double_be);
  T.geo.M2_double.to_be(ct.m2_double_be);
  T.geo.M3.to_be(ct.m3_be);
  T.geo.M3_double.to_be(ct.m3_double_be);
  return khb_load_check_tables(c, &ct);
}

int Session::open(const Tables& T, const SearchConfig& cfg, std::string& err) {
  close();
  T_ = &T;
  cfg_ = cfg;
  std::vector<uint8_t> bf = T.l1_concat();
  std::vector<uint8_t> gsn = T.giant_table_be();
  std::vector<uint8_t> offs = T.lane_offsets_be();
  for (int d : cfg.devices) {
    khb_ctx* c = nullptr;
    int rc = khb_open(d, cfg.lanes, &c);
    if (!rc) rc = khb_load_bloom(c, bf.data(), T.l1[0].bytes, T.l1[0].bits, T.l1[0].hashes);
    if (!rc && T.gate_log2 && cfg.use_gate) rc = khb_load_gate(c, T.gate.data(), T.gate_log2, T.gate_probes);
    if (!rc) rc = khb_load_giant_table(c, gsn.data());
    if (!rc) rc = khb_load_lane_offsets(c, offs.data(), (uint32_t)T.lane_offs.size(), T.gpl);
    if (!rc && cfg.cand_cap) rc = khb_set_candidate_capacity(c, cfg.cand_cap);
    if (!rc && cfg.check_mode != kCheckHost) rc = load_check_tables(c, T);
    if (rc) {
      err = "[E] GPU " + std::to_string(d) + ": " + khb_strerror(rc);
      if (c) khb_close(c);
      close();
      return rc;
    }
    ctx_.push_back(c);
  }
  return 0;
}

int Session::set_test_hooks(uint32_t cand_cap, bool use_gate, const uint8_t* l1_concat) {
  if (!T_) return KHB_ESTATE;
  for (void* c : ctx_) {
    khb_ctx* x = (khb_ctx*)c;
    int rc = khb_set_candidate_capacity(x, cand_cap ? cand_cap : (1u << 20));
    if (!rc && l1_concat) rc = khb_load_bloom(x, l1_concat, T_->l1[0].bytes, T_->l1[0].bits, T_->l1[0].hashes);
    if (!rc) rc = use_gate && T_->gate_log2 ? khb_load_gate(x, T_->gate.data(), T_->gate_log2, T_->gate_probes)
                                            : khb_load_gate(x, nullptr, 0, 0);
    if (rc) return rc;
  }
  cfg_.cand_cap = cand_cap;
  cfg_.use_gate = use_gate;
  return 0;
}

int Session::set_check_mode(int mode) {
  if (!T_) return KHB_ESTATE;
  if (mode < kCheckHost || mode > kCheckAuto) return KHB_EINVAL;
  if (mode != kCheckHost && cfg_.check_mode == kCheckHost)
    for (void* c : ctx_) {
      const int rc = load_check_tables((khb_ctx*)c, *T_);
      if (rc) return rc;
    }
  cfg_.check_mode = mode;
  return 0;
}

void Session::close() {
  for (void* c : ctx_) khb_close((khb_ctx*)c);
  ctx_.clear();
}

int Session::run(const std::vector<Target>& targets, const U256& start, const U256& end, const SearchCallbacks& cb,
                 std::vector<int>& found, std::vector<U256>& keys, SearchStats& stats, std::string& err,
                 uint64_t max_chunks, bool random_chunks) {
  found.assign(targets.size(), 0);
  keys.assign(targets.size(), U256());
  stats = SearchStats();
  if (targets.empty()) { err = "[E] no targets"; return KHB_EINVAL; }
  if (ctx_.empty() || !T_) { err = "[E] session not open"; return KHB_ESTATE; }
  SearchConfig cfg = cfg_;
  cfg.max_chunks = max_chunks;
  cfg.random_chunks = random_chunks;
  if (const char* q = getenv("KHB_QUEUE_DEPTH")) cfg.queue_depth = atoi(q);   // A/B timing of the tail overlap
  Shared S(*T_, targets, cfg, cb, found, keys, stats);
  S.start = start;
  S.end = end;
  uint64_t seed = 0;
  if (getrandom(&seed, sizeof seed, 0) != (ssize_t)sizeof seed) seed = (uint64_t)time(nullptr);
  S.chunks = ChunkCursor(cfg.random_chunks ? kChunkRandom : cfg.chunk_mode, start, end, T_->geo.N_double, seed);
  std::vector<std::thread> th;
  for (void* c : ctx_) th.emplace_back(device_thread, std::ref(S), (khb_ctx*)c);
  for (auto& t : th) t.join();
  if (S.error) err = S.err;
  return S.error;
}

int run_search(const Tables& T, const std::vector<Target>& targets, const U256& start, const U256& end,
               const SearchConfig& cfg, const SearchCallbacks& cb, std::vector<int>& found, std::vector<U256>& keys,
               SearchStats& stats, std::string& err) {
  Session s;
  int rc = s.open(T, cfg, err);
  if (rc) return rc;
  return s.run(targets, start, end, cb, found, keys, stats, err, cfg.max_chunks, cfg.random_chunks);
}

}  // namespace khb
