// Search driver: the role of keyhunt.cpp's thread_process_bsgs workers (3778-4009) and the chunk
// scheduler (BSGS_CURRENT += 2N under a mutex, 3824-3844), re-shaped for GPUs:
//   - one host thread per device owns a libkhbsgs context;
//   - a thread claims a batch of consecutive chunks, computes every (chunk, target) centre with a
//     batched AddDirect, submits the batch, and while the GPU scans it confirms the previous
//     batch's level-1 candidates on a CPU pool (bsgs_secondcheck/thirdcheck);
//   - confirmations run speculatively in parallel and are resolved in (chunk, target, a) order, so
//     the found keys are those a sequential `-t 1` reference run reports.
#pragma once
#include <stdint.h>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include "bsgs_host.hpp"

struct khb_ctx;

namespace khb {

struct Target {
  Pt p;
  bool compressed = true;
};

// Centres of the jobs (chunk c, target j) -> out[64 * (c * nt + j)], x||y big-endian:
// tp[j] + (order - bases[c] - intaux) G (keyhunt.cpp:3861-3869), batched (engine.cpp).
void job_centres(const Tables& T, const std::vector<U256>& bases, const std::vector<Pt>& tp, uint8_t* out,
                 int threads);

struct SearchConfig {
  std::vector<int> devices{0};
  uint32_t lanes = 0;              // per device, 0 = library default
  uint32_t chunks_per_batch = 0;   // 0 = auto (fill the device)
  int check_threads = 0;           // CPU confirmation pool, 0 = auto
  uint64_t max_chunks = 0;         // 0 = until range end
  bool random_chunks = false;      // -B random: every chunk base drawn uniformly in the range
  // keyhunt's -B mode (keyhunt.cpp:227 bsgs_modes, the thread_process_bsgs* variants 3778-5700): how chunk
  // bases are claimed.  kChunkRandom is also selected by random_chunks.
  int chunk_mode = 0;
  bool use_gate = true;            // load the tables' level-0 gate (khb_load_gate) when they have one
  int queue_depth = 2;             // batches queued per device (1 or 2; 2 overlaps launch tails)
  uint32_t cand_cap = 0;           // candidate ring entries per launch (0 = library default, 2^20); tests
                                   // lower it to drive the overflow path (split + rescan)
  bool record_candidates = false;  // tests: report every level-1 candidate (SearchCallbacks::on_candidate)
  // Where the level-1 candidates are confirmed (bsgs_secondcheck/thirdcheck, keyhunt.cpp:4271-4368):
  // kCheckHost on the CPU pool, kCheckDevice on the GPU that scanned them (khb_check), kCheckAuto on
  // the GPU when a batch holds more than kCheckAutoMin candidates (the gated scan's ~30/s stay on the
  // host, whose pool answers in microseconds; an ungated or dense-bloom scan moves to the device).
  int check_mode = 0;
};
enum : int { kCheckHost = 0, kCheckDevice = 1, kCheckAuto = 2 };
// -B modes in keyhunt's order: sequential (thread_process_bsgs, 3824-3844: a cursor from the range start up
// by 2N), backward (5072-5325: from the range end down by 2N, the last chunk clamped to the start), both
// (5329-5700: each claim from the top or the bottom at random until they meet), random (4014-4264: a
// uniform base in the range), dance (4794-5068: top, bottom or a uniform base between them, at random).
enum : int { kChunkSequential = 0, kChunkBackward = 1, kChunkBoth = 2, kChunkRandom = 3, kChunkDance = 4 };
constexpr uint32_t kCheckAutoMin = 4096;
// The --check argument of keyhunt_amd / bsgsd_amd: "host", "gpu" or "auto"; -1 for anything else.
int parse_check_mode(const char* s);

// The chunk bases of one search in claim order (keyhunt's BSGS_CURRENT / n_range_end under bsgs_thread),
// for a -B mode (kChunk*); the seed drives the both / dance side choices.  Shared by every device thread
// under the engine's lock.
class ChunkCursor {
 public:
  ChunkCursor() = default;
  ChunkCursor(int mode, const U256& start, const U256& end, const U256& two_n, uint64_t seed);
  bool next(U256& base);     // false when the mode's range is exhausted (random: never)

 private:
  bool top(const U256& lower, U256& base);
  bool bottom(const U256& upper, U256& base);
  int mode_ = kChunkSequential;
  U256 start_, end_, two_n_, cursor_, top_;
  std::mt19937_64 rng_;
};

struct SearchStats {
  uint64_t launches = 0;           // GPU scan launches (one per batch per device)
  uint64_t chunks = 0;
  uint64_t giant_steps = 0;
  uint64_t candidates = 0;
  uint64_t degenerate = 0;
  uint64_t rescans = 0;            // launches whose candidate ring overflowed and were rescanned in parts
  double kernel_seconds = 0;       // summed over launches and devices (per-launch event time)
  double busy_seconds = 0;         // union of each device's launch intervals, summed over devices: the
                                   // device-busy time (two launches in flight overlap, so < kernel_seconds)
  double shader_mhz_sum = 0;       // sum of the launches' average shader clocks (khb_stats.shader_mhz)
  uint64_t shader_mhz_n = 0;
  uint64_t device_checked = 0;     // candidates confirmed on the GPU (khb_check)
  double device_check_seconds = 0; // wall time of those khb_check calls
  double event_seconds = 0;        // summed HIP-event times of the launches (khb_stats.event_ms: dispatch
                                   // to end, what rocprofv3's kernel trace reports per launch)
};

struct SearchCallbacks {
  // key found for target k (called in order, under the engine's report lock)
  std::function<void(int k, const U256& key)> on_found;
  // progress: base of the chunk a device just claimed (for `-q`-less "Thread 0x..." lines)
  std::function<void(const U256& base)> on_chunk;
  std::function<void(const std::string& msg)> on_warning;
  // every level-1 candidate (chunk base, target, giant step a) of a complete launch, before its check
  // (only with SearchConfig::record_candidates)
  std::function<void(const U256& base, int k, uint32_t a)> on_candidate;
};

// A set of opened devices with the tables resident in HBM (libkhbsgs contexts), reusable across
// searches.  The CLI opens one; bench.py times run() on an open session.
class Session {
 public:
  Session() = default;
  ~Session() { close(); }
  Session(const Session&) = delete;
  Session& operator=(const Session&) = delete;
  int open(const Tables& T, const SearchConfig& cfg, std::string& err);
  int run(const std::vector<Target>& targets, const U256& start, const U256& end, const SearchCallbacks& cb,
          std::vector<int>& found, std::vector<U256>& keys, SearchStats& stats, std::string& err,
          uint64_t max_chunks = 0, bool random_chunks = false);
  void close();
  const SearchConfig& config() const { return cfg_; }
  SearchConfig& config() { return cfg_; }
  // tests: candidate ring capacity per launch (0 = default), the level-0 gate on/off, and optionally
  // a replacement level-1 bloom of the same geometry (256 sub-blooms concatenated; null = the tables')
  int set_test_hooks(uint32_t cand_cap, bool use_gate, const uint8_t* l1_concat = nullptr);
  // SearchConfig::check_mode for later runs; loads the device check tables when a device mode needs them.
  int set_check_mode(int mode);

 private:
  const Tables* T_ = nullptr;
  SearchConfig cfg_;
  std::vector<void*> ctx_;   // khb_ctx*
};

// The check tables of T (level-2/3 blooms, bPtable, AMP2/AMP3, GTable, M constants) into a context.
int load_check_tables(khb_ctx* c, const Tables& T);

// Runs the search over [start, end) on a temporary session.  Returns 0, or a negative khbsgs error code.  found/keys are
// sized to targets.size().  stats is updated live (read it from another thread for the
// periodic "Total ... keys" line).
int run_search(const Tables& T, const std::vector<Target>& targets, const U256& start, const U256& end,
               const SearchConfig& cfg, const SearchCallbacks& cb, std::vector<int>& found, std::vector<U256>& keys,
               SearchStats& stats, std::string& err);

}  // namespace khb
