// Host side of keyhunt's -m address / -m rmd160 modes (BTC P2PKH, with or without -e) on libkhbsgs:
// target loading (forceReadFileAddress, keyhunt.cpp:6300-6358), the generator table
// (init_generator, keyhunt.cpp:4386-4399), chunk claiming (thread_process, keyhunt.cpp:2546-2567),
// and the confirmation of GPU bloom hits (searchbinary + key recovery, keyhunt.cpp:2789-2937).
#pragma once
#include <stdint.h>

#include <array>
#include <functional>
#include <string>
#include <vector>

#include "bloom_host.hpp"
#include "secp_host.hpp"
#include "u256.hpp"

namespace khb {

using H160 = std::array<uint8_t, 20>;

// b58tobin into 25 bytes with keyhunt's acceptance rule (decoded size == 25, base58.c:39-112).
bool b58decode25(const char* s, uint8_t out[25]);
// rmd160toaddress_dst (keyhunt.cpp:2274-2284): base58check of 0x00 || rmd.
std::string rmd_to_address(const uint8_t rmd[20]);
void sha256(const uint8_t* msg, size_t len, uint8_t out[32]);
// GetHash160(P2PKH, compressed, P) (SECP256K1.cpp:671-705) / GetHash160_fromX (:707-789)
void hash160_pub(const Pt& p, bool compressed, uint8_t out[20]);
void hash160_x(uint8_t prefix, const Pt& p, uint8_t out[20]);

struct AddrTargets {
  std::vector<H160> table;             // sorted (memcmp), the reference's addressTable after _sort
  BloomFilter bloom;                   // initBloomFilter(counted lines)
  uint64_t counted = 0;                // lines longer than 20 characters (sizes the bloom)
  std::vector<std::string> skipped;    // "[I] Ommiting invalid line"

  // text: the target file's contents.  Returns false with *err on an unusable bloom.
  static bool load_text(const std::string& text, int bloom_multiplier, AddrTargets& out, std::string* err);
  static bool load_file(const char* path, int bloom_multiplier, AddrTargets& out, std::string* err);
  bool searchbinary(const uint8_t h[20]) const;   // keyhunt.cpp:2311-2335, literal
};

struct AddrGen {
  U256 stride{1};
  std::vector<Pt> gn;                  // Gn[0..511] = (i+1)*stride*G, gn[512] = _2Gn = 1024*stride*G
  std::vector<Pt> offs;                // offs[m] = m*gpl*_2Gn  (lane starts within a chunk)
  uint32_t gpl = 0;
  void build(const U256& stride, uint32_t groups_per_chunk, uint32_t gpl, int threads);
  std::vector<uint8_t> table_be() const;
  std::vector<uint8_t> offs_be() const;
};

struct AddrConfig {
  int search = 2;                      // 0 uncompress, 1 compress, 2 both (-l; keyhunt.cpp:59-61, 300)
  bool endomorphism = false;           // -e (keyhunt.cpp:579-585): beta*x, beta^2*x and negated points
  U256 start{1}, end{1};               // [start, end): n_range_start / n_range_end
  uint64_t n_seq = 1ull << 32;         // keys per claimed chunk (-n, N_SEQUENTIAL_MAX)
  bool random = false;                 // -R: each chunk starts at a random key in [start, end)
  std::vector<int> devices{0};
  uint32_t lanes = 0;                  // 0 = library default
  uint32_t gpl = 16;                   // groups per GPU lane
  uint64_t max_chunks = 0;             // 0 = until the range is exhausted
  uint32_t hit_cap = 0;                // tests: the launch's bloom-hit capacity (0 = library default)
};

struct AddrFound {
  U256 key;
  bool compressed;
  H160 rmd;
};

struct AddrStats {
  uint64_t launches = 0, chunks = 0, keys = 0, hits = 0, found = 0, degenerate = 0;
  uint64_t rescans = 0;            // launches whose bloom hits overflowed the ring (rescanned in parts)
  double kernel_seconds = 0;
  double shader_mhz_sum = 0;       // sum of the launches' average shader clocks (khb_stats.shader_mhz)
  uint64_t shader_mhz_n = 0;
};

struct AddrCallbacks {
  std::function<void(const AddrFound&)> on_found;             // called in range order per batch
  std::function<void(const U256& base, int device)> on_chunk;  // "Base key: ..." progress
  std::function<bool()> stop;                                  // polled between batches
  std::function<void(const std::string&)> on_warning;          // e.g. the depth-1 fallback
};

// Confirm one GPU bloom hit (khb_addr_hit.kind = form | e << 2) of the point whose key is `key`: searchbinary of the
// hash the kind names, then the reference's key recovery (keyhunt.cpp:2789-2937): lambda^e * key, negated when the
// hit is the other point of the pair.  False when the hash is not a target (a bloom false positive).
bool confirm_hit(const AddrTargets& T, const U256& key, uint32_t kind, AddrFound* out);
// lambda and lambda^2 mod n (keyhunt.cpp:582-583)
const U256& endo_lambda(int e);

// Sequential (or -R random) search over the range; returns 0 or a KHB_E* / -100 code with *err.
int addr_search(const AddrTargets& T, const AddrGen& G, const AddrConfig& cfg, const AddrCallbacks& cb,
                AddrStats* stats, std::string* err);

}  // namespace khb
