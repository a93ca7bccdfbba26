// BSGS host engine: everything of keyhunt's `-m bsgs` except the giant-step scan itself, which
// runs on the GPU through libkhbsgs (include/khbsgs.h).
//
//   geometry      keyhunt.cpp:1045-1213   (N, M = sqrt(N)*k, M2, M3, aux, bloom entry counts)
//   giant tables  keyhunt.cpp:1309-1364   (GSn, _2GSn, AMP2, AMP3)
//   baby tables   keyhunt.cpp:1615-1880 + thread_bPload 4404-4592 (3-level blooms, bPtable)
//   chunk centre  keyhunt.cpp:3861-3869
//   confirmation  bsgs_secondcheck/thirdcheck 4271-4368, bsgs_searchbinary 3748-3773,
//                 calcualteindex 6680-6689
#pragma once
#include <stdint.h>
#include <functional>
#include <string>
#include <vector>

#include "bloom_host.hpp"
#include "secp_host.hpp"
#include "u256.hpp"

namespace khb {

struct Geometry {
  U256 N, M, M2, M3, M_double, M2_double, M3_double, N_double, intaux;
  uint64_t m = 0, m2 = 0, m3 = 0, aux = 0, cycles = 0, l1ext = 0;
  uint64_t items1 = 0, items2 = 0, items3 = 0;
};

// n_str: the -n argument ("0x..." hex or decimal) or nullptr for the default 2^44.
bool make_geometry(const char* n_str, int kfactor, Geometry& g, std::string& err);

struct XValue {            // struct bsgs_xvalue, keyhunt.cpp:70-73
  uint8_t value[6];
  uint8_t pad[2];
  uint64_t index;
};

// -S table files (keyhunt.cpp:1373-1613 read, 1881-2025 write): which of them a Tables holds
// from disk.  Bits: 1 = L1 keyhunt_bsgs_4_<m>.blm, 2 = L2 _6_<m2>.blm, 4 = bPtable _2_<m3>.tbl,
// 8 = L3 _7_<m3>.blm.
enum : uint32_t { kFileL1 = 1, kFileL2 = 2, kFileBp = 4, kFileL3 = 8, kFileAll = 15 };

struct Tables {
  Geometry geo;
  std::vector<BloomFilter> l1, l2, l3;   // 256 sub-blooms each
  std::vector<XValue> bp;                // sorted by value (bsgs_sort)
  Pt gsn[512], g2sn, amp2[32], amp3[32];
  uint32_t gpl = 0;                      // GPU groups per lane
  // Level-0 gate for the GPU probe (khb_load_gate): a blocked bloom (64-bit blocks, gate_probes
  // bits per x) holding every x of the L1 set.  Built with the baby steps when the L1 set is
  // walked (always on the GPU path; on the CPU path only when L1 is built, not read from a file);
  // gate_log2 = 0: none.
  std::vector<uint8_t> gate;
  uint32_t gate_log2 = 0, gate_probes = 0;
  // Gate size for a geometry: 2^KHB_GATE_SPARSITY (default 64) bits per L1 x rounded up to a
  // power of two, at most 2^30 bits (128 MiB) or 2^KHB_GATE_LOG2 from the environment (0
  // disables); 0 when the map would be more than ~22 % full (fewer than 4 bits per x).  Probes:
  // KHB_GATE_PROBES (default 3).  k = 1: 2^28 bits, 3 bits per x in one 64-bit block.
  static uint32_t gate_log2_for(const Geometry& g);
  static uint32_t gate_probes_for();
  std::vector<Pt> lane_offs;             // offs[m] = (m*gpl) * _2GSn

  // progress(done, total) is called from the builder threads' coordinator.  `have` marks tables
  // already loaded from -S files (load_files): their baby-step work is skipped, and with L1 loaded
  // only the first m2 baby steps are walked (keyhunt.cpp:1617-1700, "only 3% of the work").
  // gpu_device >= 0 walks the baby steps on that GPU (khb_build_baby); the tables are identical.
  bool build(const Geometry& g, int nthreads, uint32_t groups_per_lane, std::string& err,
             const std::function<void(uint64_t, uint64_t)>& progress = nullptr, uint32_t have = 0,
             int gpu_device = -1);
  double build_gpu_ms = 0;               // kernel time of the last GPU baby-step build
  // -S: read the reference's table files for this geometry from dir (prepare() first).  Returns the
  // kFile* mask read; false + err on a short read or checksum mismatch (the reference exits).
  void prepare(const Geometry& g);
  bool load_files(const std::string& dir, bool skip_checksum, uint32_t& have, std::string& err,
                  const std::function<void(const std::string&)>& log) ;
  // -S: write every table not in `have` in the reference's format.
  bool save_files(const std::string& dir, uint32_t have, std::string& err,
                  const std::function<void(const std::string&)>& log) const;
  static std::string file_name(const Geometry& g, uint32_t which);
  std::vector<uint8_t> l1_concat() const;
  std::vector<uint8_t> bloom_concat(int level) const;    // level 1..3: 256 sub-blooms concatenated
  std::vector<uint8_t> amp_table_be(int level) const;    // level 2, 3: BSGS_AMP2 / BSGS_AMP3, 32 x||y BE
  std::vector<uint8_t> giant_table_be() const;
  std::vector<uint8_t> lane_offsets_be() const;

  // (order - base - intaux) * G, shared by every target of a chunk (keyhunt.cpp:3862-3866)
  Pt chunk_aux(const U256& base) const;
  // chunk_aux of n consecutive chunks base0 + c * 2N, batched (one scalar multiplication per 64)
  void chunk_aux_run(const U256& base0, size_t n, Pt* aux, int threads) const;
  bool secondcheck(const U256& base, uint32_t a, const Pt& target, U256& key) const;

 private:
  bool thirdcheck(const U256& base2, uint32_t i2, const Pt& target, U256& key) const;
  bool searchbinary(const uint8_t* x, uint64_t& idx) const;
};

// Batched chunk centres: out[k] = AddDirect(targets[k], aux) with one shared inversion.
void batch_add_direct(const Pt* targets, const Pt& aux, size_t n, Pt* out);
// out[i] = AddDirect(a[i], b[i]) with one shared inversion
void batch_add_pairs(const Pt* a, const Pt* b, size_t n, Pt* out);

}  // namespace khb
