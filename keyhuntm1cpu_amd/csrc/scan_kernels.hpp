// Device side of libkhbsgs (gfx950): the giant-step walk and its kernel k_giant_scan<MODE>, shared by
// the translation units that instantiate it (k_bsgs.hip: -m bsgs scan / x dump; k_addr.hip: -m address;
// k_baby.hip: baby-step tables) and by khbsgs.hip (types, self-test kernels, the C ABI).  Splitting the
// instances over translation units lets `make -j` compile them in parallel.
//
// Hot path replaced: keyhunt.cpp:3867-4004 (thread_process_bsgs group loop + level-1 bloom probe).
//
// Work decomposition:
//   job   = one (chunk, target) pair; the host supplies its group-0 centre startP.
//   item  = consecutive 1024-point groups of one job (scan_batch: 8 groups with two inversions).
//   grid  = persistent: one residency of lanes; each wave takes the next 64 items from a launch counter.
// One lane's group maps 1:1 onto one reference group, so a collapsed batch inverse (dx == 0)
// reproduces the reference's all-zero inverses exactly (IntGroup.cpp:36-58 + IntMod.cpp:497-500).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/khbsgs.h"
#include "device/fe.hpp"
#include "device/fe_asm.hpp"
#include "device/bloom_probe.hpp"
#include "device/hash160.hpp"

using namespace khb;

namespace khbk {

struct AffPt {
  Fe x, y;
};

#ifndef KHB_GATE1
#define KHB_GATE1 1               // default stage-1 fold of the level-0 gate: KHB_GATE_STAGE1_AUTO (khbsgs.h)
#endif
#ifndef KHB_GATE0
// default stage-0 filter in front of the fold (khb_set_gate_stage0): none.  The 2 MiB filter at k = 4 (KHB_GATE_STAGE0_AUTO)
// ran 4.6 % SLOWER on config C (48,629 vs 50,948 Mkeys/s, 3 + 3 alternating runs, profiles/r06a/gate0): it cuts the
// fold's MALL reads to 63 % but adds one L2 lane-load per x, and a gate lane-load costs its memory-pipeline cycles
// wherever it is served.
#define KHB_GATE0 0
#endif
#ifndef KHB_WAVES_PER_SIMD
// occupancy target of k_giant_scan (launch bounds).  Round 4: 4 waves/SIMD (128 VGPRs, 262,144 lanes; the walk's
// hot path has the same 1,171 VALU per step as at 3 waves) ran 3.0 % faster than 3 (168 VGPRs) with two
// launches in flight, at 3,072 and at 4,096 chunks per launch, and 5 waves (96 VGPRs, spilling) 16 % slower
// (profiles/r04q/waves_pipe_ab.txt).  Round 3, before the L2 gate fold and the non-temporal prefix stream,
// had measured 3 waves 1.4-1.6 % faster than 4 (profiles/r03_calibration/occupancy_ab*.txt).
#define KHB_WAVES_PER_SIMD 4
#endif
constexpr uint32_t kBlock = 256;
#ifndef KHB_BATCH
#define KHB_BATCH 8               // -m bsgs groups per work item (scan_batch): two inversions per item
#endif
constexpr uint32_t kBatch = KHB_BATCH;
#ifndef KHB_HALF_STREAM
// 1 (the product since round 6): the half prefix stream (walk_group_g_half): the gated scan's forward pass stores only
// the odd prefixes and the walk rebuilds each even one from its odd neighbour, one extra product per two walk steps
// for half the HBM stream.  Exact (the same products of the same operands in the same order).  Whole-bench +1.1 % on
// one box (round 5, profiles/r05e) and +1.2 % on another (55,423 vs 54,777 Mkeys/s, 3 + 3 alternating runs,
// profiles/r06a/half); the board runs at its power cap and the halved stream lowers the energy per cycle (launch
// clock 2,310 vs 2,184 MHz).  DESIGN.md §5.
#define KHB_HALF_STREAM 1
#endif
constexpr bool kHalfStream = KHB_HALF_STREAM != 0;

// Kernel modes (template argument of scan_group / k_giant_scan).
enum : int {
  kScan = 0,       // -m bsgs: level-1 bloom probe of every x
  kDump = 1,       // -m bsgs parity: write every x
  kAddrU = 2,      // -m address, -l uncompress   (2 + keyhunt SEARCH_UNCOMPRESS, keyhunt.cpp:59-61)
  kAddrC = 3,      // -m address, -l compress
  kAddrB = 4,      // -m address, -l both (the reference default, keyhunt.cpp:300)
  kAddrDump = 5,   // -m address parity: write every x||y
  kBaby = 6,       // baby-step table build: bloom_add of every x into L1/L2/L3 + bPtable records
  kScanG = 7,      // -m bsgs with a level-0 gate (the product path: walk_group_g)
  kScanG1 = 8,     // kScanG with the gate's stage-1 fold in front (khb_set_gate_stage1)
  kScanG2 = 9,     // kScanG1 with the stage-0 filter in front of the fold (khb_set_gate_stage0; k >= 4)
  kAddrUE = 10,    // kAddrU / kAddrC / kAddrB with -e (KHB_SEARCH_ENDOMORPHISM: beta*x, beta^2*x, negated y;
  kAddrCE = 11,    //   keyhunt.cpp:2646-2763)
  kAddrBE = 12,
};
constexpr bool is_gated(int m) { return m == kScanG || m == kScanG1 || m == kScanG2; }
// filter stages in front of the full gate: 0 (kScanG), 1 (the fold, kScanG1), 2 (filter + fold, kScanG2)
constexpr int gate_stages(int m) { return m == kScanG2 ? 2 : m == kScanG1 ? 1 : 0; }
constexpr bool is_scan(int m) { return m == kScan || is_gated(m); }
constexpr bool is_endo(int m) { return m >= kAddrUE && m <= kAddrBE; }
constexpr bool is_addr(int m) { return (m >= kAddrU && m <= kAddrDump) || is_endo(m); }
constexpr bool needs_y(int m) { return m == kAddrU || m == kAddrB || m == kAddrDump || m == kAddrUE || m == kAddrBE; }
constexpr bool addr_compressed(int m) { return m == kAddrC || m == kAddrB || m == kAddrCE || m == kAddrBE; }
constexpr bool addr_uncompressed(int m) { return m == kAddrU || m == kAddrB || m == kAddrUE || m == kAddrBE; }
constexpr bool is_dump(int m) { return m == kDump || m == kAddrDump || m == kBaby; }
#ifndef KHB_ADDR_WAVES_PER_SIMD
#define KHB_ADDR_WAVES_PER_SIMD KHB_WAVES_PER_SIMD   // occupancy target of the -m address hash kernels
#endif
#ifndef KHB_ADDR_E_WAVES_PER_SIMD
#define KHB_ADDR_E_WAVES_PER_SIMD KHB_ADDR_WAVES_PER_SIMD   // occupancy target of the -e address kernels
#endif
constexpr int waves_per_simd(int m) {
  return is_endo(m) ? KHB_ADDR_E_WAVES_PER_SIMD : is_addr(m) ? KHB_ADDR_WAVES_PER_SIMD : KHB_WAVES_PER_SIMD;
}
constexpr uint32_t kHalf = KHB_GROUP / 2;            // 512
constexpr uint32_t kCandCap = 1u << 20;
constexpr uint32_t kAddrHitCap = 1u << 18;
constexpr uint32_t kDegenCap = 4096;
constexpr size_t kCounterBytes = 64;                 // ScanArgs::counters
constexpr size_t kHostCounterBytes = 128;            // ScanArgs::host_counters (launch_epilogue)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// Prefix-scratch stream (written once by the forward pass, read once by the walk ~512 steps later, from
// HBM: ~35 GB per slot at 262,144 lanes).  Non-temporal loads and stores keep it from displacing the level-0 gate's L2-sized
// stage-1 fold (khb_set_gate_stage1): -1.5 % time with two launches in flight, -0.3 % as one launch
// (profiles/r04i/nt_ab.txt, r04h/ntall_ab.txt).  Without the fold (round 1, 4 waves/SIMD) they measured
// slower (profiles/r01_gate_experiments_raw.txt); tools/experiments/plainscr_patch.py builds the plain form.
__device__ __forceinline__ void scr_st(Fe* p, const Fe& v) {
  v4u* q = reinterpret_cast<v4u*>(p);
  __builtin_nontemporal_store(v4u{v.v[0], v.v[1], v.v[2], v.v[3]}, q);
  __builtin_nontemporal_store(v4u{v.v[4], v.v[5], v.v[6], v.v[7]}, q + 1);
}
__device__ __forceinline__ Fe scr_ld(const Fe* p) {
  const v4u* q = reinterpret_cast<const v4u*>(p);
  const v4u lo = __builtin_nontemporal_load(q), hi = __builtin_nontemporal_load(q + 1);
  return Fe{{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w}};
}

struct ScanArgs {
  const uint8_t* __restrict__ bloom;
  BloomGeom geom;
  const AffPt* __restrict__ gsn;       // [0..511] GSn, [512] _2GSn
  const AffPt* __restrict__ offs;      // lane start offsets
  const AffPt* __restrict__ gofs;      // per-group centre offsets j*_2GSn (scan_batch)
  const AffPt* __restrict__ centres;   // per-job group-0 centre (khb_submit: pinned host memory, read in place)
  Fe* __restrict__ scratch;            // prefix products [512][lanes]
  khb_cand* __restrict__ cand;         // candidate ring (khb_submit: pinned host memory, written in place)
  khb_degenerate* __restrict__ degen;  // degenerate-group ring (same)
  uint32_t* __restrict__ counters;     // [0] candidates [1] degenerate groups [2] work-item cursor (dynamic items)
                                       // [3] waves finished (launch_epilogue)
                                       // [4..5] groups walked (u64, count_walked)
                                       // [8..15] shader clock probe (clock_probe): memtime, realtime at the
                                       // first wave's start, then at its end (u64 each)
  uint32_t* __restrict__ host_counters;  // launch_epilogue: the last wave copies counters[0..15] here (pinned host
                                         // memory), adds its end clocks at [16..19] and zeroes counters[0..7] for
                                         // the slot's next launch; null = off
  uint32_t total_waves;                // waves of the launch (launch_epilogue)
  uint8_t* __restrict__ xdump;         // dump modes only
  uint32_t* __restrict__ ahits;        // -m address hits: {job, group, t, kind} x ahit_cap
  uint32_t ahit_cap;
  // kBaby: word-aligned blooms (sub-bloom stride bwords[l] 32-bit words; null = level skipped)
  uint32_t* __restrict__ bw[3];
  BloomGeom bgeom[3];
  uint64_t bwords[3];
  uint64_t blimit[3];                  // ic < blimit[l] goes into level l (l1ext, m2, m3)
  uint32_t* __restrict__ bp;           // m3 x 16-byte struct bsgs_xvalue records (null = skipped)
  // level-0 gate (khb_load_gate): a blocked bloom of (gate_mask + 1) 64-bit blocks; x selects
  // block x.v[0] & gate_mask and in it bit (x.v[1] >> 5p) & 31 of word p & 1, p < gate_probes, all
  // set for every x of the L1 set; null = no gate.  kBaby writes it (gate_w, ic < glimit).
  const uint8_t* __restrict__ gate;
  uint32_t* __restrict__ gate_w;
  uint32_t gate_probes;
  uint64_t glimit;
  uint32_t gate_mask;                  // blocks - 1
  // stage-1 gate (khb_set_gate_stage1): the level-0 gate OR-folded to (gate1_mask + 1) blocks, block i of
  // the fold = OR of blocks j of the gate with j & gate1_mask == i; null = no stage 1
  const uint8_t* __restrict__ gate1;
  uint32_t gate1_mask;
  // stage-0 filter (khb_set_gate_stage0): one bit per baby-step x, the gate's hi words (probe 1) OR-folded to
  // (gate0_mask + 1) 32-bit words, word i = OR of the hi words of the gate's blocks j with j & gate0_mask == i;
  // null = no stage 0
  const uint32_t* __restrict__ gate0;
  uint32_t gate0_mask;
  uint64_t job_keys;                   // baby steps per job
  uint64_t n_items;
  uint32_t n_jobs, group_begin, group_end, gpl, lanes_per_job, stride, cand_cap, degen_cap;
};

__device__ __forceinline__ void emit_cand(const ScanArgs& A, uint32_t job, uint32_t a) {
  uint32_t k = atomicAdd(&A.counters[0], 1u);
  if (k < A.cand_cap) A.cand[k] = khb_cand{job, a};
}

// ---- level-1 probe with a per-wave survivor queue ---------------------------------------------
// Without a gate every x pays the first XXH64 and one bit load: L1 bit 0; the ~50 % whose bit is
// set are pushed to a per-wave LDS queue (x, a, job, giant-step index); whenever 64 are queued the
// whole wave finishes 64 of them together (second XXH64 + remaining bits, bloom_rest).  Without
// the queue a wave would run the second hash and the dependent bit loads whenever ANY of its lanes
// survived, i.e. for every x, with one memory round trip per bit per probe site.
//
// With a level-0 gate (khb_load_gate) x pays no hash at all: one byte of a 2^L-bit map (L = 28 at
// k = 1, 32 MiB) addressed by the low L bits of x, with the bit of every baby-step x of the L1 set
// set, so no L1 member is ever dropped.  Only the gate's survivors (~1.5 %) are queued, and the
// drain runs the whole L1 check (XXH64 a, bloom_full).  The candidate stream is the L1 candidates
// whose gate bit is set: every true member, and ~1.5 % of the false positives that
// bsgs_secondcheck would reject.
constexpr uint32_t kDrainAt = 64;          // drain threshold (entries): one per lane
constexpr uint32_t kQCap = kDrainAt + 64;           // entries per wave: < kDrainAt resident + <= 64 pushed
constexpr uint32_t kQWords = 10;           // x[8], job, step index (SoA in LDS)
constexpr uint32_t kWavesPerBlock = kBlock / 64;

// The count lives in LDS, not in a register: lanes of a wave may diverge (the ragged last lane of
// a job, the tail of the item loop), and a register copy would go stale in the inactive lanes.
struct ProbeQueue {
  uint32_t* q;            // this wave's LDS region: kQWords arrays of kQCap words
  // this wave's queued-entry count, typed as an LDS pointer: through a generic (flat) pointer
  // every count access was a flat_load/flat_store, which counts against vmcnt AND lgkmcnt and
  // made each one wait for all outstanding vector-memory operations (the prefetched prefix).
  volatile __attribute__((address_space(3))) uint32_t* n;
};

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Read queued entry k (x, job, step).
__device__ __forceinline__ void q_read(const ProbeQueue& Q, uint32_t k, Fe& x, uint32_t& job, uint32_t& step) {
#pragma unroll
  for (int d = 0; d < 8; ++d) x.v[d] = Q.q[d * kQCap + k];
  job = Q.q[8 * kQCap + k];
  step = Q.q[9 * kQCap + k];
}

// Finish the newest min(n, active lanes) queued entries, one per lane, while n >= threshold.
__device__ __forceinline__ void q_drain(const ScanArgs& A, ProbeQueue& Q, uint32_t threshold) {
  for (;;) {
    const uint32_t n = *Q.n;
    if (n < threshold || n == 0) break;
    const uint64_t em = __ballot(1);
    const uint32_t take = min(n, (uint32_t)__popcll(em));
    const uint32_t r = lane_rank(em);
    *Q.n = n - take;
    asm volatile("" ::: "memory");
    if (r < take) {
      Fe x;
      uint32_t job, step;
      q_read(Q, n - take + r, x, job, step);
      fm_canon(x, x);                   // gated pushes hold lazy x (x_out)
      uint64_t w[4];
      x_words(w, x);
      // the whole level-1 check (bit 0 again for ungated pushes: the first hash is not queued)
      if (bloom_full<1>(sub_bloom(A.bloom, A.geom, x), A.geom, w, xxh64_32(w, KHB_BLOOM_SEED)))
        emit_cand(A, job, step);
    }
    asm volatile("" ::: "memory");
  }
}

// Queue x if its first bit (L1 bit 0, or the gate bit) is set.
__device__ __forceinline__ void q_push(ProbeQueue& Q, bool hit, const Fe& x, uint32_t job, uint32_t step) {
  const uint64_t m = __ballot(hit);
  const uint32_t n = *Q.n;
  if (hit) {
    const uint32_t k = n + lane_rank(m);
#pragma unroll
    for (int d = 0; d < 8; ++d) Q.q[d * kQCap + k] = x.v[d];
    Q.q[8 * kQCap + k] = job;
    Q.q[9 * kQCap + k] = step;
  }
  asm volatile("" ::: "memory");
  *Q.n = n + (uint32_t)__popcll(m);
}

// The gate's bits in x's 64-bit block (lo, hi words): probe p tests bit b_p = (w1 >> 5p) mod 32 of word
// p mod 2 (p = 0: lo, 1: hi, 2: lo), w1 = x.v[1].  Each probe is one left shift by 31 - b_p = (~w1 >> 5p)
// mod 32 that brings its bit to bit 31 (the hardware takes a 32-bit shift's amount mod 32, so the amounts
// need no mask and no word select); the block passes when the AND of the three shifted words is negative.
// The amounts are computed once per x and shared by the stage-1 fold's test and the full gate's.  Fewer
// probes than 3 need no per-lane masks: probe 2 repeats probe 0 (shift distance 0 instead of 10,
// wave-uniform), and for one probe khb_load_gate sets every block's hi word, so probe 1 always passes.
struct GateBits {
  uint32_t a0, a1, a2;   // left-shift amounts (mod 32) of probes 0, 1, 2
};
__device__ __forceinline__ uint32_t gate_s2(const ScanArgs& A) { return A.gate_probes >= 3 ? 10u : 0u; }
__device__ __forceinline__ GateBits gate_bits(uint32_t w1, uint32_t s2) {
  const uint32_t n = ~w1;
  return GateBits{n, n >> 5, n >> s2};
}
// v_lshlrev_b32 as the hardware reads it (amount mod 32); opaque to the compiler, which otherwise masks
// an amount computed in another basic block with a v_and_b32 (round-4 ISA of the fold's second test)
__device__ __forceinline__ uint32_t shl_mod32(uint32_t x, uint32_t s) {
  uint32_t r;
  asm("v_lshlrev_b32 %0, %1, %2" : "=v"(r) : "v"(s), "v"(x));
  return r;
}
__device__ __forceinline__ bool gate_block_pass(uint2 w, GateBits b) {
  return (int32_t)(shl_mod32(w.x, b.a0) & shl_mod32(w.y, b.a1) & shl_mod32(w.x, b.a2)) < 0;
}
__device__ __forceinline__ uint2 gate_block(const uint8_t* g, uint32_t mask, const Fe& x) {
  return reinterpret_cast<const uint2*>(g)[x.v[0] & mask];
}

// kScanG: gate test of one walk step's two x (x2 absent at step 511: has2 = false, uniform).  Both
// blocks are loaded before either is waited for; survivors (~0.04 % of x) go to the queue.
// STAGES (gate_stages): 1 tests the stage-1 fold first, 2 tests the stage-0 filter before the fold.  Each stage
// is a superset of the next, so the queued x are exactly the full gate's survivors in every case.
template <int STAGES>
__device__ __forceinline__ void gate_pair(const ScanArgs& A, ProbeQueue& Q, const Fe& x1, uint32_t step1, bool has2,
                                          const Fe& x2, uint32_t step2, uint32_t job) {
  bool h1, h2;
  const uint32_t s2 = gate_s2(A);
  const GateBits b1 = gate_bits(x1.v[1], s2), b2 = gate_bits(x2.v[1], s2);
  if constexpr (STAGES >= 1) {
    bool s1 = true, s2p = has2;
    if constexpr (STAGES == 2) {
      // stage 0 (L2-resident, one bit per member: ~63 % of x pass at k = 4); the fold's line (read from the MALL at
      // k = 4) is fetched only for its survivors.  No ballot: with ~63 % passing a wave almost never skips.
      const uint32_t v1 = A.gate0[x1.v[0] & A.gate0_mask], v2 = A.gate0[x2.v[0] & A.gate0_mask];
      s1 = (int32_t)shl_mod32(v1, b1.a1) < 0;
      s2p = has2 && (int32_t)shl_mod32(v2, b2.a1) < 0;
    }
    // stage 1 (the fold: L2-resident at k = 1); the full gate's line is fetched only for its survivors
    uint2 f1, f2;                                  // read only where loaded (s1 / s2p)
    if (STAGES == 1 || s1) f1 = gate_block(A.gate1, A.gate1_mask, x1);
    if (STAGES == 1 || s2p) f2 = gate_block(A.gate1, A.gate1_mask, x2);
    s1 = s1 && gate_block_pass(f1, b1);
    s2p = s2p && gate_block_pass(f2, b2);
    if (__ballot(s1 || s2p) == 0) return;
    uint2 w1, w2;                                  // read only where loaded (s1 / s2p)
    if (s1) w1 = gate_block(A.gate, A.gate_mask, x1);
    if (s2p) w2 = gate_block(A.gate, A.gate_mask, x2);
    h1 = s1 && gate_block_pass(w1, b1);
    h2 = s2p && gate_block_pass(w2, b2);
  } else {
    const uint2 w1 = gate_block(A.gate, A.gate_mask, x1), w2 = gate_block(A.gate, A.gate_mask, x2);
    h1 = gate_block_pass(w1, b1);
    h2 = has2 && gate_block_pass(w2, b2);
  }
  if (__ballot(h1 || h2) == 0) return;
  q_push(Q, h1, x1, job, step1);
  q_drain(A, Q, kDrainAt);
  q_push(Q, h2, x2, job, step2);
  q_drain(A, Q, kDrainAt);
}

// Gate bits of x (blocked gate), or without a gate L1 bit 0 (a = the first XXH64).
__device__ __forceinline__ bool first_bit(const ScanArgs& A, const Fe& x, uint64_t& a) {
  if (A.gate) {
    a = 0;
    return gate_block_pass(gate_block(A.gate, A.gate_mask, x), gate_bits(x.v[1], gate_s2(A)));
  }
  uint64_t w[4];
  x_words(w, x);
  a = xxh64_32(w, KHB_BLOOM_SEED);
  return test_bit(sub_bloom(A.bloom, A.geom, x), mod_bits(a, A.geom));
}

template <bool DUMP>
__device__ __forceinline__ void probe(const ScanArgs& A, ProbeQueue& Q, const Fe& x, uint32_t job, uint32_t j,
                                      uint32_t t) {
  if (DUMP) {
    uint8_t* o = A.xdump + ((uint64_t)(j - A.group_begin) * KHB_GROUP + t) * 32;
    fe_to_be(o, x);
  } else {
    uint64_t a;
    const bool hit = first_bit(A, x, a);
    q_push(Q, hit, x, job, j * KHB_GROUP + t);
    q_drain(A, Q, kDrainAt);
  }
}

// The two points of one backward step (C - GSn[i], C + GSn[i]): both first hashes are computed
// before either bloom bit is awaited, so the two loads share one memory round trip.
template <bool DUMP>
__device__ __forceinline__ void probe_pair(const ScanArgs& A, ProbeQueue& Q, const Fe& x1, const Fe& x2,
                                           uint32_t job, uint32_t j, uint32_t t1, uint32_t t2) {
  if (!DUMP) {
    uint64_t a1, a2;
    const bool h1 = first_bit(A, x1, a1);
    const bool h2 = first_bit(A, x2, a2);
    q_push(Q, h1, x1, job, j * KHB_GROUP + t1);
    q_drain(A, Q, kDrainAt);
    q_push(Q, h2, x2, job, j * KHB_GROUP + t2);
    q_drain(A, Q, kDrainAt);
    return;
  }
  probe<DUMP>(A, Q, x1, job, j, t1);
  probe<DUMP>(A, Q, x2, job, j, t2);
}

// GSn / _2GSn rows (wave-uniform index), read through the constant address space, so rows arrive
// by scalar loads into SGPRs (lgkmcnt) instead of taking 16 VGPRs and four vector-memory slots per
// backward step.
struct GsnTable {
  const AffPt* p;
  typedef const __attribute__((address_space(4))) uint32_t* CW;
  __device__ __forceinline__ Fe ld(uint32_t word) const {
    CW w = (CW)p + word;
    Fe r;
#pragma unroll
    for (int k = 0; k < 8; ++k) r.v[k] = w[k];
    return r;
  }
  __device__ __forceinline__ Fe x(uint32_t i) const { return ld(16 * i); }
  __device__ __forceinline__ AffPt pt(uint32_t i) const { return AffPt{ld(16 * i), ld(16 * i + 8)}; }
  // p - GSn[i].x (0 for x = 0), stored after the 513 points (khb_load_giant_table)
  __device__ __forceinline__ Fe nx(uint32_t i) const { return ld(16 * KHB_GIANT_TABLE + 8 * i); }
};

// -m address handling of one point (keyhunt.cpp:2716-2937, BTC, no endomorphism): hash160 of
// the compressed key for both prefixes from x alone (covers +k and -k, keyhunt.cpp:2719-2733) and/or
// of the uncompressed key, each probed in the single target bloom; hits go to the host, which runs
// searchbinary and the key recovery.  x and y are canonical.
template <int MODE>
__device__ __forceinline__ void addr_point(const ScanArgs& A, const Fe& x, const Fe& y, uint32_t job, uint32_t j,
                                           uint32_t t) {
  if constexpr (MODE == kAddrDump) {
    uint8_t* o = A.xdump + ((uint64_t)(j - A.group_begin) * KHB_GROUP + t) * 64;
    fe_to_be(o, x);
    fe_to_be(o + 32, y);
  } else {
    uint32_t h[5];
    auto emit = [&](uint32_t kind) {
      const uint32_t k = atomicAdd(&A.counters[0], 1u);
      if (k < A.ahit_cap) {
        uint32_t* o = A.ahits + 4 * (size_t)k;
        o[0] = job; o[1] = j; o[2] = t; o[3] = kind;
      }
    };
    if constexpr (is_endo(MODE)) {
      // -e (keyhunt.cpp:2646-2763): lambda*P = (beta*x, y) and lambda^2*P = (beta^2*x, y) (keyhunt.cpp:582-585).
      // Compressed: the 02 and 03 hashes of x, beta*x, beta^2*x (kinds 0|e<<2, 1|e<<2); uncompressed: (x_e, y) and
      // (x_e, p - y), the negated point (kinds 2|e<<2, 3|e<<2).  Every x_e is canonical before it is hashed.
      // beta (keyhunt.cpp:584); beta^2*x is computed as beta*(beta*x), the same canonical value as the reference's
      // ModMulK1(x, beta2) (beta2 = beta^2 mod p, keyhunt.cpp:585), with one constant and no indexed table
      const Fe kBeta = {{0x719501eeu, 0xc1396c28u, 0x12f58995u, 0x9cf04975u, 0xac3434e9u, 0x6e64479eu, 0x657c0710u,
                         0x7ae96a2bu}};
      Fe ny;
      if constexpr (addr_uncompressed(MODE)) {
        Fe p;
#pragma unroll
        for (int k = 0; k < 8; ++k) p.v[k] = k == 0 ? KHB_P0 : (k == 1 ? KHB_P1 : 0xFFFFFFFFu);
        fm_sub(ny, p, y);                          // y != 0 on the curve: p - y is canonical
        fm_canon(ny, ny);
      }
      Fe xe = x;
#pragma unroll 1
      for (uint32_t e = 0; e < 3; ++e) {
        if (e) {
          fm_mul(xe, xe, kBeta);
          fm_canon(xe, xe);
        }
        if constexpr (addr_compressed(MODE)) {
#pragma unroll 1
          for (uint32_t pre = 2; pre <= 3; ++pre) {
            hash160_compressed(h, pre, xe);
            if (bloom_check20(A.bloom, A.geom, h)) emit((pre - 2) | (e << 2));
          }
        }
        if constexpr (addr_uncompressed(MODE)) {
          // one copy of the two-block hash in the loop body (unrolled twice it spilled ~700 VGPRs)
#pragma unroll 1
          for (uint32_t neg = 0; neg < 2; ++neg) {
            Fe yy;
#pragma unroll
            for (int k = 0; k < 8; ++k) yy.v[k] = neg ? ny.v[k] : y.v[k];
            hash160_uncompressed(h, xe, yy);
            if (bloom_check20(A.bloom, A.geom, h)) emit((2u + neg) | (e << 2));
          }
        }
      }
    } else {
      if constexpr (MODE == kAddrC || MODE == kAddrB) {
#pragma unroll 1
        for (uint32_t pre = 2; pre <= 3; ++pre) {
          hash160_compressed(h, pre, x);
          if (bloom_check20(A.bloom, A.geom, h)) emit(pre - 2);
        }
      }
      if constexpr (MODE == kAddrU || MODE == kAddrB) {
        hash160_uncompressed(h, x, y);
        if (bloom_check20(A.bloom, A.geom, h)) emit(2);
      }
    }
  }
}

// bloom_add (bloom.cpp:61-85, 159-162) of a 32-byte x into sub-bloom x[0] of a word-aligned level.
__device__ __forceinline__ void bloom_add_words(uint32_t* __restrict__ words, const BloomGeom& g, uint64_t a,
                                                uint64_t b) {
  uint64_t pos = mod_bits(a, g);
  const uint64_t bm = mod_bits(b, g);
  uint64_t h = a;
  for (uint32_t i = 0; i < g.hashes; ++i) {
    if (i) {
      const uint64_t nh = h + b;
      const bool wrapped = nh < h;
      h = nh;
      pos += bm;
      if (pos >= g.bits) pos -= g.bits;
      if (wrapped) pos = (pos >= g.wrap) ? pos - g.wrap : pos + g.bits - g.wrap;
    }
    // bf[pos >> 3] |= 1 << (pos & 7): little-endian words, so bit (pos & 31) of word pos >> 5
    atomicOr(words + (pos >> 5), 1u << (pos & 31));
  }
}

// Baby step ic = job * job_keys + 1024 j + t (key ic + 1): thread_bPload (keyhunt.cpp:4404-4592).
__device__ __forceinline__ void baby_point(const ScanArgs& A, const Fe& x, uint32_t job, uint32_t j, uint32_t t) {
  const uint64_t ic = (uint64_t)job * A.job_keys + (uint64_t)j * KHB_GROUP + t;
  if (ic >= A.blimit[0] && ic >= A.blimit[1] && ic >= A.blimit[2] && ic >= A.glimit) return;
  uint64_t w[4];
  x_words(w, x);
  const uint64_t a = xxh64_32(w, KHB_BLOOM_SEED);
  if (A.gate_w && ic < A.glimit) {
    const uint32_t blk = x.v[0] & A.gate_mask;
    for (uint32_t p = 0; p < A.gate_probes; ++p)      // gate_block_pass: bit (w1 >> 5p) mod 32 of word p mod 2
      atomicOr(A.gate_w + 2 * blk + (p & 1u), 1u << ((x.v[1] >> (5 * p)) & 31u));
  }
  const uint64_t b = xxh64_32(w, a);
  const uint32_t sub = x.v[7] >> 24;
#pragma unroll 1
  for (int l = 0; l < 3; ++l)
    if (A.bw[l] && ic < A.blimit[l]) bloom_add_words(A.bw[l] + sub * A.bwords[l], A.bgeom[l], a, b);
  if (A.bp && ic < A.blimit[2]) {
    // struct bsgs_xvalue {value = x bytes 16..21 (Get32Bytes order), pad[2] = 0, index = ic}
    uint32_t* o = A.bp + 4 * ic;
    o[0] = __builtin_bswap32(x.v[3]);
    o[1] = (x.v[2] >> 24) | (((x.v[2] >> 16) & 0xffu) << 8);
    o[2] = (uint32_t)ic;
    o[3] = (uint32_t)(ic >> 32);
  }
}

// x for the probe.  With a gate only the low word of x is read before the drain, and a lazy x
// (< 2^256, congruent) differs from the canonical one only when x >= p, which needs x.v[7] ==
// 0xffffffff (p's top word): the full canonicalisation runs only then (wave-uniform skip, ~2^-26
// per wave), and the drain canonicalises its survivors before hashing.
template <int MODE>
__device__ __forceinline__ void x_out(const ScanArgs& A, Fe& x) {
  if ((MODE == kScan && A.gate) || is_gated(MODE)) {
    if (x.v[7] == 0xffffffffu) fm_canon(x, x);
  } else {
    fm_canon(x, x);
  }
}

// The 1023 x-only additions C -/+ GSn[i] and the centre of one reference group, in the
// reference's backward order (keyhunt.cpp:3873-3943 / 2586-2711), given inv = the inverse of
// prod_{i<512} (GSn[i].x - C.x) and the forward prefix products in scr[0..510] (stride lanes).
// C is canonical; products are lazy (< 2^256) and every x (and y) is canonicalised before it is
// hashed or dumped (fe_asm.hpp value contract).
template <int MODE>
__device__ __forceinline__ void walk_group(const ScanArgs& A, ProbeQueue& Q, const AffPt& C, Fe inv, uint32_t job,
                                           uint32_t j, const Fe* scr) {
  constexpr bool DUMP = MODE == kDump;
  const uint32_t S = A.stride;
  const GsnTable gsn{A.gsn};
  Fe pre, dx;
  // scan modes: the prefix for step i-1 is loaded during step i, so its HBM latency hides behind a
  // whole step's arithmetic instead of being waited for right after the load.
  constexpr bool PREFETCH = is_scan(MODE);
  // The load goes into `pre` itself right after its last use (no loop-carried copy: a copy at the
  // loop latch would make the wave wait for the load there).
  if (PREFETCH) pre = scr[(size_t)(kHalf - 2) * S];
  // -m bsgs x-only walks: C.x is carried as negCx = p - C.x, so dx = GSn.x + negCx and
  // x = s^2 + (negCx - GSn.x) need no separate modular subtraction of the centre.
  constexpr bool FUSED = MODE == kScan || MODE == kDump;
  Fe negCx;
  if constexpr (FUSED) {
    Fe p;
#pragma unroll
    for (int k = 0; k < 8; ++k) p.v[k] = k == 0 ? KHB_P0 : (k == 1 ? KHB_P1 : 0xFFFFFFFFu);
    fm_sub(negCx, p, C.x);
  }
  for (int i = (int)kHalf - 1; i >= 0; --i) {
    Fe idx;
    if (i > 0) {
      if (!PREFETCH) pre = scr[(size_t)(i - 1) * S];
      fm_mul(idx, inv, pre);
      if (PREFETCH && i > 1) pre = scr[(size_t)(i - 2) * S];
      const Fe gx = gsn.x(i);
      if constexpr (FUSED) fm_add_lazy(dx, gx, negCx); else fm_sub(dx, gx, C.x);
      fm_mul(inv, inv, dx);
    } else {
      idx = inv;
    }
    Fe u, s, x1, y1;
    const AffPt g = gsn.pt(i);
    if constexpr (FUSED) {
      // x = s^2 + nu, nu = -(C.x + GSn.x): the addend rides in the squaring's reduction
      // (fm_sqr_add), and s = (GSn.y + C.y)*dx^-1 takes a lazy sum (it only feeds a product).
      fm_sub(u, negCx, g.x);
      fm_add_lazy(s, g.y, C.y);
      fm_mul(s, s, idx);
      fm_sqr_add(x1, s, u);
      x_out<MODE>(A, x1);
      if (i < (int)kHalf - 1) {
        Fe x2;
        fm_sub(s, g.y, C.y);
        fm_mul(s, s, idx);
        fm_sqr_add(x2, s, u);
        x_out<MODE>(A, x2);
        if constexpr (is_scan(MODE))          // both x before either probe load is issued
          asm volatile("" ::"v"(x1.v[0]), "v"(x2.v[0]), "v"(x1.v[7]), "v"(x2.v[7]) : "memory");
        probe_pair<DUMP>(A, Q, x1, x2, job, j, kHalf - 1 - (uint32_t)i, kHalf + 1 + (uint32_t)i);
      } else {
        probe<DUMP>(A, Q, x1, job, j, kHalf - 1 - (uint32_t)i);
      }
      continue;
    }
    fm_add(u, C.x, g.x);                  // x = s^2 - (C.x + GSn.x)
    // C - GSn[i]: s = (-GSn.y - C.y)/dx; x needs only s^2, and with s' = -s = (GSn.y + C.y)/dx
    // y = (GSn.x - x)*s + GSn.y = (x - GSn.x)*s' + GSn.y   (keyhunt.cpp:2628-2641)
    fm_add(s, g.y, C.y);
    fm_mul(s, s, idx);
    fm_sqr(x1, s);
    fm_sub(x1, x1, u);
    x_out<MODE>(A, x1);
    if constexpr (needs_y(MODE)) {
      Fe t;
      fm_sub(t, x1, g.x);
      fm_mul(t, t, s);
      fm_canon(t, t);
      fm_add(y1, t, g.y);
    }
    if (i < (int)kHalf - 1) {
      // C + GSn[i]: s = (GSn.y - C.y)/dx; y = (GSn.x - x)*s - GSn.y   (keyhunt.cpp:2611-2624)
      Fe x2, y2;
      fm_sub(s, g.y, C.y);
      fm_mul(s, s, idx);
      fm_sqr(x2, s);
      fm_sub(x2, x2, u);
      x_out<MODE>(A, x2);
      if constexpr (MODE == kBaby) {
        baby_point(A, x1, job, j, kHalf - 1 - (uint32_t)i);
        baby_point(A, x2, job, j, kHalf + 1 + (uint32_t)i);
      } else if constexpr (is_addr(MODE)) {
        if constexpr (needs_y(MODE)) {
          fm_sub(y2, g.x, x2);
          fm_mul(y2, y2, s);
          fm_sub(y2, y2, g.y);
          fm_canon(y2, y2);
        }
        addr_point<MODE>(A, x1, y1, job, j, kHalf - 1 - (uint32_t)i);
        addr_point<MODE>(A, x2, y2, job, j, kHalf + 1 + (uint32_t)i);
      } else {
        if constexpr (MODE == kScan)                       // both x before either probe load is issued
          asm volatile("" ::"v"(x1.v[0]), "v"(x2.v[0]), "v"(x1.v[7]), "v"(x2.v[7]) : "memory");
        probe_pair<DUMP>(A, Q, x1, x2, job, j, kHalf - 1 - (uint32_t)i, kHalf + 1 + (uint32_t)i);
      }
    } else {
      if constexpr (MODE == kBaby)
        baby_point(A, x1, job, j, kHalf - 1 - (uint32_t)i);
      else if constexpr (is_addr(MODE))
        addr_point<MODE>(A, x1, y1, job, j, kHalf - 1 - (uint32_t)i);
      else
        probe<DUMP>(A, Q, x1, job, j, kHalf - 1 - (uint32_t)i);
    }
  }
  if constexpr (MODE == kBaby)
    baby_point(A, C.x, job, j, kHalf);
  else if constexpr (is_addr(MODE))
    addr_point<MODE>(A, C.x, C.y, job, j, kHalf);
  else
    probe<DUMP>(A, Q, C.x, job, j, kHalf);
}

// walk_group for kScanG (-m bsgs with a level-0 gate), the product path: same points, same order,
// with the fused x-only arithmetic (x = s^2 + nu), the prefix of step i-1 loaded right
// after step i's last use of the prefix register (its HBM latency hides behind a whole step), and
// each step's two x gate-tested together (gate_pair).  The first step is peeled and the prefix
// load is unconditional, so the loop body issues the same vector-memory sequence every time and
// the waitcnt pass waits for exactly the operand it needs.
template <int STAGES>
__device__ __forceinline__ void walk_group_g(const ScanArgs& A, ProbeQueue& Q, const AffPt& C, Fe inv,
                                             uint32_t job, uint32_t j, const Fe* scr) {
  const size_t S = A.stride;
  const GsnTable gsn{A.gsn};
  const uint32_t base = j * KHB_GROUP;
  // the centre enters as p - C.x and p - C.y, so every per-step add/sub is a lazy add
  Fe negCx, negCy;
  {
    Fe p;
#pragma unroll
    for (int k = 0; k < 8; ++k) p.v[k] = k == 0 ? KHB_P0 : (k == 1 ? KHB_P1 : 0xFFFFFFFFu);
    fm_sub(negCx, p, C.x);
    fm_sub(negCy, p, C.y);
  }
  Fe pre = scr_ld(scr + (size_t)(kHalf - 2) * S);
  Fe idx, dx, u, s, x1, x2;
  // step 511: pts[0] = C - GSn[511] only
  {
    fm_mul(idx, inv, pre);
    pre = scr_ld(scr + (size_t)(kHalf - 3) * S);
    fm_add_lazy(dx, gsn.x(kHalf - 1), negCx);
    fm_mul(inv, inv, dx);
    const AffPt g = gsn.pt(kHalf - 1);
    fm_add_lazy(u, gsn.nx(kHalf - 1), negCx);
    fm_add_lazy(s, g.y, C.y);
    fm_mul(s, s, idx);
    fm_sqr_add(x1, s, u);
    x_out<kScanG>(A, x1);
    gate_pair<STAGES>(A, Q, x1, base, false, x1, 0, job);
  }
  for (int i = (int)kHalf - 2; i >= 0; --i) {
    if (i > 0) {
      fm_mul(idx, inv, pre);
      pre = scr_ld(scr + (size_t)(i >= 2 ? i - 2 : 0) * S);   // i = 1: a harmless reload of prefix 0
      fm_add_lazy(dx, gsn.x(i), negCx);
      fm_mul(inv, inv, dx);
    } else {
      idx = inv;
    }
    const AffPt g = gsn.pt(i);
    fm_add_lazy(u, gsn.nx(i), negCx);         // nu = -(C.x + GSn.x)
    // C - GSn[i] (pts[511 - i]) and C + GSn[i] (pts[513 + i])
    fm_add_lazy(s, g.y, C.y);
    fm_mul(s, s, idx);
    fm_sqr_add(x1, s, u);
    x_out<kScanG>(A, x1);
    fm_add_lazy(s, g.y, negCy);               // GSn.y - C.y
    fm_mul(s, s, idx);
    fm_sqr_add(x2, s, u);
    x_out<kScanG>(A, x2);
    gate_pair<STAGES>(A, Q, x1, base + kHalf - 1 - (uint32_t)i, true, x2, base + kHalf + 1 + (uint32_t)i, job);
  }
  probe<false>(A, Q, C.x, job, j, kHalf);        // the centre, pts[512]
}

// The half prefix stream (KHB_HALF_STREAM): walk_group_g over a forward pass that stored only the odd prefixes
// P_1, P_3, ..., P_509 (P_i = prod_{k<=i} dx_k).  After the peeled step 511 the walk goes in pairs (even i, odd
// i - 1): the even step needs P_{i-1}, stored, and then loads P_{i-3}; the odd step rebuilds P_{i-2} =
// P_{i-3} * dx_{i-2} (one extra product per pair).  Same points, same order and bit-identical x: P_{i-2} is the
// forward pass's own product of the same operands in the same order.  Half the stream's HBM bytes (16 B per
// giant step instead of 32) for +4.3 % VALU.
template <int STAGES>
__device__ __forceinline__ void half_points(const ScanArgs& A, ProbeQueue& Q, const AffPt& C, const Fe& negCx,
                                            const Fe& negCy, const Fe& idx, int i, uint32_t base, uint32_t job) {
  const GsnTable gsn{A.gsn};
  Fe u, s, x1, x2;
  const AffPt g = gsn.pt(i);
  fm_add_lazy(u, gsn.nx(i), negCx);             // nu = -(C.x + GSn.x)
  fm_add_lazy(s, g.y, C.y);
  fm_mul(s, s, idx);
  fm_sqr_add(x1, s, u);
  x_out<kScanG>(A, x1);
  fm_add_lazy(s, g.y, negCy);
  fm_mul(s, s, idx);
  fm_sqr_add(x2, s, u);
  x_out<kScanG>(A, x2);
  gate_pair<STAGES>(A, Q, x1, base + kHalf - 1 - (uint32_t)i, true, x2, base + kHalf + 1 + (uint32_t)i, job);
}

template <int STAGES>
__device__ __forceinline__ void walk_group_g_half(const ScanArgs& A, ProbeQueue& Q, const AffPt& C, Fe inv,
                                                  uint32_t job, uint32_t j, const Fe* scr) {
  const size_t S = A.stride;
  const GsnTable gsn{A.gsn};
  const uint32_t base = j * KHB_GROUP;
  Fe negCx, negCy;
  {
    Fe p;
#pragma unroll
    for (int k = 0; k < 8; ++k) p.v[k] = k == 0 ? KHB_P0 : (k == 1 ? KHB_P1 : 0xFFFFFFFFu);
    fm_sub(negCx, p, C.x);
    fm_sub(negCy, p, C.y);
  }
  Fe pre = scr_ld(scr + (size_t)(kHalf - 3) * S);          // P_509
  Fe idx, dx;
  // odd step 511: pts[0] = C - GSn[511] only
  {
    Fe u, s, x1;
    fm_add_lazy(dx, gsn.x(kHalf - 2), negCx);
    fm_mul(idx, pre, dx);                                  // P_510 = P_509 * dx_510
    fm_mul(idx, inv, idx);
    fm_add_lazy(dx, gsn.x(kHalf - 1), negCx);
    fm_mul(inv, inv, dx);
    const AffPt g = gsn.pt(kHalf - 1);
    fm_add_lazy(u, gsn.nx(kHalf - 1), negCx);
    fm_add_lazy(s, g.y, C.y);
    fm_mul(s, s, idx);
    fm_sqr_add(x1, s, u);
    x_out<kScanG>(A, x1);
    gate_pair<STAGES>(A, Q, x1, base, false, x1, 0, job);
  }
  // pairs (even i, odd i - 1), i = 510 ... 2; pre = P_{i-1} on entry
  for (int i = (int)kHalf - 2; i >= 2; i -= 2) {
    fm_mul(idx, inv, pre);                                 // even step i: P_{i-1} (odd index, stored)
    if (i > 2) pre = scr_ld(scr + (size_t)(i - 3) * S);    // P_{i-3} for step i - 1 (and i - 2)
    fm_add_lazy(dx, gsn.x(i), negCx);
    fm_mul(inv, inv, dx);
    half_points<STAGES>(A, Q, C, negCx, negCy, idx, i, base, job);
    // odd step i - 1: P_{i-2} = P_{i-3} * dx_{i-2} (i - 1 = 1: P_0 = dx_0)
    fm_add_lazy(dx, gsn.x(i - 2), negCx);
    if (i > 2) {
      fm_mul(idx, pre, dx);
      fm_mul(idx, inv, idx);
    } else {
      fm_mul(idx, inv, dx);
    }
    fm_add_lazy(dx, gsn.x(i - 1), negCx);
    fm_mul(inv, inv, dx);
    half_points<STAGES>(A, Q, C, negCx, negCy, idx, i - 1, base, job);
  }
  half_points<STAGES>(A, Q, C, negCx, negCy, inv, 0, base, job);     // step 0: idx = inv
  probe<false>(A, Q, C.x, job, j, kHalf);
}

// One reference group centred on C, walked on its own (-m address, baby steps): the 513-element
// batch of IntGroup.cpp:36-58 including dx[512] = _2GSn.x - C.x, whose inverse advances C to the
// next centre (keyhunt.cpp:3986-3999).  For -m address this is keyhunt.cpp:2586-2711 with the
// table Gn (same point order t = 0..1023, pts[t] = key + t), plus y where the search needs it.
template <int MODE>
__device__ __forceinline__ void scan_group(const ScanArgs& A, ProbeQueue& Q, AffPt& C, uint32_t job, uint32_t j,
                                           Fe* scr) {
  const uint32_t S = A.stride;
  // GSn rows are wave-uniform: read them through the constant address space so they arrive by
  // scalar loads (SGPRs, lgkmcnt) instead of occupying 16 VGPRs and the vector-memory queue.
  const GsnTable gsn{A.gsn};
  Fe acc, dx;
  // forward pass: prefix products of dx[i] = GSn[i].x - C.x (i < 512) and _2GSn.x - C.x
  {
    const Fe gx = gsn.x(0);
    fm_sub(acc, gx, C.x);
  }
  scr[0] = acc;
  for (uint32_t i = 1; i < kHalf; ++i) {
    const Fe gx = gsn.x(i);
    fm_sub(dx, gx, C.x);
    fm_mul(acc, acc, dx);
    scr[(size_t)i * S] = acc;
  }
  {
    const Fe gx = gsn.x(kHalf);
    fm_sub(dx, gx, C.x);
  }
  fm_mul(acc, acc, dx);
  Fe accc;
  fm_canon(accc, acc);
  const bool degenerate = fe_is_zero(accc);
  Fe inv;
  fm_inv(inv, acc);                       // == 0 (mod p) when degenerate -> every inverse 0, as the reference
  {
    // i = 512's inverse is only needed for the next centre: park it in prefix slot 511, which
    // is read exactly once (here), instead of holding 8 VGPRs through the backward loop.
    Fe inv2;
    const Fe pre = scr[(size_t)(kHalf - 1) * S];
    fm_mul(inv2, inv, pre);
    scr[(size_t)(kHalf - 1) * S] = inv2;
    asm volatile("" ::: "memory");
  }
  fm_mul(inv, inv, dx);
  walk_group<MODE>(A, Q, C, inv, job, j, scr);
  // next centre: C + _2GSn with y (keyhunt.cpp:3986-3999)
  {
    asm volatile("" ::: "memory");
    const Fe inv2 = scr[(size_t)(kHalf - 1) * S];
    const AffPt g2 = gsn.pt(kHalf);
    Fe s, nx, ny;
    fm_sub(s, g2.y, C.y);
    fm_mul(s, s, inv2);
    fm_sqr(nx, s);
    fm_sub(nx, nx, C.x);
    fm_sub(nx, nx, g2.x);
    fm_canon(nx, nx);
    fm_sub(ny, g2.x, nx);
    fm_mul(ny, ny, s);
    fm_sub(ny, ny, g2.y);
    fm_canon(ny, ny);
    C.x = nx;
    C.y = ny;
  }
  if (!is_dump(MODE) && degenerate) {
    uint32_t k = atomicAdd(&A.counters[1], 1u);
    if (k < A.degen_cap) A.degen[k] = khb_degenerate{job, j};
  }
}

// AddDirect (SECP256K1.cpp:242-265) with its own inversion; used once per lane.
__device__ __forceinline__ bool add_direct(AffPt& r, const AffPt& p1, const AffPt& p2) {
  Fe dy, dx, s, x, y;
  fm_sub(dy, p2.y, p1.y);
  fm_sub(dx, p2.x, p1.x);
  const bool degenerate = fe_is_zero(dx);
  fm_inv(dx, dx);
  fm_mul(s, dy, dx);
  fm_sqr(x, s);
  fm_sub(x, x, p1.x);
  fm_sub(x, x, p2.x);
  fm_canon(x, x);
  fm_sub(y, p2.x, x);
  fm_mul(y, y, s);
  fm_sub(y, y, p2.y);
  fm_canon(y, y);
  r.x = x;
  r.y = y;
  return degenerate;
}

__device__ __forceinline__ Fe fe_small(uint32_t v) {
  Fe r;
#pragma unroll
  for (int k = 0; k < 8; ++k) r.v[k] = k ? 0u : v;
  return r;
}

// -m bsgs work item: groups [g0, g1) (at most kBatch) of one job with TWO field inversions in
// total instead of one per group plus one per lane start:
//  0. centres C_g = startP + gofs[g0+g] (gofs[j] = j*_2GSn), all from startP, batch-inverted
//     together (Montgomery over the <= kBatch x-differences; AddDirect, SECP256K1.cpp:242-265);
//  1. per group the forward prefix products of dx_i = GSn[i].x - C.x, i < 512, into scratch;
//     the group totals T_g are chained into one product;
//  2. one inversion of that product, split back into inv(T_g) (Montgomery again);
//  3. per group the reference's backward walk (walk_group).
// The reference's batch per group also holds dx[512] = _2GSn.x - C.x (the next-centre add); its
// inverse is not needed here (centres come from step 0), but a group whose 513-element product is
// zero gets all-zero inverses in the reference (IntGroup.cpp:36-58 + IntMod.cpp:497-500): such a
// group is kept out of the chained product and walked with inv = 0, which reproduces its x values
// bit for bit (and is reported, as scan_group does).
// Scratch (lane-private, stride = lanes, 32 B entries): g*512 + i (i < 511) prefixes of group g,
// g*512 + 511 = T_g then inv(T_g); kBatch*512 + 2g (+1) = C_g.x (.y); kBatch*514 + g = chained
// products.
template <int MODE>
__device__ __forceinline__ uint32_t scan_batch(const ScanArgs& A, ProbeQueue& Q, uint32_t job, uint32_t g0,
                                               uint32_t g1, Fe* scr) {
  const size_t S = A.stride;
  const GsnTable gsn{A.gsn};
  const uint32_t nb = g1 - g0;
  Fe* const sc = scr + (size_t)kBatch * kHalf * S;          // centres
  Fe* const sq = scr + (size_t)kBatch * (kHalf + 2) * S;    // chained products
  const AffPt P = A.centres[job];
  // 0. centres
  uint32_t skip = 0;      // bit g: no add (group 0 is startP) or a degenerate add (gofs.x == P.x)
  Fe acc;
  for (uint32_t g = 0; g < nb; ++g) {
    const uint32_t jg = g0 + g;
    Fe d = fe_small(1);
    if (jg != 0) {
      fm_sub(d, A.gofs[jg].x, P.x);
      Fe dc;
      fm_canon(dc, d);
      if (fe_is_zero(dc)) {
        d = fe_small(1);
        skip |= 1u << g;
        if (MODE != kDump) {
          const uint32_t k = atomicAdd(&A.counters[1], 1u);
          if (k < A.degen_cap) A.degen[k] = khb_degenerate{job, jg | 0x80000000u};
        }
      }
    } else {
      skip |= 1u << g;
    }
    if (g == 0) acc = d; else fm_mul(acc, acc, d);
    sq[g * S] = acc;
  }
  Fe inv;
  fm_inv(inv, acc);
  for (int g = (int)nb - 1; g >= 0; --g) {
    const uint32_t jg = g0 + (uint32_t)g;
    const AffPt O = A.gofs[jg];
    Fe ig;
    if (g > 0) {
      fm_mul(ig, inv, sq[(g - 1) * S]);
      Fe d = fe_small(1);
      if (!((skip >> g) & 1u)) fm_sub(d, O.x, P.x);
      fm_mul(inv, inv, d);
    } else {
      ig = inv;
    }
    AffPt C = P;
    if (jg != 0) {
      if ((skip >> g) & 1u) ig = fe_small(0);      // as add_direct: inverse of 0 is 0
      Fe s, x, y;
      fm_sub(s, O.y, P.y);
      fm_mul(s, s, ig);
      fm_sqr(x, s);
      fm_sub(x, x, P.x);
      fm_sub(x, x, O.x);
      fm_canon(x, x);
      fm_sub(y, O.x, x);
      fm_mul(y, y, s);
      fm_sub(y, y, O.y);
      fm_canon(y, y);
      C.x = x;
      C.y = y;
    }
    sc[2 * g * S] = C.x;
    sc[(2 * g + 1) * S] = C.y;
  }
  // 1. forward passes
  const Fe g2x = gsn.x(kHalf);
  uint32_t degen = 0;
  for (uint32_t g = 0; g < nb; ++g) {
    Fe* const sg = scr + (size_t)g * kHalf * S;
    const Fe cx = sc[2 * g * S];
    Fe a, dx, negCx;
    {
      Fe p;
#pragma unroll
      for (int k = 0; k < 8; ++k) p.v[k] = k == 0 ? KHB_P0 : (k == 1 ? KHB_P1 : 0xFFFFFFFFu);
      fm_sub(negCx, p, cx);
    }
    // dx_i = GSn[i].x - C.x as the lazy sum GSn[i].x + (p - C.x) (congruent; feeds products only)
    fm_add_lazy(a, gsn.x(0), negCx);
    if (!(kHalfStream && is_gated(MODE))) scr_st(sg, a);       // P_0 is not stored by the half stream
    for (uint32_t i = 1; i < kHalf - 1; ++i) {
      fm_add_lazy(dx, gsn.x(i), negCx);
      fm_mul(a, a, dx);
      if (!(kHalfStream && is_gated(MODE)) || (i & 1u)) scr_st(sg + i * S, a);
    }
    fm_add_lazy(dx, gsn.x(kHalf - 1), negCx);
    fm_mul(a, a, dx);
    Fe ac;
    fm_canon(ac, a);
    if (fe_is_zero(ac) || fe_eq(g2x, cx)) {
      degen |= 1u << g;
      a = fe_small(1);
    }
    sg[(kHalf - 1) * S] = a;
    if (g == 0) acc = a; else fm_mul(acc, acc, a);
    sq[g * S] = acc;
  }
  // 2. one inversion for the batch
  fm_inv(inv, acc);
  for (int g = (int)nb - 1; g >= 0; --g) {
    Fe* const sg = scr + (size_t)g * kHalf * S;
    Fe ig;
    if (g > 0) {
      fm_mul(ig, inv, sq[(g - 1) * S]);
      fm_mul(inv, inv, sg[(kHalf - 1) * S]);
    } else {
      ig = inv;
    }
    if ((degen >> g) & 1u) ig = fe_small(0);
    sg[(kHalf - 1) * S] = ig;
  }
  // 3. backward walks
  uint32_t walked = 0;
  for (uint32_t g = 0; g < nb; ++g, ++walked) {
    Fe* const sg = scr + (size_t)g * kHalf * S;
    asm volatile("" ::: "memory");
    const AffPt C{sc[2 * g * S], sc[(2 * g + 1) * S]};
    if constexpr (is_gated(MODE) && kHalfStream)
      walk_group_g_half<gate_stages(MODE)>(A, Q, C, sg[(kHalf - 1) * S], job, g0 + g, sg);
    else if constexpr (is_gated(MODE))
      walk_group_g<gate_stages(MODE)>(A, Q, C, sg[(kHalf - 1) * S], job, g0 + g, sg);
    else
      walk_group<MODE>(A, Q, C, sg[(kHalf - 1) * S], job, g0 + g, sg);
    if (MODE != kDump && ((degen >> g) & 1u)) {
      const uint32_t k = atomicAdd(&A.counters[1], 1u);
      if (k < A.degen_cap) A.degen[k] = khb_degenerate{job, g0 + g};
    }
  }
  return walked;
}

// Groups walked by the launch: a wave sum of every lane's count, one 64-bit atomic per wave into
// counters[4..5].  The host compares it with n_jobs x group_count (khb_collect: KHB_EINCOMPLETE), so
// a work-item handout that skipped or repeated a group cannot go unnoticed.  Called with the wave
// reconverged (after the item loop).
__device__ __forceinline__ void count_walked(uint32_t* counters, uint32_t walked) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) walked += __shfl_xor(walked, o);
  if ((threadIdx.x & 63u) == 0 && walked)
    atomicAdd(reinterpret_cast<unsigned long long*>(counters + 4), (unsigned long long)walked);
}

// Shader clock over the launch: the first wave of block 0 samples s_memtime (shader clock) and
// s_memrealtime (100 MHz) when it starts and when it leaves (it takes work items until the launch's
// queue is empty, so it spans the launch); the host turns the two deltas into MHz (khb_stats.shader_mhz).
// The samples are stored with ordinary (vector) global stores by one lane.
__device__ __forceinline__ void clock_probe(uint32_t* counters, int at) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const uint64_t t = __builtin_amdgcn_s_memtime(), r = __builtin_amdgcn_s_memrealtime();
    uint64_t* c = reinterpret_cast<uint64_t*>(counters + 8) + 2 * at;
    // agent-scope (write-through) vector stores: launch_epilogue's last wave may run on another XCD
    __hip_atomic_store(c, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(c + 1, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// End of a launch without copy kernels (round 5): every wave releases its counter updates and adds one to
// counters[3]; the wave whose add is the launch's last reads the counters memory-side (agent-scope atomics,
// coherent across the XCDs' L2s), writes them to the slot's pinned host block with vector stores and zeroes
// counters[0..7] for the slot's next launch.  With the candidate / degenerate rings and the centres in
// pinned host memory as well, a khb_submit stream holds only this kernel and its two events: no memset
// before it and no device-to-host blit after it, which had waited for CU slots behind the other slot's
// persistent scan.  khb_collect checks host counters[3] == total_waves.
__device__ __forceinline__ void launch_epilogue(const ScanArgs& A) {
  if (!A.host_counters) return;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");     // this wave's atomics and probe stores have landed
  uint32_t prev = 0;
  if ((threadIdx.x & 63u) == 0)
    prev = __hip_atomic_fetch_add(&A.counters[3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  prev = __shfl(prev, 0);
  if (prev != A.total_waves - 1) return;
  const uint32_t l = threadIdx.x & 63u;
  if (l < 16) {
    const uint32_t v = l < 8 ? __hip_atomic_exchange(&A.counters[l], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : __hip_atomic_fetch_add(&A.counters[l], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    A.host_counters[l] = v;
  }
  // the launch's end on the shader clock and the 100 MHz clock ([16..19]): with block 0's start sample on the
  // 100 MHz clock ([10..11]; s_memrealtime is one clock for the device, s_memtime one per XCD) the host gets
  // the launch's execution span, which the events cannot give while the other slot's launch still holds the
  // CUs the queued kernel waits for (khb_stats.kernel_ms)
  const uint64_t t = __builtin_amdgcn_s_memtime(), r = __builtin_amdgcn_s_memrealtime();
  if (l < 4) A.host_counters[16 + l] = (uint32_t)((l < 2 ? t : r) >> (32 * (l & 1u)));
  __threadfence_system();
}

template <int MODE>
__global__ __launch_bounds__(kBlock, waves_per_simd(MODE)) void k_giant_scan(ScanArgs A) {
  clock_probe(A.counters, 0);
  constexpr bool QUEUE = is_scan(MODE);
  constexpr bool BATCH = is_scan(MODE) || MODE == kDump;
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  Fe* scr = A.scratch + lane;
  __shared__ uint32_t s_queue[QUEUE ? kWavesPerBlock : 1][QUEUE ? kQWords * kQCap : 1];
  __shared__ uint32_t s_count[kWavesPerBlock];
  const uint32_t wave = QUEUE ? threadIdx.x >> 6 : 0;
  ProbeQueue Q{s_queue[wave], (volatile __attribute__((address_space(3))) uint32_t*)&s_count[wave]};
  if (QUEUE) *Q.n = 0;
  uint32_t walked = 0;     // groups this lane walked (count_walked: the host checks the launch's total)
  if constexpr (BATCH) {
    // Dynamic work items: each wave takes the next 64 items from a launch-wide counter
    // (counters[2], zeroed per launch), so a wave that runs ahead keeps taking work and every SIMD
    // stays 4 waves deep until the queue is empty; a static lane-strided split left the launch's
    // tail to its slowest waves.  Each lane keeps its own scratch column (scr) for every item.
    const uint32_t wl = threadIdx.x & 63u;
    for (;;) {
      uint32_t b = 0;
      if (wl == 0) b = atomicAdd(&A.counters[2], 64u);
      b = __builtin_amdgcn_readfirstlane(b);
      if (b >= A.n_items) break;
      const uint64_t item = (uint64_t)b + wl;
      if (item < A.n_items) {
        const uint32_t job = (uint32_t)(item / A.lanes_per_job);
        const uint32_t m = (uint32_t)(item % A.lanes_per_job);
        const uint32_t g0 = A.group_begin + m * kBatch;
        const uint32_t g1 = min(g0 + kBatch, A.group_end);
        walked += scan_batch<MODE>(A, Q, job, g0, g1, scr);
      }
    }
  } else {
    // dynamic per-wave items, as above (counters[2])
    const uint32_t wl = threadIdx.x & 63u;
    for (;;) {
      uint32_t b = 0;
      if (wl == 0) b = atomicAdd(&A.counters[2], 64u);
      b = __builtin_amdgcn_readfirstlane(b);
      if (b >= A.n_items) break;
      const uint64_t item = (uint64_t)b + wl;
      if (item >= A.n_items) continue;
      const uint32_t job = (uint32_t)(item / A.lanes_per_job);
      const uint32_t m = (uint32_t)(item % A.lanes_per_job);
      const uint32_t g0 = A.group_begin + m * A.gpl;
      const uint32_t g1 = min(g0 + A.gpl, A.group_end);
      AffPt C = A.centres[job];
      const uint32_t mo = g0 / A.gpl;
      if (mo != 0) {
        if (add_direct(C, C, A.offs[mo]) && !is_dump(MODE)) {
          uint32_t k = atomicAdd(&A.counters[1], 1u);
          if (k < A.degen_cap) A.degen[k] = khb_degenerate{job, g0 | 0x80000000u};
        }
      }
      for (uint32_t j = g0; j < g1; ++j, ++walked) scan_group<MODE>(A, Q, C, job, j, scr);
    }
  }
  if (QUEUE) q_drain(A, Q, 1);   // the wave has reconverged: finish what is still queued
  count_walked(A.counters, walked);
  clock_probe(A.counters, 1);
  launch_epilogue(A);
}

// Launchers of the k_giant_scan instances (one translation unit each, see above).
void launch_bsgs(int mode, uint32_t blocks, hipStream_t stream, const ScanArgs& A);   // kScan, kScanG, kScanG1, kScanG2, kDump
void launch_addr(int mode, uint32_t blocks, hipStream_t stream, const ScanArgs& A);   // kAddrU, kAddrC, kAddrB, kAddrDump
void launch_addr_e(int mode, uint32_t blocks, hipStream_t stream, const ScanArgs& A);  // kAddrUE, kAddrCE, kAddrBE
void launch_baby(uint32_t blocks, hipStream_t stream, const ScanArgs& A);             // kBaby

}  // namespace khbk
