// libkhbsgs.so — MI355X (gfx950) BSGS giant-step engine behind the C ABI of include/khbsgs.h.
//
// Hot path replaced: keyhunt.cpp:3867-4004 (thread_process_bsgs group loop + level-1 bloom probe).
//
// Work decomposition:
//   job   = one (chunk, target) pair; the host supplies its group-0 centre startP.
//   lane  = one work item = `groups_per_lane` consecutive 1024-point groups of one job.  The lane
//           derives its first centre as startP + offs[m] (one affine add), then walks its groups
//           exactly as the reference walks a chunk: per group a 513-element Montgomery batch
//           inverse (prefix products spilled to a lane-private HBM scratch, coalesced across the
//           wave), 1023 x-only affine additions, 1024 bloom probes, and the next-centre add.
//   grid  = persistent: `lanes` work lanes stride over n_jobs * lanes_per_job items.
// One lane's group maps 1:1 onto one reference group, so a collapsed batch inverse (dx == 0)
// reproduces the reference's all-zero inverses exactly (IntGroup.cpp:36-58 + IntMod.cpp:497-500).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <new>
#include <vector>
#include "../../include/khbsgs.h"
#include "device/fe.hpp"
#include "device/fe_asm.hpp"
#include "device/bloom_probe.hpp"
#include "device/hash160.hpp"

using namespace khb;

namespace {

struct AffPt {
  Fe x, y;
};

#ifndef KHB_PROBE_MODE
#define KHB_PROBE_MODE 0          // 0 = product; 1..3 = perf experiments (tools/perf_variants.py)
#endif
#ifndef KHB_PROBE_BITS
#define KHB_PROBE_BITS 1          // bloom bits per round trip in the drain (2 and 4 measured slower)
#endif
#ifndef KHB_GSN_SCALAR
#define KHB_GSN_SCALAR 1          // GSn table through scalar loads
#endif
#ifndef KHB_PIPE
#define KHB_PIPE 1                // walk_group software pipelining (bit 0 prefix prefetch, bit 1 paired gate loads)
#endif
#ifndef KHB_LDSCOUNT
#define KHB_LDSCOUNT 1            // probe-queue count through an LDS-typed pointer (ds_* not flat_*)
#endif
#ifndef KHB_NT
#define KHB_NT 0                  // prefix scratch through non-temporal loads/stores
#endif
#ifndef KHB_FUSE
#define KHB_FUSE 1                // -m bsgs walk: x = s^2 + nu fused into the squaring's reduction
#endif
#ifndef KHB_GATE1
#define KHB_GATE1 25              // default log2 bytes of the stage-1 fold of a larger level-0 gate (0 = none)
#endif
#ifndef KHB_DYN
#define KHB_DYN 1                 // scan_batch kernels: dynamic per-wave work items (launch counter)
#endif
#ifndef KHB_WAVES_PER_SIMD
#define KHB_WAVES_PER_SIMD 4      // occupancy target of k_giant_scan (launch bounds); w4 measured best
#endif
constexpr uint32_t kBlock = 256;
#ifndef KHB_BATCH
#define KHB_BATCH 8               // -m bsgs groups per work item (scan_batch): two inversions per item
#endif
constexpr uint32_t kBatch = KHB_BATCH;

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
  kScanG1 = 8,     // kScanG with the gate's stage-1 fold in front (khb_set_gate_stage1; k >= 4)
};
constexpr bool is_gated(int m) { return m == kScanG || m == kScanG1; }
constexpr bool is_scan(int m) { return m == kScan || is_gated(m); }
constexpr bool is_addr(int m) { return m >= kAddrU && m <= kAddrDump; }
constexpr bool needs_y(int m) { return m == kAddrU || m == kAddrB || m == kAddrDump; }
constexpr bool is_dump(int m) { return m == kDump || m == kAddrDump || m == kBaby; }
constexpr uint32_t kHalf = KHB_GROUP / 2;            // 512
constexpr uint32_t kCandCap = 1u << 20;
constexpr uint32_t kAddrHitCap = 1u << 18;
constexpr uint32_t kDegenCap = 4096;
constexpr size_t kCounterBytes = 32;                 // ScanArgs::counters

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// Prefix-scratch stream (written once by the forward pass, read once by the walk): with
// KHB_NT the accesses are non-temporal, so the stream does not evict the level-0 gate from L2.
__device__ __forceinline__ void scr_st(Fe* p, const Fe& v) {
#if KHB_NT
  v4u* q = reinterpret_cast<v4u*>(p);
  __builtin_nontemporal_store(v4u{v.v[0], v.v[1], v.v[2], v.v[3]}, q);
  __builtin_nontemporal_store(v4u{v.v[4], v.v[5], v.v[6], v.v[7]}, q + 1);
#else
  *p = v;
#endif
}
__device__ __forceinline__ Fe scr_ld(const Fe* p) {
#if KHB_NT
  const v4u* q = reinterpret_cast<const v4u*>(p);
  const v4u a = __builtin_nontemporal_load(q), b = __builtin_nontemporal_load(q + 1);
  return Fe{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}};
#else
  return *p;
#endif
}

struct ScanArgs {
  const uint8_t* __restrict__ bloom;
  BloomGeom geom;
  const AffPt* __restrict__ gsn;       // [0..511] GSn, [512] _2GSn
  const AffPt* __restrict__ offs;      // lane start offsets
  const AffPt* __restrict__ gofs;      // per-group centre offsets j*_2GSn (scan_batch)
  const AffPt* __restrict__ centres;   // per-job group-0 centre
  Fe* __restrict__ scratch;            // prefix products [512][lanes]
  khb_cand* __restrict__ cand;
  khb_degenerate* __restrict__ degen;
  uint32_t* __restrict__ counters;     // [0] candidates [1] degenerate groups [2] work-item cursor (KHB_DYN)
                                       // [4..5] groups walked (u64, count_walked)
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
  // block x.v[0] & gate_mask and bits (x.v[1] >> 6p) & 63, p < gate_probes, in it, all set for
  // every x of the L1 set; null = no gate.  kBaby writes it (gate_w, ic < glimit).
  const uint8_t* __restrict__ gate;
  uint32_t* __restrict__ gate_w;
  uint32_t gate_probes;
  uint64_t glimit;
  uint32_t gate_mask;                  // blocks - 1
  // stage-1 gate (khb_set_gate_stage1): the level-0 gate OR-folded to (gate1_mask + 1) blocks, block i of
  // the fold = OR of blocks j of the gate with j & gate1_mask == i; null = no stage 1
  const uint8_t* __restrict__ gate1;
  uint32_t gate1_mask;
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
#if KHB_LDSCOUNT
  volatile __attribute__((address_space(3))) uint32_t* n;
#else
  volatile uint32_t* n;
#endif
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
      if (bloom_full<KHB_PROBE_BITS>(sub_bloom(A.bloom, A.geom, x), A.geom, w, xxh64_32(w, KHB_BLOOM_SEED)))
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

// The gate's bit positions in x's block: (x.v[1] >> 6p) & 63 for p < probes, packed 6 bits each
// into three slots (unused probes repeat the last used one, so every test checks three bits).
__device__ __forceinline__ uint32_t gate_bits(const ScanArgs& A, const Fe& x) {
  const uint32_t w = x.v[1];
  const uint32_t b0 = w & 63u, b1 = A.gate_probes > 1 ? (w >> 6) & 63u : b0;
  const uint32_t b2 = A.gate_probes > 2 ? (w >> 12) & 63u : b1;
  return b0 | (b1 << 6) | (b2 << 12);
}

// All three packed bits set in the 64-bit block (lo, hi)?
__device__ __forceinline__ bool gate_block_pass(uint32_t lo, uint32_t hi, uint32_t bits) {
  uint32_t r = 1u;
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    const uint32_t b = (bits >> (6 * p)) & 63u;
    r &= ((b & 32u) ? hi : lo) >> (b & 31u);
  }
  return r & 1u;
}

// A gate test: x's 64-bit block of the map (one 8-byte load: a single cache line per x whatever
// the probe count) and the packed bit positions.
struct GatePend {
  uint32_t lo, hi, bits;
  __device__ __forceinline__ bool pass() const { return gate_block_pass(lo, hi, bits); }
};

#ifndef KHB_GATE_NT
#define KHB_GATE_NT 0             // 1 = gate blocks through non-temporal loads (experiment)
#endif
__device__ __forceinline__ GatePend gate_issue(const ScanArgs& A, const Fe& x) {
#if KHB_GATE_NT
  const uint64_t v = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(A.gate) + (x.v[0] & A.gate_mask));
  const uint2 w = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
#else
  const uint2 w = reinterpret_cast<const uint2*>(A.gate)[x.v[0] & A.gate_mask];
#endif
  return GatePend{w.x, w.y, gate_bits(A, x)};
}

// kScanG: gate test of one walk step's two x (x2 absent at step 511: has2 = false, uniform).  Both
// blocks are loaded before either is waited for; survivors (~0.04 % of x) go to the queue.
template <bool STAGE1>
__device__ __forceinline__ void gate_pair(const ScanArgs& A, ProbeQueue& Q, const Fe& x1, uint32_t step1, bool has2,
                                          const Fe& x2, uint32_t step2, uint32_t job) {
  bool h1, h2;
  if constexpr (STAGE1) {
    // stage 1 (L2-resident fold); the full gate's line is fetched only for its survivors
    const uint32_t b1 = gate_bits(A, x1), b2 = gate_bits(A, x2);
    const uint2 f1 = reinterpret_cast<const uint2*>(A.gate1)[x1.v[0] & A.gate1_mask];
    const uint2 f2 = reinterpret_cast<const uint2*>(A.gate1)[x2.v[0] & A.gate1_mask];
    const bool s1 = gate_block_pass(f1.x, f1.y, b1), s2 = has2 && gate_block_pass(f2.x, f2.y, b2);
    if (__ballot(s1 || s2) == 0) return;
    uint2 w1 = make_uint2(0u, 0u), w2 = make_uint2(0u, 0u);
    if (s1) w1 = reinterpret_cast<const uint2*>(A.gate)[x1.v[0] & A.gate_mask];
    if (s2) w2 = reinterpret_cast<const uint2*>(A.gate)[x2.v[0] & A.gate_mask];
    h1 = s1 && gate_block_pass(w1.x, w1.y, b1);
    h2 = s2 && gate_block_pass(w2.x, w2.y, b2);
  } else {
    const GatePend q1 = gate_issue(A, x1), q2 = gate_issue(A, x2);
    h1 = q1.pass();
    h2 = has2 && q2.pass();
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
    const uint2 w = reinterpret_cast<const uint2*>(A.gate)[x.v[0] & A.gate_mask];
    return gate_block_pass(w.x, w.y, gate_bits(A, x));
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
#if KHB_PROBE_MODE == 0
    uint64_t a;
    const bool hit = first_bit(A, x, a);
    q_push(Q, hit, x, job, j * KHB_GROUP + t);
    q_drain(A, Q, kDrainAt);
#elif KHB_PROBE_MODE == 1      // perf experiment: first hash only, no bloom access
    uint64_t w[4];
    x_words(w, x);
    if (xxh64_32(w, KHB_BLOOM_SEED) == 0x0123456789abcdefull) emit_cand(A, job, j * KHB_GROUP + t);
#elif KHB_PROBE_MODE == 2      // perf experiment: first hash + first bit only
    uint64_t w[4];
    x_words(w, x);
    const uint64_t a = xxh64_32(w, KHB_BLOOM_SEED);
    const uint8_t* bf = sub_bloom(A.bloom, A.geom, x);
    const uint64_t pos = mod_bits(a, A.geom);
    if ((bf[pos >> 3] >> (pos & 7)) & 1u & (a == 0x0123456789abcdefull)) emit_cand(A, job, j * KHB_GROUP + t);
#elif KHB_PROBE_MODE == 4      // perf experiment: first hash + one random bit of a 4 MiB table
    uint64_t w[4];
    x_words(w, x);
    const uint64_t a = xxh64_32(w, KHB_BLOOM_SEED);
    const uint8_t byte = A.bloom[a >> 42];
    if (((byte >> ((a >> 39) & 7)) & 1u) & (a == 0x0123456789abcdefull)) emit_cand(A, job, j * KHB_GROUP + t);
#elif KHB_PROBE_MODE == 5      // perf experiment: as 4 with a 2 MiB table
    uint64_t w[4];
    x_words(w, x);
    const uint64_t a = xxh64_32(w, KHB_BLOOM_SEED);
    const uint8_t byte = A.bloom[a >> 43];
    if (((byte >> ((a >> 40) & 7)) & 1u) & (a == 0x0123456789abcdefull)) emit_cand(A, job, j * KHB_GROUP + t);
#else                          // perf experiment: no probe at all
    if (x.v[0] == 0x01234567u && x.v[1] == 0x89abcdefu) emit_cand(A, job, j * KHB_GROUP + t);
#endif
  }
}

// The two points of one backward step (C - GSn[i], C + GSn[i]): both first hashes are computed
// before either bloom bit is awaited, so the two loads share one memory round trip.
template <bool DUMP>
__device__ __forceinline__ void probe_pair(const ScanArgs& A, ProbeQueue& Q, const Fe& x1, const Fe& x2,
                                           uint32_t job, uint32_t j, uint32_t t1, uint32_t t2) {
#if KHB_PROBE_MODE == 0
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
#endif
  probe<DUMP>(A, Q, x1, job, j, t1);
  probe<DUMP>(A, Q, x2, job, j, t2);
}

// GSn / _2GSn rows (wave-uniform index).  With KHB_GSN_SCALAR the table is read through the
// constant address space, so rows arrive by scalar loads into SGPRs (lgkmcnt) instead of taking
// 16 VGPRs and four vector-memory slots per backward step.
struct GsnTable {
  const AffPt* p;
#if KHB_GSN_SCALAR
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
#else
  __device__ __forceinline__ Fe x(uint32_t i) const { return p[i].x; }
  __device__ __forceinline__ AffPt pt(uint32_t i) const { return p[i]; }
  __device__ __forceinline__ Fe nx(uint32_t i) const { return reinterpret_cast<const Fe*>(p + KHB_GIANT_TABLE)[i]; }
#endif
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
    for (uint32_t p = 0; p < A.gate_probes; ++p) {
      const uint32_t b = (x.v[1] >> (6 * p)) & 63u;
      atomicOr(A.gate_w + 2 * blk + (b >> 5), 1u << (b & 31));
    }
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
  // KHB_PIPE bit 0: the prefix for step i-1 is loaded during step i, so its HBM latency hides
  // behind a whole step's arithmetic instead of being waited for right after the load.
  constexpr bool PREFETCH = (KHB_PIPE & 1) && is_scan(MODE);
  // The load goes into `pre` itself right after its last use (no loop-carried copy: a copy at the
  // loop latch would make the wave wait for the load there).
  if (PREFETCH) pre = scr[(size_t)(kHalf - 2) * S];
  // KHB_FUSE (-m bsgs x-only walks): C.x is carried as negCx = p - C.x, so dx = GSn.x + negCx and
  // x = s^2 + (negCx - GSn.x) need no separate modular subtraction of the centre.
  constexpr bool FUSED = KHB_FUSE && (MODE == kScan || MODE == kDump);
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
        if constexpr ((KHB_PIPE & 2) && is_scan(MODE))
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
        if constexpr ((KHB_PIPE & 2) && MODE == kScan)   // both x before either gate load is issued
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
// with the fused x-only arithmetic (x = s^2 + nu, KHB_FUSE), the prefix of step i-1 loaded right
// after step i's last use of the prefix register (its HBM latency hides behind a whole step), and
// each step's two x gate-tested together (gate_pair).  The first step is peeled and the prefix
// load is unconditional, so the loop body issues the same vector-memory sequence every time and
// the waitcnt pass waits for exactly the operand it needs.
template <bool STAGE1>
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
    gate_pair<STAGE1>(A, Q, x1, base, false, x1, 0, job);
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
    gate_pair<STAGE1>(A, Q, x1, base + kHalf - 1 - (uint32_t)i, true, x2, base + kHalf + 1 + (uint32_t)i, job);
  }
  probe<false>(A, Q, C.x, job, j, kHalf);        // the centre, pts[512]
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
    scr_st(sg, a);
    for (uint32_t i = 1; i < kHalf - 1; ++i) {
      fm_add_lazy(dx, gsn.x(i), negCx);
      fm_mul(a, a, dx);
      scr_st(sg + i * S, a);
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
    if constexpr (is_gated(MODE))
      walk_group_g<MODE == kScanG1>(A, Q, C, sg[(kHalf - 1) * S], job, g0 + g, sg);
    else
      walk_group<MODE>(A, Q, C, sg[(kHalf - 1) * S], job, g0 + g, sg);
    if (MODE != kDump && ((degen >> g) & 1u)) {
      const uint32_t k = atomicAdd(&A.counters[1], 1u);
      if (k < A.degen_cap) A.degen[k] = khb_degenerate{job, g0 + g};
    }
  }
  return walked;
}

// Per-group centre offsets gofs[j] = j*_2GSn from lane offsets offs[m] = (m*gpl)*_2GSn:
// gofs[m*gpl + k] = offs[m] + k*_2GSn (gofs[0] is unused: group 0's centre is startP).
__global__ void k_expand_offsets(const AffPt* __restrict__ offs, uint32_t gpl, const AffPt* __restrict__ gsn,
                                 AffPt* __restrict__ out, uint32_t n) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t m = j / gpl, k = j % gpl;
  const AffPt D = gsn[kHalf];
  AffPt p = offs[m];
  uint32_t todo = k;
  if (m == 0 && k) {
    p = D;
    todo = k - 1;
  }
  for (uint32_t t = 0; t < todo; ++t) {
    if (fe_eq(p.x, D.x)) {      // p == D (small multiples never meet -D): DoubleDirect, SECP256K1.cpp:376-401
      Fe x2, num, den, s, x, y;
      fm_sqr(x2, p.x);
      fm_canon(x2, x2);
      fm_add(num, x2, x2);
      fm_add(num, num, x2);
      fm_add(den, p.y, p.y);
      fm_inv(den, den);
      fm_mul(s, num, den);
      fm_canon(s, s);
      fm_sqr(x, s);
      fm_sub(x, x, p.x);
      fm_sub(x, x, p.x);
      fm_canon(x, x);
      fm_sub(y, p.x, x);
      fm_mul(y, y, s);
      fm_sub(y, y, p.y);
      fm_canon(y, y);
      p = AffPt{x, y};
    } else {
      add_direct(p, p, D);
    }
  }
  out[j] = p;
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

template <int MODE>
__global__ __launch_bounds__(kBlock, KHB_WAVES_PER_SIMD) void k_giant_scan(ScanArgs A) {
  constexpr bool QUEUE = is_scan(MODE);
  constexpr bool BATCH = is_scan(MODE) || MODE == kDump;
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  Fe* scr = A.scratch + lane;
  __shared__ uint32_t s_queue[QUEUE ? kWavesPerBlock : 1][QUEUE ? kQWords * kQCap : 1];
  __shared__ uint32_t s_count[kWavesPerBlock];
  const uint32_t wave = QUEUE ? threadIdx.x >> 6 : 0;
#if KHB_LDSCOUNT
  ProbeQueue Q{s_queue[wave], (volatile __attribute__((address_space(3))) uint32_t*)&s_count[wave]};
#else
  ProbeQueue Q{s_queue[wave], &s_count[wave]};
#endif
  if (QUEUE) *Q.n = 0;
  uint32_t walked = 0;     // groups this lane walked (count_walked: the host checks the launch's total)
  if constexpr (BATCH) {
#if KHB_DYN
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
#else
    for (uint64_t item = lane; item < A.n_items; item += A.stride) {
      const uint32_t job = (uint32_t)(item / A.lanes_per_job);
      const uint32_t m = (uint32_t)(item % A.lanes_per_job);
      const uint32_t g0 = A.group_begin + m * kBatch;
      const uint32_t g1 = min(g0 + kBatch, A.group_end);
      walked += scan_batch<MODE>(A, Q, job, g0, g1, scr);
    }
#endif
  } else {
#if KHB_DYN
    // dynamic per-wave items, as above (counters[2])
    const uint32_t wl = threadIdx.x & 63u;
    for (;;) {
      uint32_t b = 0;
      if (wl == 0) b = atomicAdd(&A.counters[2], 64u);
      b = __builtin_amdgcn_readfirstlane(b);
      if (b >= A.n_items) break;
      const uint64_t item = (uint64_t)b + wl;
      if (item >= A.n_items) continue;
#else
    for (uint64_t item = lane; item < A.n_items; item += A.stride) {
#endif
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
}

// hash160 self-test: for x||y points, kind 0/1 = compressed with prefix 02/03, 2 = uncompressed;
// out = 20 hash bytes + 1 byte bloom_check20 result (when a bloom is given).
__global__ void k_hash160(const Fe* __restrict__ xy, int kind, const uint8_t* __restrict__ bloom, BloomGeom g,
                          uint8_t* __restrict__ out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fe x = xy[2 * i], y = xy[2 * i + 1];
  uint32_t h[5];
  if (kind < 2)
    hash160_compressed(h, 2u + (uint32_t)kind, x);
  else
    hash160_uncompressed(h, x, y);
  uint8_t* o = out + 21 * (size_t)i;
  for (int k = 0; k < 5; ++k)
    for (int b = 0; b < 4; ++b) o[4 * k + b] = (uint8_t)(h[k] >> (8 * b));
  o[20] = bloom ? (bloom_check20(bloom, g, h) ? 1 : 0) : 0;
}

// Field self-test: the fast (fe_asm.hpp) operations, results canonicalised.
__global__ void k_field_op(int op, const Fe* __restrict__ a, const Fe* __restrict__ b, Fe* __restrict__ r, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fe x = a[i], y = b[i], z;
  switch (op) {
    case 0: fm_mul(z, x, y); break;
    case 1: fm_sqr(z, x); break;
    case 2: fm_add(z, x, y); break;
    case 3: fm_sub(z, x, y); break;
    case 5: fm_add_lazy(z, x, y); break;     // x < p, y < 2^256
    case 6: fm_sqr_add(z, x, y); break;      // x, y < 2^256
    default: fm_inv(z, x); break;
  }
  fm_canon(z, z);
  r[i] = z;
}

__global__ void k_probe(const uint8_t* __restrict__ bloom, BloomGeom g, const Fe* __restrict__ xs, uint8_t* hit, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  hit[i] = bloom_probe_x(bloom, g, xs[i]) ? 1 : 0;
}

}  // namespace

// One submission's device state.  A context owns two (KHB_QUEUE_DEPTH): khb_submit fills the next
// free slot on its own stream, so a second batch's workgroups take the CUs the first batch's last
// waves leave idle (its launch tail), and khb_collect retires the slots in submission order.
struct Slot {
  hipStream_t stream = nullptr;
  Fe* d_scratch = nullptr;             // lane-private prefix scratch (allocated on the slot's first use)
  AffPt* d_centres = nullptr;
  AffPt* h_centres = nullptr;          // pinned staging
  uint32_t centres_cap = 0;
  khb_cand* d_cand = nullptr;
  khb_degenerate* d_degen = nullptr;
  uint32_t* d_ahits = nullptr;         // -m address hits
  uint32_t* d_counters = nullptr;
  uint32_t* h_counters = nullptr;      // pinned
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  uint64_t pending_steps = 0;
  int kind = 0;                        // in flight: 1 = -m bsgs scan, 2 = -m address scan
};
constexpr int kQueueDepth = 2;

struct khb_ctx {
  int device = -1;
  int last_hip = 0;
  uint32_t lanes = 0;
  uint8_t* d_bloom = nullptr;
  BloomGeom geom{};
  uint8_t* d_gate = nullptr;           // level-0 gate (khb_load_gate), null = none
  uint8_t* d_gate1 = nullptr;          // its stage-1 fold, null = none
  uint32_t gate1_mask = 0;
  uint32_t gate1_log2 = KHB_GATE1;     // khb_set_gate_stage1: fold size for gates loaded later
  uint32_t gate_mask = 0, gate_probes = 0;
  AffPt* d_gsn = nullptr;
  AffPt* d_offs = nullptr;
  uint32_t n_offs = 0, gpl = 0;
  AffPt* d_gofs = nullptr;             // per-group offsets expanded from gpl > 1 lane offsets
  bool gofs_stale = true;
  Slot slot[kQueueDepth];              // slot[0] also serves the synchronous helpers (dump, self-tests)
  int head = 0;                        // oldest in-flight slot
  int queued = 0;                      // submissions in flight (0..kQueueDepth)
  // -m address
  uint8_t* d_abloom = nullptr;
  BloomGeom ageom{};
};

namespace {

int hip_fail(khb_ctx* c, hipError_t e) {
  if (c) c->last_hip = (int)e;
  return e == hipErrorOutOfMemory ? KHB_ENOMEM : KHB_EHIP;
}
#define KHB_TRY(c, x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return hip_fail((c), e_); } while (0)

void pts_from_be(AffPt* dst, const uint8_t* src, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) {
    fe_from_be(dst[i].x, src + 64 * (size_t)i);
    fe_from_be(dst[i].y, src + 64 * (size_t)i + 32);
  }
}

// Groups the slot's last launch walked (count_walked, copied back with the counters).
uint64_t walked_groups(const Slot& S) {
  uint64_t v;
  memcpy(&v, S.h_counters + 4, sizeof v);
  return v;
}

// Entries (32 B) of lane-private scratch: scan_group needs 512, scan_batch kBatch*514 + kBatch.
constexpr size_t kScratchEntries = (size_t)kBatch * (kHalf + 3) > kHalf ? (size_t)kBatch * (kHalf + 3) : kHalf;

// Device state of a slot, created on its first use (a context that never queues a second
// submission never pays for a second scratch).
int ensure_slot(khb_ctx* c, Slot& S) {
  if (S.d_scratch) return KHB_OK;
  KHB_TRY(c, hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking));
  KHB_TRY(c, hipMalloc(&S.d_scratch, sizeof(Fe) * kScratchEntries * c->lanes));
  KHB_TRY(c, hipMalloc(&S.d_cand, sizeof(khb_cand) * kCandCap));
  KHB_TRY(c, hipMalloc(&S.d_degen, sizeof(khb_degenerate) * kDegenCap));
  KHB_TRY(c, hipMalloc(&S.d_counters, kCounterBytes));
  KHB_TRY(c, hipHostMalloc((void**)&S.h_counters, kCounterBytes, hipHostMallocDefault));
  KHB_TRY(c, hipEventCreate(&S.ev0));
  KHB_TRY(c, hipEventCreate(&S.ev1));
  return KHB_OK;
}

void free_slot(Slot& S) {
  if (S.stream) hipStreamSynchronize(S.stream);
  hipFree(S.d_scratch);
  hipFree(S.d_centres);
  hipFree(S.d_cand);
  hipFree(S.d_degen);
  hipFree(S.d_ahits);
  hipFree(S.d_counters);
  if (S.h_counters) hipHostFree(S.h_counters);
  if (S.h_centres) hipHostFree(S.h_centres);
  if (S.ev0) hipEventDestroy(S.ev0);
  if (S.ev1) hipEventDestroy(S.ev1);
  if (S.stream) hipStreamDestroy(S.stream);
  S = Slot{};
}

int ensure_centres(khb_ctx* c, Slot& S, uint32_t n) {
  if (n <= S.centres_cap) return KHB_OK;
  if (S.d_centres) hipFree(S.d_centres);
  if (S.h_centres) hipHostFree(S.h_centres);
  S.d_centres = nullptr;
  S.h_centres = nullptr;
  S.centres_cap = 0;
  uint32_t cap = n < 1024 ? 1024 : n;
  KHB_TRY(c, hipMalloc(&S.d_centres, sizeof(AffPt) * cap));
  KHB_TRY(c, hipHostMalloc((void**)&S.h_centres, sizeof(AffPt) * cap, hipHostMallocDefault));
  S.centres_cap = cap;
  return KHB_OK;
}

// The slot the next submission uses (KHB_EBUSY when every slot is in flight).
Slot* next_slot(khb_ctx* c, int& rc) {
  if (c->queued >= kQueueDepth) { rc = KHB_EBUSY; return nullptr; }
  Slot& S = c->slot[(c->head + c->queued) % kQueueDepth];
  rc = ensure_slot(c, S);
  return rc ? nullptr : &S;
}

// per_item: groups per work item (the lane-offset stride gpl, or kBatch for scan_batch modes)
ScanArgs make_args(khb_ctx* c, const Slot& S, uint32_t n_jobs, uint32_t group_begin, uint32_t group_count,
                   uint32_t per_item = 0) {
  ScanArgs A{};
  if (per_item == 0) per_item = c->gpl;
  A.bloom = c->d_bloom;
  A.geom = c->geom;
  A.gate = c->d_gate;
  A.gate_mask = c->gate_mask;
  A.gate_probes = c->gate_probes;
  A.gate1 = c->d_gate1;
  A.gate1_mask = c->gate1_mask;
  A.gsn = c->d_gsn;
  A.offs = c->d_offs;
  A.gofs = c->gpl == 1 ? c->d_offs : c->d_gofs;
  A.centres = S.d_centres;
  A.scratch = S.d_scratch;
  A.cand = S.d_cand;
  A.degen = S.d_degen;
  A.counters = S.d_counters;
  A.n_jobs = n_jobs;
  A.group_begin = group_begin;
  A.group_end = group_begin + group_count;
  A.gpl = c->gpl;
  A.lanes_per_job = (group_count + per_item - 1) / per_item;
  A.n_items = (uint64_t)n_jobs * A.lanes_per_job;
  A.stride = c->lanes;
  A.cand_cap = kCandCap;
  A.degen_cap = kDegenCap;
  return A;
}

int check_scan_args(khb_ctx* c, const uint8_t* centres, uint32_t n_jobs, uint32_t group_begin, uint32_t group_count,
                    bool bsgs = true) {
  if (!c || !centres || n_jobs == 0 || group_count == 0) return KHB_EINVAL;
  if (!c->d_gsn || !c->d_offs || c->gpl == 0) return KHB_ESTATE;
  if (group_begin % c->gpl) return KHB_EINVAL;
  uint64_t end = (uint64_t)group_begin + group_count;
  if (end > 0xFFFFFFFFull) return KHB_EINVAL;
  if (bsgs && end * KHB_GROUP > 0xFFFFFFFFull) return KHB_EINVAL;  // a = j*1024+t fits 32 bits (keyhunt.cpp:3948)
  if ((end + c->gpl - 1) / c->gpl > c->n_offs) return KHB_EINVAL;  // offsets table too short
  return KHB_OK;
}

// Per-group centre offsets for scan_batch: the lane offsets themselves when gpl == 1, else
// expanded once on the device (k_expand_offsets) after the giant table and offsets are loaded.
int ensure_gofs(khb_ctx* c) {
  if (c->gpl == 1 || !c->gofs_stale) return KHB_OK;
  const uint32_t n = c->n_offs * c->gpl;
  if (c->d_gofs) { hipFree(c->d_gofs); c->d_gofs = nullptr; }
  KHB_TRY(c, hipMalloc(&c->d_gofs, sizeof(AffPt) * (size_t)n));
  hipLaunchKernelGGL(k_expand_offsets, dim3((n + 255) / 256), dim3(256), 0, c->slot[0].stream, c->d_offs, c->gpl,
                     c->d_gsn, c->d_gofs, n);
  KHB_TRY(c, hipGetLastError());
  KHB_TRY(c, hipStreamSynchronize(c->slot[0].stream));
  c->gofs_stale = false;
  return KHB_OK;
}

}  // namespace

extern "C" {

const char* khb_strerror(int code) {
  switch (code) {
    case KHB_OK: return "ok";
    case KHB_EINVAL: return "invalid argument";
    case KHB_ENODEV: return "no usable gfx950 device";
    case KHB_ENOMEM: return "out of memory";
    case KHB_EHIP: return "HIP runtime error";
    case KHB_ESTATE: return "call order violated (tables not loaded?)";
    case KHB_EBUSY: return "submission in flight";
    case KHB_EINCOMPLETE: return "the device walked a different number of groups than submitted";
    default: return "unknown error";
  }
}

int khb_last_hip_error(const khb_ctx* c) { return c ? c->last_hip : 0; }
void* khb_stream(khb_ctx* c) { return c ? (void*)c->slot[0].stream : nullptr; }
uint32_t khb_lanes(const khb_ctx* c) { return c ? c->lanes : 0; }
uint32_t khb_groups_per_item(void) { return kBatch; }

uint32_t khb_default_lanes(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 0;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return 0;
  return (uint32_t)prop.multiProcessorCount * 4u * KHB_WAVES_PER_SIMD * 64u;
}

int khb_device_count(int* n) {
  if (!n) return KHB_EINVAL;
  int k = 0;
  if (hipGetDeviceCount(&k) != hipSuccess) k = 0;
  *n = k;
  return KHB_OK;
}

int khb_open(int device, uint32_t lanes, khb_ctx** out) {
  if (!out) return KHB_EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return KHB_ENODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return KHB_ENODEV;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return KHB_ENODEV;
  khb_ctx* c = new (std::nothrow) khb_ctx();
  if (!c) return KHB_ENOMEM;
  c->device = device;
  if (lanes == 0) lanes = (uint32_t)prop.multiProcessorCount * 4u * KHB_WAVES_PER_SIMD * 64u;   // one full residency
  lanes = (lanes + kBlock - 1) / kBlock * kBlock;
  c->lanes = lanes;
  hipError_t e = hipSetDevice(device);
  int rc = e == hipSuccess ? ensure_slot(c, c->slot[0]) : hip_fail(c, e);
  if (rc) {
    khb_close(c);
    return rc;
  }
  *out = c;
  return KHB_OK;
}

int khb_close(khb_ctx* c) {
  if (!c) return KHB_OK;
  if (c->device >= 0) hipSetDevice(c->device);
  for (Slot& S : c->slot) free_slot(S);
  hipFree(c->d_bloom);
  hipFree(c->d_gate);
  hipFree(c->d_gate1);
  hipFree(c->d_gsn);
  hipFree(c->d_offs);
  hipFree(c->d_gofs);
  hipFree(c->d_abloom);
  delete c;
  return KHB_OK;
}

int khb_load_gate(khb_ctx* c, const uint8_t* gate, uint32_t log2_bits, uint32_t probes) {
  if (!c || (gate && (log2_bits < 13 || log2_bits > 32 || probes < 1 || probes > KHB_GATE_MAX_PROBES)))
    return KHB_EINVAL;
  if (c->queued) return KHB_EBUSY;
  KHB_TRY(c, hipSetDevice(c->device));
  if (c->d_gate) { hipFree(c->d_gate); c->d_gate = nullptr; }
  if (c->d_gate1) { hipFree(c->d_gate1); c->d_gate1 = nullptr; }
  c->gate_mask = c->gate1_mask = 0;
  if (!gate) return KHB_OK;
  const size_t bytes = (size_t)1 << (log2_bits - 3);
  KHB_TRY(c, hipMalloc(&c->d_gate, bytes));
  KHB_TRY(c, hipMemcpy(c->d_gate, gate, bytes, hipMemcpyHostToDevice));
  c->gate_mask = (uint32_t)((1ull << (log2_bits - 6)) - 1);
  c->gate_probes = probes;
  if (c->gate1_log2 && (size_t)1 << c->gate1_log2 < bytes) {
    // stage 1: the gate OR-folded to 2^gate1_log2 bytes (a superset: no member is ever dropped)
    const size_t nb1 = ((size_t)1 << c->gate1_log2) / 8, nb = bytes / 8;
    std::vector<uint64_t> f(nb1, 0);
    const uint64_t* g = reinterpret_cast<const uint64_t*>(gate);
    for (size_t j = 0; j < nb; ++j) f[j & (nb1 - 1)] |= g[j];
    KHB_TRY(c, hipMalloc(&c->d_gate1, nb1 * 8));
    KHB_TRY(c, hipMemcpy(c->d_gate1, f.data(), nb1 * 8, hipMemcpyHostToDevice));
    c->gate1_mask = (uint32_t)(nb1 - 1);
  }
  return KHB_OK;
}

int khb_set_gate_stage1(khb_ctx* c, uint32_t log2_bytes) {
  if (!c || (log2_bytes && (log2_bytes < 10 || log2_bytes > 31))) return KHB_EINVAL;
  if (c->queued) return KHB_EBUSY;
  c->gate1_log2 = log2_bytes;
  return KHB_OK;
}

int khb_load_bloom(khb_ctx* c, const uint8_t* bf, uint64_t bytes_per_sub, uint64_t bits_per_sub, uint32_t hashes) {
  if (!c || !bf || bytes_per_sub == 0 || bits_per_sub < 2 || hashes == 0 || hashes > 255) return KHB_EINVAL;
  if ((bits_per_sub + 7) / 8 != bytes_per_sub) return KHB_EINVAL;    // bloom.cpp:110-113
  if (c->queued) return KHB_EBUSY;
  KHB_TRY(c, hipSetDevice(c->device));
  if (c->d_bloom) { hipFree(c->d_bloom); c->d_bloom = nullptr; }
  const size_t total = (size_t)bytes_per_sub * 256;
  KHB_TRY(c, hipMalloc(&c->d_bloom, total));
  KHB_TRY(c, hipMemcpy(c->d_bloom, bf, total, hipMemcpyHostToDevice));
  c->geom.bytes_per_sub = bytes_per_sub;
  c->geom.bits = bits_per_sub;
  c->geom.magic = (uint64_t)(((unsigned __int128)1 << 64) / bits_per_sub);
  c->geom.wrap = (uint64_t)(((unsigned __int128)1 << 64) % bits_per_sub);
  c->geom.hashes = hashes;
  return KHB_OK;
}

int khb_load_giant_table(khb_ctx* c, const uint8_t* gsn) {
  if (!c || !gsn) return KHB_EINVAL;
  if (c->queued) return KHB_EBUSY;
  KHB_TRY(c, hipSetDevice(c->device));
  // 513 points, then p - x of each (the walk's negated table, GsnTable::nx)
  struct {
    AffPt pt[KHB_GIANT_TABLE];
    Fe nx[KHB_GIANT_TABLE];
  } h;
  pts_from_be(h.pt, gsn, KHB_GIANT_TABLE);
  const Fe zero{};
  for (int i = 0; i < KHB_GIANT_TABLE; ++i) fe_sub(h.nx[i], zero, h.pt[i].x);
  if (!c->d_gsn) KHB_TRY(c, hipMalloc(&c->d_gsn, sizeof(h)));
  KHB_TRY(c, hipMemcpy(c->d_gsn, &h, sizeof(h), hipMemcpyHostToDevice));
  c->gofs_stale = true;
  return KHB_OK;
}

int khb_load_lane_offsets(khb_ctx* c, const uint8_t* offs, uint32_t n, uint32_t gpl) {
  if (!c || !offs || n == 0 || gpl == 0) return KHB_EINVAL;
  if (c->queued) return KHB_EBUSY;
  KHB_TRY(c, hipSetDevice(c->device));
  AffPt* h = (AffPt*)malloc(sizeof(AffPt) * n);
  if (!h) return KHB_ENOMEM;
  pts_from_be(h, offs, n);
  if (c->d_offs) { hipFree(c->d_offs); c->d_offs = nullptr; }
  hipError_t e = hipMalloc(&c->d_offs, sizeof(AffPt) * n);
  if (e == hipSuccess) e = hipMemcpy(c->d_offs, h, sizeof(AffPt) * n, hipMemcpyHostToDevice);
  free(h);
  if (e != hipSuccess) return hip_fail(c, e);
  c->n_offs = n;
  c->gpl = gpl;
  c->gofs_stale = true;
  return KHB_OK;
}

int khb_submit(khb_ctx* c, const uint8_t* centres, uint32_t n_jobs, uint32_t group_begin, uint32_t group_count) {
  int rc = check_scan_args(c, centres, n_jobs, group_begin, group_count);
  if (rc) return rc;
  if (!c->d_bloom) return KHB_ESTATE;
  if (c->queued && c->slot[c->head].kind != 1) return KHB_EBUSY;     // an -m address scan is in flight
  KHB_TRY(c, hipSetDevice(c->device));
  Slot* Sp = next_slot(c, rc);
  if (!Sp) return rc;
  Slot& S = *Sp;
  if ((rc = ensure_centres(c, S, n_jobs)) || (rc = ensure_gofs(c))) return rc;
  ScanArgs A = make_args(c, S, n_jobs, group_begin, group_count, kBatch);
  if (A.n_items > 0xFFFFFF00ull) return KHB_EINVAL;      // the 32-bit work-item counter (KHB_DYN)
  pts_from_be(S.h_centres, centres, n_jobs);
  KHB_TRY(c, hipMemcpyAsync(S.d_centres, S.h_centres, sizeof(AffPt) * n_jobs, hipMemcpyHostToDevice, S.stream));
  KHB_TRY(c, hipMemsetAsync(S.d_counters, 0, kCounterBytes, S.stream));
  const uint32_t blocks = c->lanes / kBlock;
  KHB_TRY(c, hipEventRecord(S.ev0, S.stream));
  if (c->d_gate1)
    hipLaunchKernelGGL(k_giant_scan<kScanG1>, dim3(blocks), dim3(kBlock), 0, S.stream, A);
  else if (c->d_gate)
    hipLaunchKernelGGL(k_giant_scan<kScanG>, dim3(blocks), dim3(kBlock), 0, S.stream, A);
  else
    hipLaunchKernelGGL(k_giant_scan<kScan>, dim3(blocks), dim3(kBlock), 0, S.stream, A);
  KHB_TRY(c, hipGetLastError());
  KHB_TRY(c, hipEventRecord(S.ev1, S.stream));
  KHB_TRY(c, hipMemcpyAsync(S.h_counters, S.d_counters, kCounterBytes, hipMemcpyDeviceToHost, S.stream));
  S.kind = 1;
  S.pending_steps = (uint64_t)n_jobs * group_count * KHB_GROUP;
  c->queued++;
  return KHB_OK;
}

int khb_collect(khb_ctx* c, khb_cand* cand, uint32_t cap, khb_degenerate* degen, uint32_t degen_cap, khb_stats* st) {
  if (!c) return KHB_EINVAL;
  if (!c->queued || c->slot[c->head].kind != 1) return KHB_ESTATE;
  KHB_TRY(c, hipSetDevice(c->device));
  Slot& S = c->slot[c->head];
  S.kind = 0;
  c->head = (c->head + 1) % kQueueDepth;
  c->queued--;
  KHB_TRY(c, hipStreamSynchronize(S.stream));
  const uint32_t nc = S.h_counters[0], nd = S.h_counters[1];
  uint32_t take = nc < kCandCap ? nc : kCandCap;
  if (take > cap) take = cap;
  if (take && cand) KHB_TRY(c, hipMemcpy(cand, S.d_cand, sizeof(khb_cand) * take, hipMemcpyDeviceToHost));
  uint32_t dt = nd < kDegenCap ? nd : kDegenCap;
  if (dt > degen_cap) dt = degen_cap;
  if (dt && degen) KHB_TRY(c, hipMemcpy(degen, S.d_degen, sizeof(khb_degenerate) * dt, hipMemcpyDeviceToHost));
  const uint64_t steps = walked_groups(S) * KHB_GROUP;
  if (st) {
    st->n_cand = nc;
    st->n_degenerate = nd;
    st->giant_steps = steps;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, S.ev0, S.ev1) != hipSuccess) ms = -1.f;
    st->kernel_ms = ms;
  }
  return steps == S.pending_steps ? KHB_OK : KHB_EINCOMPLETE;
}

int khb_scan(khb_ctx* c, const uint8_t* centres, uint32_t n_jobs, uint32_t group_begin, uint32_t group_count,
             khb_cand* cand, uint32_t cap, khb_stats* st) {
  int rc = khb_submit(c, centres, n_jobs, group_begin, group_count);
  if (rc) return rc;
  return khb_collect(c, cand, cap, nullptr, 0, st);
}

int khb_dump_x(khb_ctx* c, const uint8_t* centre, uint32_t group_begin, uint32_t group_count, uint8_t* xs) {
  int rc = check_scan_args(c, centre, 1, group_begin, group_count);
  if (rc) return rc;
  if (!xs) return KHB_EINVAL;
  if (c->queued) return KHB_EBUSY;
  KHB_TRY(c, hipSetDevice(c->device));
  Slot& S = c->slot[0];
  if ((rc = ensure_centres(c, S, 1)) || (rc = ensure_gofs(c))) return rc;
  pts_from_be(S.h_centres, centre, 1);
  const size_t bytes = (size_t)group_count * KHB_GROUP * 32;
  uint8_t* d_x = nullptr;
  KHB_TRY(c, hipMalloc(&d_x, bytes));
  hipError_t e = hipMemcpyAsync(S.d_centres, S.h_centres, sizeof(AffPt), hipMemcpyHostToDevice, S.stream);
  if (e == hipSuccess) e = hipMemsetAsync(S.d_counters, 0, kCounterBytes, S.stream);
  if (e == hipSuccess) {
    ScanArgs A = make_args(c, S, 1, group_begin, group_count, kBatch);
    A.xdump = d_x;
    const uint32_t blocks = (uint32_t)((A.n_items + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_giant_scan<kDump>, dim3(blocks < c->lanes / kBlock ? blocks : c->lanes / kBlock),
                       dim3(kBlock), 0, S.stream, A);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(S.stream);
  if (e == hipSuccess) e = hipMemcpy(xs, d_x, bytes, hipMemcpyDeviceToHost);
  hipFree(d_x);
  if (e != hipSuccess) return hip_fail(c, e);
  return KHB_OK;
}

int khb_field_op(khb_ctx* c, int op, const uint8_t* a, const uint8_t* b, uint8_t* r, uint32_t n) {
  if (!c || !a || !r || n == 0 || op < 0 || op > 6 || (op != 1 && op != 4 && !b)) return KHB_EINVAL;
  KHB_TRY(c, hipSetDevice(c->device));
  Slot& S = c->slot[0];
  Fe* h = (Fe*)malloc(sizeof(Fe) * n * 3);
  if (!h) return KHB_ENOMEM;
  for (uint32_t i = 0; i < n; ++i) {
    fe_from_be(h[i], a + 32 * (size_t)i);
    if (b) fe_from_be(h[n + i], b + 32 * (size_t)i); else h[n + i] = Fe{};
  }
  Fe* d = nullptr;
  hipError_t e = hipMalloc(&d, sizeof(Fe) * n * 3);
  if (e == hipSuccess) e = hipMemcpy(d, h, sizeof(Fe) * n * 2, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_field_op, dim3((n + 255) / 256), dim3(256), 0, S.stream, op, d, d + n, d + 2 * n, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(S.stream);
  if (e == hipSuccess) e = hipMemcpy(h + 2 * n, d + 2 * n, sizeof(Fe) * n, hipMemcpyDeviceToHost);
  if (e == hipSuccess)
    for (uint32_t i = 0; i < n; ++i) fe_to_be(r + 32 * (size_t)i, h[2 * n + i]);
  hipFree(d);
  free(h);
  if (e != hipSuccess) return hip_fail(c, e);
  return KHB_OK;
}

int khb_probe(khb_ctx* c, const uint8_t* xs, uint8_t* hit, uint32_t n) {
  if (!c || !xs || !hit || n == 0) return KHB_EINVAL;
  if (!c->d_bloom) return KHB_ESTATE;
  KHB_TRY(c, hipSetDevice(c->device));
  Slot& S = c->slot[0];
  Fe* h = (Fe*)malloc(sizeof(Fe) * n);
  if (!h) return KHB_ENOMEM;
  for (uint32_t i = 0; i < n; ++i) fe_from_be(h[i], xs + 32 * (size_t)i);
  Fe* d = nullptr;
  uint8_t* dh = nullptr;
  hipError_t e = hipMalloc(&d, sizeof(Fe) * n);
  if (e == hipSuccess) e = hipMalloc(&dh, n);
  if (e == hipSuccess) e = hipMemcpy(d, h, sizeof(Fe) * n, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_probe, dim3((n + 255) / 256), dim3(256), 0, S.stream, c->d_bloom, c->geom, d, dh, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(S.stream);
  if (e == hipSuccess) e = hipMemcpy(hit, dh, n, hipMemcpyDeviceToHost);
  hipFree(d);
  hipFree(dh);
  free(h);
  if (e != hipSuccess) return hip_fail(c, e);
  return KHB_OK;
}


// ---------------------------------------------------------------------------------- -m address
int khb_load_addr_bloom(khb_ctx* c, const uint8_t* bf, uint64_t bytes, uint64_t bits, uint32_t hashes) {
  if (!c || !bf || bytes == 0 || bits < 2 || hashes == 0 || hashes > 255) return KHB_EINVAL;
  if ((bits + 7) / 8 != bytes) return KHB_EINVAL;    // bloom.cpp:110-113
  if (c->queued) return KHB_EBUSY;
  KHB_TRY(c, hipSetDevice(c->device));
  if (c->d_abloom) { hipFree(c->d_abloom); c->d_abloom = nullptr; }
  KHB_TRY(c, hipMalloc(&c->d_abloom, bytes));
  KHB_TRY(c, hipMemcpy(c->d_abloom, bf, bytes, hipMemcpyHostToDevice));
  c->ageom.bytes_per_sub = bytes;
  c->ageom.bits = bits;
  c->ageom.magic = (uint64_t)(((unsigned __int128)1 << 64) / bits);
  c->ageom.wrap = (uint64_t)(((unsigned __int128)1 << 64) % bits);
  c->ageom.hashes = hashes;
  return KHB_OK;
}

int khb_addr_submit(khb_ctx* c, const uint8_t* centres, uint32_t n_jobs, uint32_t group_begin, uint32_t group_count,
                    int search) {
  int rc = check_scan_args(c, centres, n_jobs, group_begin, group_count, false);
  if (rc) return rc;
  if (search < 0 || search > 2) return KHB_EINVAL;
  if (!c->d_abloom) return KHB_ESTATE;
  if (c->queued && c->slot[c->head].kind != 2) return KHB_EBUSY;     // an -m bsgs scan is in flight
  KHB_TRY(c, hipSetDevice(c->device));
  Slot* Sp = next_slot(c, rc);
  if (!Sp) return rc;
  Slot& S = *Sp;
  if ((rc = ensure_centres(c, S, n_jobs))) return rc;
  if (!S.d_ahits) KHB_TRY(c, hipMalloc(&S.d_ahits, sizeof(khb_addr_hit) * kAddrHitCap));
  pts_from_be(S.h_centres, centres, n_jobs);
  KHB_TRY(c, hipMemcpyAsync(S.d_centres, S.h_centres, sizeof(AffPt) * n_jobs, hipMemcpyHostToDevice, S.stream));
  KHB_TRY(c, hipMemsetAsync(S.d_counters, 0, kCounterBytes, S.stream));
  ScanArgs A = make_args(c, S, n_jobs, group_begin, group_count);
  A.bloom = c->d_abloom;
  A.geom = c->ageom;
  A.ahits = S.d_ahits;
  A.ahit_cap = kAddrHitCap;
  const uint32_t blocks = c->lanes / kBlock;
  KHB_TRY(c, hipEventRecord(S.ev0, S.stream));
  switch (search) {
    case 0: hipLaunchKernelGGL(k_giant_scan<kAddrU>, dim3(blocks), dim3(kBlock), 0, S.stream, A); break;
    case 1: hipLaunchKernelGGL(k_giant_scan<kAddrC>, dim3(blocks), dim3(kBlock), 0, S.stream, A); break;
    default: hipLaunchKernelGGL(k_giant_scan<kAddrB>, dim3(blocks), dim3(kBlock), 0, S.stream, A); break;
  }
  KHB_TRY(c, hipGetLastError());
  KHB_TRY(c, hipEventRecord(S.ev1, S.stream));
  KHB_TRY(c, hipMemcpyAsync(S.h_counters, S.d_counters, kCounterBytes, hipMemcpyDeviceToHost, S.stream));
  S.kind = 2;
  S.pending_steps = (uint64_t)n_jobs * group_count * KHB_GROUP;
  c->queued++;
  return KHB_OK;
}

int khb_addr_collect(khb_ctx* c, khb_addr_hit* hits, uint32_t cap, khb_stats* st) {
  if (!c) return KHB_EINVAL;
  if (!c->queued || c->slot[c->head].kind != 2) return KHB_ESTATE;
  KHB_TRY(c, hipSetDevice(c->device));
  Slot& S = c->slot[c->head];
  S.kind = 0;
  c->head = (c->head + 1) % kQueueDepth;
  c->queued--;
  KHB_TRY(c, hipStreamSynchronize(S.stream));
  const uint32_t nh = S.h_counters[0], nd = S.h_counters[1];
  uint32_t take = nh < kAddrHitCap ? nh : kAddrHitCap;
  if (take > cap) take = cap;
  if (take && hits) KHB_TRY(c, hipMemcpy(hits, S.d_ahits, sizeof(khb_addr_hit) * take, hipMemcpyDeviceToHost));
  const uint64_t steps = walked_groups(S) * KHB_GROUP;
  if (st) {
    st->n_cand = nh;
    st->n_degenerate = nd;
    st->giant_steps = steps;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, S.ev0, S.ev1) != hipSuccess) ms = -1.f;
    st->kernel_ms = ms;
  }
  return steps == S.pending_steps ? KHB_OK : KHB_EINCOMPLETE;
}

int khb_addr_scan(khb_ctx* c, const uint8_t* centres, uint32_t n_jobs, uint32_t group_begin, uint32_t group_count,
                  int search, khb_addr_hit* hits, uint32_t cap, khb_stats* st) {
  int rc = khb_addr_submit(c, centres, n_jobs, group_begin, group_count, search);
  if (rc) return rc;
  return khb_addr_collect(c, hits, cap, st);
}

int khb_addr_dump(khb_ctx* c, const uint8_t* centre, uint32_t group_begin, uint32_t group_count, uint8_t* xy) {
  int rc = check_scan_args(c, centre, 1, group_begin, group_count, false);
  if (rc) return rc;
  if (!xy) return KHB_EINVAL;
  if (c->queued) return KHB_EBUSY;
  KHB_TRY(c, hipSetDevice(c->device));
  Slot& S = c->slot[0];
  if ((rc = ensure_centres(c, S, 1))) return rc;
  pts_from_be(S.h_centres, centre, 1);
  const size_t bytes = (size_t)group_count * KHB_GROUP * 64;
  uint8_t* d_xy = nullptr;
  KHB_TRY(c, hipMalloc(&d_xy, bytes));
  hipError_t e = hipMemcpyAsync(S.d_centres, S.h_centres, sizeof(AffPt), hipMemcpyHostToDevice, S.stream);
  if (e == hipSuccess) e = hipMemsetAsync(S.d_counters, 0, kCounterBytes, S.stream);
  if (e == hipSuccess) {
    ScanArgs A = make_args(c, S, 1, group_begin, group_count);
    A.xdump = d_xy;
    const uint32_t blocks = (uint32_t)((A.n_items + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_giant_scan<kAddrDump>, dim3(blocks < c->lanes / kBlock ? blocks : c->lanes / kBlock),
                       dim3(kBlock), 0, S.stream, A);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(S.stream);
  if (e == hipSuccess) e = hipMemcpy(xy, d_xy, bytes, hipMemcpyDeviceToHost);
  hipFree(d_xy);
  if (e != hipSuccess) return hip_fail(c, e);
  return KHB_OK;
}

int khb_hash160(khb_ctx* c, int kind, const uint8_t* xy, uint8_t* out, uint32_t n) {
  if (!c || !xy || !out || n == 0 || kind < 0 || kind > 2) return KHB_EINVAL;
  KHB_TRY(c, hipSetDevice(c->device));
  Slot& S = c->slot[0];
  AffPt* h = (AffPt*)malloc(sizeof(AffPt) * n);
  if (!h) return KHB_ENOMEM;
  pts_from_be(h, xy, n);
  AffPt* d = nullptr;
  uint8_t* dout = nullptr;
  hipError_t e = hipMalloc(&d, sizeof(AffPt) * n);
  if (e == hipSuccess) e = hipMalloc(&dout, 21 * (size_t)n);
  if (e == hipSuccess) e = hipMemcpy(d, h, sizeof(AffPt) * n, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_hash160, dim3((n + 255) / 256), dim3(256), 0, S.stream, (const Fe*)d, kind, c->d_abloom,
                       c->ageom, dout, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(S.stream);
  if (e == hipSuccess) e = hipMemcpy(out, dout, 21 * (size_t)n, hipMemcpyDeviceToHost);
  hipFree(d);
  hipFree(dout);
  free(h);
  if (e != hipSuccess) return hip_fail(c, e);
  return KHB_OK;
}


// ------------------------------------------------------------------------- baby-step tables
int khb_build_baby(khb_ctx* c, const uint8_t* centres, uint32_t n_jobs, uint32_t groups_per_job, uint64_t l1ext,
                   uint64_t m2, uint64_t m3, const uint64_t bytes_per_sub[3], const uint64_t bits_per_sub[3],
                   const uint32_t hashes[3], uint8_t* l1, uint8_t* l2, uint8_t* l3, uint8_t* bp, uint8_t* gate,
                   uint32_t gate_log2, uint32_t gate_probes, float* kernel_ms) {
  int rc = check_scan_args(c, centres, n_jobs, 0, groups_per_job, false);
  if (rc) return rc;
  if (!bytes_per_sub || !bits_per_sub || !hashes) return KHB_EINVAL;
  if (gate && (gate_log2 < 13 || gate_log2 > 32 || gate_probes < 1 || gate_probes > KHB_GATE_MAX_PROBES))
    return KHB_EINVAL;
  uint8_t* outs[3] = {l1, l2, l3};
  for (int l = 0; l < 3; ++l)
    if (outs[l] && (bits_per_sub[l] < 2 || (bits_per_sub[l] + 7) / 8 != bytes_per_sub[l] || hashes[l] == 0 ||
                    hashes[l] > 255))
      return KHB_EINVAL;
  if (c->queued) return KHB_EBUSY;
  KHB_TRY(c, hipSetDevice(c->device));
  Slot& S = c->slot[0];
  if ((rc = ensure_centres(c, S, n_jobs))) return rc;
  pts_from_be(S.h_centres, centres, n_jobs);
  ScanArgs A = make_args(c, S, n_jobs, 0, groups_per_job);
  A.job_keys = (uint64_t)groups_per_job * KHB_GROUP;
  A.blimit[0] = l1 ? l1ext : 0;
  A.blimit[1] = l2 ? m2 : 0;
  A.blimit[2] = (l3 || bp) ? m3 : 0;
  uint32_t* dw[3] = {nullptr, nullptr, nullptr};
  uint32_t* dbp = nullptr;
  uint32_t* dgate = nullptr;
  const uint64_t gate_bytes = gate ? (1ull << gate_log2) / 8 : 0;
  hipError_t e = hipSuccess;
  if (gate) {
    e = hipMalloc(&dgate, gate_bytes);
    if (e == hipSuccess) e = hipMemsetAsync(dgate, 0, gate_bytes, S.stream);
    A.gate_w = dgate;
    A.glimit = l1ext;
    A.gate_mask = (uint32_t)((1ull << (gate_log2 - 6)) - 1);
    A.gate_probes = gate_probes;
  }
  for (int l = 0; l < 3 && e == hipSuccess; ++l) {
    if (!outs[l]) continue;
    const uint64_t words = (bytes_per_sub[l] + 3) / 4;
    e = hipMalloc(&dw[l], 256 * words * 4);
    if (e == hipSuccess) e = hipMemsetAsync(dw[l], 0, 256 * words * 4, S.stream);
    A.bw[l] = dw[l];
    A.bwords[l] = words;
    BloomGeom& g = A.bgeom[l];
    g.bytes_per_sub = bytes_per_sub[l];
    g.bits = bits_per_sub[l];
    g.magic = (uint64_t)(((unsigned __int128)1 << 64) / g.bits);
    g.wrap = (uint64_t)(((unsigned __int128)1 << 64) % g.bits);
    g.hashes = hashes[l];
  }
  if (e == hipSuccess && bp && m3) {
    e = hipMalloc(&dbp, 16 * m3);
    A.bp = dbp;
  }
  if (e == hipSuccess)
    e = hipMemcpyAsync(S.d_centres, S.h_centres, sizeof(AffPt) * n_jobs, hipMemcpyHostToDevice, S.stream);
  if (e == hipSuccess) e = hipMemsetAsync(S.d_counters, 0, kCounterBytes, S.stream);
  if (e == hipSuccess) e = hipEventRecord(S.ev0, S.stream);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_giant_scan<kBaby>, dim3(c->lanes / kBlock), dim3(kBlock), 0, S.stream, A);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipEventRecord(S.ev1, S.stream);
  if (e == hipSuccess) e = hipStreamSynchronize(S.stream);
  uint64_t walked = 0;
  if (e == hipSuccess) e = hipMemcpy(S.h_counters, S.d_counters, kCounterBytes, hipMemcpyDeviceToHost);
  if (e == hipSuccess) walked = walked_groups(S);
  if (e == hipSuccess && kernel_ms) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, S.ev0, S.ev1) != hipSuccess) ms = -1.f;
    *kernel_ms = ms;
  }
  for (int l = 0; l < 3 && e == hipSuccess; ++l) {
    if (!outs[l]) continue;
    const uint64_t words = A.bwords[l], nb = bytes_per_sub[l];
    uint8_t* tmp = (uint8_t*)malloc(256 * words * 4);
    if (!tmp) { e = hipErrorOutOfMemory; break; }
    e = hipMemcpy(tmp, dw[l], 256 * words * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess)
      for (int sub = 0; sub < 256; ++sub) memcpy(outs[l] + sub * nb, tmp + sub * words * 4, nb);
    free(tmp);
  }
  if (e == hipSuccess && dbp) e = hipMemcpy(bp, dbp, 16 * m3, hipMemcpyDeviceToHost);
  if (e == hipSuccess && dgate) e = hipMemcpy(gate, dgate, gate_bytes, hipMemcpyDeviceToHost);
  for (int l = 0; l < 3; ++l) hipFree(dw[l]);
  hipFree(dbp);
  hipFree(dgate);
  if (e != hipSuccess) return hip_fail(c, e);
  return walked == (uint64_t)n_jobs * groups_per_job ? KHB_OK : KHB_EINCOMPLETE;
}

}  // extern "C"
