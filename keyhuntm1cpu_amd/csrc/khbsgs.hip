// libkhbsgs.so — MI355X (gfx950) BSGS giant-step engine behind the C ABI of include/khbsgs.h:
// contexts, submission slots, table loads, the self-test kernels and the launches of the
// k_giant_scan instances (scan_kernels.hpp; instantiated in k_bsgs.hip, k_addr.hip, k_baby.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <new>
#include <vector>
#include "scan_kernels.hpp"
#include "check_kernel.hpp"
#include <utility>

using namespace khbk;

namespace {

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
//
// Round 5: the scans' host hand-over lives in pinned, coherent host memory that the kernel reads and writes in
// place: the centres (read once per work item), the candidate / degenerate / -m address hit rings (written as
// hits occur, a few per launch) and a copy of the counters that the launch's last wave writes
// (launch_epilogue).  A khb_submit stream is then [event, kernel, event] with no memset or copy kernels, and
// khb_collect only waits for the slot's end event and copies from host memory.
struct Slot {
  hipStream_t stream = nullptr;
  Fe* d_scratch = nullptr;             // lane-private prefix scratch (allocated on the slot's first use)
  AffPt* d_centres = nullptr;          // device copy for the synchronous helpers (dump, baby build)
  AffPt* h_centres = nullptr;          // pinned, coherent; the scans read it in place
  uint32_t centres_cap = 0;
  khb_cand* h_cand = nullptr;          // pinned, coherent rings written by the kernel
  khb_degenerate* h_degen = nullptr;
  uint32_t* h_ahits = nullptr;         // -m address hits (allocated on the first -m address submission)
  uint32_t* d_counters = nullptr;
  uint32_t* h_counters = nullptr;      // pinned, coherent (launch_epilogue, or a copy after the helpers)
  bool counters_zero = false;          // d_counters is all zero (a scan's epilogue left it so): no memset
  hipEvent_t ev0 = nullptr, ev1 = nullptr;   // launch begin / end (khb_stats: kernel_ms, launch_*_ms)
  uint64_t pending_steps = 0;
  uint32_t total_waves = 0;            // of the launch in flight (host_counters_ok)
  int kind = 0;                        // in flight: 1 = -m bsgs scan, 2 = -m address scan
};
constexpr int kQueueDepth = 2;

struct khb_ctx {
  int device = -1;
  int last_hip = 0;
  uint32_t handoff_seen = 0, handoff_total = 0;   // the last collect's epilogue wave count (khb_last_handoff)
  uint32_t lanes = 0;
  uint8_t* d_bloom = nullptr;
  BloomGeom geom{};
  uint8_t* d_gate = nullptr;           // level-0 gate (khb_load_gate), null = none
  uint8_t* d_gate1 = nullptr;          // its stage-1 fold, null = none
  uint32_t gate1_mask = 0;
  uint32_t gate1_log2 = KHB_GATE1;     // khb_set_gate_stage1: fold size for gates loaded later
  uint32_t* d_gate0 = nullptr;         // the stage-0 filter, null = none
  uint32_t gate0_mask = 0;
  uint32_t gate0_log2 = KHB_GATE0;     // khb_set_gate_stage0: filter size for gates loaded later
  uint32_t gate_mask = 0, gate_probes = 0;
  AffPt* d_gsn = nullptr;
  AffPt* d_offs = nullptr;
  uint32_t n_offs = 0, gpl = 0;
  AffPt* d_gofs = nullptr;             // per-group offsets expanded from gpl > 1 lane offsets
  bool gofs_stale = true;
  Slot slot[kQueueDepth];              // slot[0] also serves the synchronous helpers (dump, self-tests)
  int head = 0;                        // oldest in-flight slot
  int queued = 0;                      // submissions in flight (0..kQueueDepth)
  uint32_t cand_cap = kCandCap;        // candidate ring entries a launch may fill (khb_set_candidate_capacity)
  // The context's clock (khb_stats.launch_begin_ms / launch_end_ms; khb_reset_epoch restarts it): the
  // `epoch` event sits epoch_ms after the clock's origin.  hipEventElapsedTime is a float, so the anchor
  // moves forward once its distance to a launch passes kReanchorMs (a float ms keeps ~4 us at 60 s, but
  // ~1 ms after 4.6 h): begin = epoch_ms + elapsed(epoch, ev0) in double, end = begin + the launch's own
  // elapsed(ev0, ev1) (the busy-time union no longer drifts on long CLI runs).
  // The previous anchor stays valid as a fallback for a launch of the other slot that began before the
  // current anchor was recorded (a negative distance).
  hipEvent_t epoch = nullptr;
  hipEvent_t epoch_prev = nullptr;
  double epoch_ms = 0.0, epoch_prev_ms = 0.0;
  bool have_prev = false;
  // -m address
  uint8_t* d_abloom = nullptr;
  BloomGeom ageom{};
  // second / third check (khb_load_check_tables, khb_check): tables, a high-priority stream of its own
  // and buffers grown to the largest batch
  khb::CheckTables ck{};
  void* d_ck = nullptr;                // one allocation holding every check table
  bool ck_loaded = false;
  hipStream_t ck_stream = nullptr;
  CheckIn* d_ck_in = nullptr;
  CheckOut* d_ck_out = nullptr;
  khb::CPt* d_ck_targets = nullptr;
  uint32_t ck_cap = 0, ck_tcap = 0;
  // the targets on the device (d_ck_targets) as the caller passed them: a khb_check with the same bytes
  // uploads only its CheckIn records (no O(n_targets) conversion and upload per batch)
  std::vector<uint8_t> ck_targets_be;
};

namespace {

int hip_fail(khb_ctx* c, hipError_t e) {
  if (c) c->last_hip = (int)e;
  // The runtime keeps the last error for hipGetLastError: a failed allocation the caller recovers
  // from (khb_reserve_slots -> depth 1) would otherwise fail the next launch check of khb_submit.
  (void)hipGetLastError();
  return e == hipErrorOutOfMemory ? KHB_ENOMEM : KHB_EHIP;
}
#define KHB_TRY(c, x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return hip_fail((c), e_); } while (0)

void pts_from_be(AffPt* dst, const uint8_t* src, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) {
    fe_from_be(dst[i].x, src + 64 * (size_t)i);
    fe_from_be(dst[i].y, src + 64 * (size_t)i + 32);
  }
}

// A bloom level's geometry with the Barrett constants of mod_bits (bloom_probe.hpp).
BloomGeom bloom_geom(uint64_t bytes_per_sub, uint64_t bits, uint32_t hashes) {
  BloomGeom g{};
  g.bytes_per_sub = bytes_per_sub;
  g.bits = bits;
  g.magic = (uint64_t)(((unsigned __int128)1 << 64) / bits);
  g.wrap = (uint64_t)(((unsigned __int128)1 << 64) % bits);
  g.hashes = hashes;
  return g;
}

// Groups the slot's last launch walked (count_walked, copied back with the counters).
uint64_t walked_groups(const Slot& S) {
  uint64_t v;
  memcpy(&v, S.h_counters + 4, sizeof v);
  return v;
}

// Entries (32 B) of lane-private scratch: scan_group needs 512, scan_batch kBatch*514 + kBatch.
constexpr size_t kScratchEntries = (size_t)kBatch * (kHalf + 3) > kHalf ? (size_t)kBatch * (kHalf + 3) : kHalf;

void free_slot(Slot& S);

// Device state of a slot: slot 0 at khb_open, slot 1 on the first queued submission or up front by
// khb_reserve_slots.  A failure part-way frees what was allocated, so the slot is either complete or
// empty (and the caller may go on with the slots it has).
int ensure_slot_alloc(khb_ctx* c, Slot& S) {
  KHB_TRY(c, hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking));
  KHB_TRY(c, hipMalloc(&S.d_scratch, sizeof(Fe) * kScratchEntries * c->lanes));
  KHB_TRY(c, hipHostMalloc((void**)&S.h_cand, sizeof(khb_cand) * kCandCap, hipHostMallocCoherent));
  KHB_TRY(c, hipHostMalloc((void**)&S.h_degen, sizeof(khb_degenerate) * kDegenCap, hipHostMallocCoherent));
  KHB_TRY(c, hipMalloc(&S.d_counters, kCounterBytes));
  // on the slot's own stream: a null-stream hipMemset of device memory may still be queued (behind the other
  // slot's running launch, for CU slots) when this slot's first launch starts, and would zero its counters
  // mid-launch (round 5: a lazily allocated slot 1 re-walked 6,144 groups, tools/debug/epilogue_diag.py)
  KHB_TRY(c, hipMemsetAsync(S.d_counters, 0, kCounterBytes, S.stream));
  S.counters_zero = true;
  KHB_TRY(c, hipHostMalloc((void**)&S.h_counters, kHostCounterBytes, hipHostMallocCoherent));
  KHB_TRY(c, hipEventCreate(&S.ev0));
  KHB_TRY(c, hipEventCreate(&S.ev1));
  return KHB_OK;
}

int ensure_slot(khb_ctx* c, Slot& S) {
  if (S.ev1) return KHB_OK;            // complete (ev1 is created last)
  const int rc = ensure_slot_alloc(c, S);
  if (rc) free_slot(S);
  return rc;
}

void free_slot(Slot& S) {
  if (S.stream) hipStreamSynchronize(S.stream);
  hipFree(S.d_scratch);
  hipFree(S.d_centres);
  if (S.h_cand) hipHostFree(S.h_cand);
  if (S.h_degen) hipHostFree(S.h_degen);
  if (S.h_ahits) hipHostFree(S.h_ahits);
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
  KHB_TRY(c, hipHostMalloc((void**)&S.h_centres, sizeof(AffPt) * cap, hipHostMallocCoherent));
  S.centres_cap = cap;
  return KHB_OK;
}

// The slot the next submission uses (KHB_EBUSY when every slot is in flight).
Slot* next_slot(khb_ctx* c, int& rc) {
  if (c->queued >= kQueueDepth) { rc = KHB_EBUSY; return nullptr; }
  // With nothing in flight the ring restarts at slot 0 (allocated by khb_open), so a caller that keeps
  // one submission in flight -- the depth-1 fallback after KHB_ENOMEM from khb_reserve_slots -- never
  // touches slot 1.  Collect order stays submission order.
  if (c->queued == 0) c->head = 0;
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
  A.gate0 = c->d_gate0;
  A.gate0_mask = c->gate0_mask;
  A.gsn = c->d_gsn;
  A.offs = c->d_offs;
  A.gofs = c->gpl == 1 ? c->d_offs : c->d_gofs;
  A.centres = S.d_centres;
  A.scratch = S.d_scratch;
  A.cand = S.h_cand;
  A.degen = S.h_degen;
  A.counters = S.d_counters;
  A.n_jobs = n_jobs;
  A.group_begin = group_begin;
  A.group_end = group_begin + group_count;
  A.gpl = c->gpl;
  A.lanes_per_job = (group_count + per_item - 1) / per_item;
  A.n_items = (uint64_t)n_jobs * A.lanes_per_job;
  A.stride = c->lanes;
  A.cand_cap = c->cand_cap;
  A.degen_cap = kDegenCap;
  return A;
}

// kernel_ms and the launch's interval on the context's clock (khb_reset_epoch), from the slot's events;
// the shader clock from the kernel's clock_probe samples.
// Called after S's stream has drained (the slot's launch is complete and the stream idle).
//
// Round 5: a scan launched by khb_submit / khb_addr_submit (launch_epilogue) is timed by its own clocks: block 0's
// first wave samples s_memtime / s_memrealtime when it starts (the launch's first workgroup) and the launch's last
// wave when it leaves, so kernel_ms is the launch's execution span on the 100 MHz clock and the shader clock is
// the average over that span.  The interval on the context's clock ends at the slot's end event and begins that
// span earlier.  The events alone would also count the time the queued launch waits, dispatched, for the CUs
// the other slot's running launch still holds (nothing but a kernel sits on the slot's stream since round 5).
constexpr float kReanchorMs = 60000.f;
void launch_times(khb_ctx* c, const Slot& S, khb_stats* st, bool epilogue) {
  uint64_t p[4], q[2];
  memcpy(p, S.h_counters + 8, sizeof p);
  memcpy(q, S.h_counters + 16, sizeof q);
  // The shader clock from block 0's first wave alone (its start and exit): s_memtime counts per XCD, so a
  // ratio across two waves on different XCDs is meaningless.  The 100 MHz s_memrealtime is one clock for the
  // whole device: the execution span runs from block 0's start to the last wave's exit (q[1]).
  const bool clocks = p[3] > p[1] && p[2] > p[0];
  st->shader_mhz = clocks ? (float)(100.0 * (double)(p[2] - p[0]) / (double)(p[3] - p[1])) : 0.f;
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, S.ev0, S.ev1) != hipSuccess) ms = -1.f;
  st->event_ms = ms;
  if (epilogue && q[1] > p[1] && ms >= 0.f) {
    const float span = (float)((double)(q[1] - p[1]) * 1e-5);     // 100 MHz ticks -> ms
    if (span < ms) ms = span;
  }
  st->kernel_ms = ms;
  float e = -1.f, ep = -1.f, b = -1.f;
  double end = -1.0;
  const bool cur = c->epoch && hipEventElapsedTime(&b, c->epoch, S.ev0) == hipSuccess && b >= 0.f;
  if (cur && hipEventElapsedTime(&e, c->epoch, S.ev1) == hipSuccess && e >= 0.f)
    end = c->epoch_ms + (double)e;
  else if (c->have_prev && hipEventElapsedTime(&ep, c->epoch_prev, S.ev1) == hipSuccess && ep >= 0.f)
    end = c->epoch_prev_ms + (double)ep;
  if (end >= 0.0 && ms >= 0.f) {
    st->launch_begin_ms = end - (double)ms;
    st->launch_end_ms = end;
  } else {
    st->launch_begin_ms = st->launch_end_ms = -1.0;
  }
  float d = 0.f;
  if (cur && b > kReanchorMs && c->epoch_prev && hipEventRecord(c->epoch_prev, S.stream) == hipSuccess &&
      hipEventSynchronize(c->epoch_prev) == hipSuccess &&
      hipEventElapsedTime(&d, c->epoch, c->epoch_prev) == hipSuccess) {
    // the new anchor (recorded now on the idle stream) becomes current; the old one the fallback
    std::swap(c->epoch, c->epoch_prev);
    c->epoch_prev_ms = c->epoch_ms;
    c->epoch_ms += (double)d;
    c->have_prev = true;
  }
}

// The scans' launch without copy kernels: centres read in place from the slot's pinned block, counters
// zeroed by the previous scan's epilogue (a memset only after a helper used them), the last wave's copy of
// them in h_counters; h_counters[3] is poisoned so that khb_collect can tell the epilogue ran.
int prepare_host_launch(khb_ctx* c, Slot& S, ScanArgs& A, uint32_t blocks) {
  if (!S.counters_zero) KHB_TRY(c, hipMemsetAsync(S.d_counters, 0, kCounterBytes, S.stream));
  S.counters_zero = false;             // until khb_collect sees the epilogue's copy
  memset(S.h_counters, 0, kHostCounterBytes);
  S.h_counters[3] = 0xFFFFFFFFu;
  A.centres = S.h_centres;
  A.host_counters = S.h_counters;
  A.total_waves = blocks * kWavesPerBlock;
  return KHB_OK;
}

// After the slot's end event: the epilogue's copy is complete iff it counted every wave of the launch.
// The launch epilogue counted every wave (else KHB_EHANDOFF; the counts are kept for khb_last_handoff).
bool host_counters_ok(khb_ctx* c, const Slot& S) {
  c->handoff_seen = S.h_counters[3];
  c->handoff_total = S.total_waves;
  return S.h_counters[3] == S.total_waves;
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
    case KHB_EHANDOFF: return "the launch's end-of-launch hand-off did not count every wave (khb_last_handoff)";
    default: return "unknown error";
  }
}

int khb_last_hip_error(const khb_ctx* c) { return c ? c->last_hip : 0; }
void* khb_stream(khb_ctx* c) { return c ? (void*)c->slot[0].stream : nullptr; }
uint32_t khb_lanes(const khb_ctx* c) { return c ? c->lanes : 0; }
int khb_abi_version(void) { return KHB_ABI_VERSION; }

#ifndef KHB_VARIANT
#define KHB_VARIANT "product"        // tools/build_variant.sh names its timing builds (-DKHB_VARIANT=\"<name>\")
#endif
#ifndef KHB_BUILD_DEFINES
#define KHB_BUILD_DEFINES ""         // the extra -D flags of a tools/build_variant.sh build, comma-separated
#endif
#define KHB_STR2(x) #x
#define KHB_STR(x) KHB_STR2(x)
const char* khb_build_info(void) {
  return "abi=" KHB_STR(KHB_ABI_VERSION) " arch=gfx950 variant=" KHB_VARIANT
         " waves_per_simd=" KHB_STR(KHB_WAVES_PER_SIMD) " addr_waves_per_simd=" KHB_STR(KHB_ADDR_WAVES_PER_SIMD)
         " batch=" KHB_STR(KHB_BATCH) " gate1=" KHB_STR(KHB_GATE1) " half_stream=" KHB_STR(KHB_HALF_STREAM)
         " gate0=" KHB_STR(KHB_GATE0) " defines=" KHB_BUILD_DEFINES " compiler=" __clang_version__;
}

int khb_last_handoff(const khb_ctx* c, uint32_t* waves_seen, uint32_t* waves_total) {
  if (!c) return KHB_EINVAL;
  if (waves_seen) *waves_seen = c->handoff_seen;
  if (waves_total) *waves_total = c->handoff_total;
  return KHB_OK;
}

uint32_t khb_groups_per_item(void) { return kBatch; }

int khb_reserve_slots(khb_ctx* c, int depth) {
  if (!c || depth < 1 || depth > kQueueDepth) return KHB_EINVAL;
  if (c->queued) return KHB_EBUSY;
  KHB_TRY(c, hipSetDevice(c->device));
  for (int i = 1; i < depth; ++i) {
    const int rc = ensure_slot(c, c->slot[i]);
    if (rc) return rc;                 // the slot is left empty (ensure_slot frees a partial one)
  }
  return KHB_OK;
}

int khb_set_candidate_capacity(khb_ctx* c, uint32_t cap) {
  if (!c || cap == 0 || cap > kCandCap) return KHB_EINVAL;
  if (c->queued) return KHB_EBUSY;
  c->cand_cap = cap;
  return KHB_OK;
}

uint32_t khb_candidate_capacity(const khb_ctx* c) { return c ? c->cand_cap : 0; }

uint32_t khb_addr_hit_capacity(const khb_ctx* c) {
  return c ? (c->cand_cap < kAddrHitCap ? c->cand_cap : kAddrHitCap) : 0;
}

int khb_reset_epoch(khb_ctx* c) {
  if (!c) return KHB_EINVAL;
  if (c->queued) return KHB_EBUSY;
  KHB_TRY(c, hipSetDevice(c->device));
  KHB_TRY(c, hipEventRecord(c->epoch, c->slot[0].stream));
  c->epoch_ms = c->epoch_prev_ms = 0.0;
  c->have_prev = false;
  return KHB_OK;
}

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
  if (!rc && (e = hipEventCreate(&c->epoch)) == hipSuccess && (e = hipEventCreate(&c->epoch_prev)) == hipSuccess)
    e = hipEventRecord(c->epoch, c->slot[0].stream);
  if (!rc && e != hipSuccess) rc = hip_fail(c, e);
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
  if (c->epoch) hipEventDestroy(c->epoch);
  if (c->epoch_prev) hipEventDestroy(c->epoch_prev);
  if (c->ck_stream) {
    hipStreamSynchronize(c->ck_stream);
    hipStreamDestroy(c->ck_stream);
  }
  hipFree(c->d_ck);
  hipFree(c->d_ck_in);
  hipFree(c->d_ck_out);
  hipFree(c->d_ck_targets);
  hipFree(c->d_bloom);
  hipFree(c->d_gate);
  hipFree(c->d_gate1);
  hipFree(c->d_gate0);
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
  if (c->d_gate0) { hipFree(c->d_gate0); c->d_gate0 = nullptr; }
  c->gate_mask = c->gate1_mask = c->gate0_mask = 0;
  if (!gate) return KHB_OK;
  const size_t bytes = (size_t)1 << (log2_bits - 3);
  // one probe: every block's hi word set on the device copy, so the kernels' fixed three-probe test
  // (scan_kernels.hpp gate_block_pass: probe 1 reads hi, probe 2 repeats probe 0) gives the one-probe answer
  std::vector<uint64_t> one;
  if (probes == 1) {
    one.resize(bytes / 8);
    memcpy(one.data(), gate, bytes);
    for (uint64_t& b : one) b |= 0xFFFFFFFF00000000ull;
    gate = reinterpret_cast<const uint8_t*>(one.data());
  }
  KHB_TRY(c, hipMalloc(&c->d_gate, bytes));
  KHB_TRY(c, hipMemcpy(c->d_gate, gate, bytes, hipMemcpyHostToDevice));
  c->gate_mask = (uint32_t)((1ull << (log2_bits - 6)) - 1);
  c->gate_probes = probes;
  // KHB_GATE_STAGE1_AUTO: an L2-sized 2 MiB fold of a gate of up to 32 MiB (k = 1: -8.6 % time with two
  // launches in flight, profiles/r04k/stage1_k1_nt_pipe_ab.txt; 4 MiB equal on the half-stream product, r06d), a
  // 32 MiB fold of a larger one (k = 4: the 128 MiB gate beside the 57.5 MiB L1 bloom).  Round 4 (full prefix stream)
  // had measured 16 MiB 3.5 % faster than 32 MiB (profiles/r04l/k4_stage1_ab.txt); with the half prefix stream's
  // halved MALL traffic 32 MiB is 1.3 % faster than 16 MiB and 0.8 % than 64 MiB (5 rounds each, profiles/r06e).
  const uint32_t f_log2 = c->gate1_log2 != KHB_GATE_STAGE1_AUTO ? c->gate1_log2 : bytes <= (1u << 25) ? 21u : 25u;
  if (f_log2 && (size_t)1 << f_log2 < bytes) {
    // stage 1: the gate OR-folded to 2^f_log2 bytes (a superset: no member is ever dropped)
    const size_t nb1 = ((size_t)1 << f_log2) / 8, nb = bytes / 8;
    std::vector<uint64_t> f(nb1, 0);
    const uint64_t* g = reinterpret_cast<const uint64_t*>(gate);
    for (size_t j = 0; j < nb; ++j) f[j & (nb1 - 1)] |= g[j];
    KHB_TRY(c, hipMalloc(&c->d_gate1, nb1 * 8));
    KHB_TRY(c, hipMemcpy(c->d_gate1, f.data(), nb1 * 8, hipMemcpyHostToDevice));
    c->gate1_mask = (uint32_t)(nb1 - 1);
    // stage 0 (off by default, KHB_GATE0): KHB_GATE_STAGE0_AUTO puts a 2 MiB one-bit-per-member filter in front of a
    // fold larger than 2 MiB (k >= 4, where the fold is read from the MALL for every x); none at k = 1, whose
    // 2 MiB fold is itself L2-resident.  With one probe every hi word is set (above), so the filter would pass
    // everything: none.
    const uint32_t z_log2 = c->gate0_log2 != KHB_GATE_STAGE0_AUTO ? c->gate0_log2 : f_log2 > 21 ? 21u : 0u;
    if (z_log2 && probes >= 2 && (size_t)1 << z_log2 < nb1 * 8) {
      // stage 0: the hi words of the gate's blocks (probe 1's bit of every member) OR-folded to 2^z_log2 bytes
      const size_t nw0 = ((size_t)1 << z_log2) / 4;
      std::vector<uint32_t> z(nw0, 0);
      for (size_t j = 0; j < nb; ++j) z[j & (nw0 - 1)] |= (uint32_t)(g[j] >> 32);
      KHB_TRY(c, hipMalloc(&c->d_gate0, nw0 * 4));
      KHB_TRY(c, hipMemcpy(c->d_gate0, z.data(), nw0 * 4, hipMemcpyHostToDevice));
      c->gate0_mask = (uint32_t)(nw0 - 1);
    }
  }
  return KHB_OK;
}

int khb_gate_stages(const khb_ctx* c) {
  if (!c) return KHB_EINVAL;
  return (c->d_gate ? 4 : 0) | (c->d_gate1 ? 2 : 0) | (c->d_gate0 ? 1 : 0);
}

int khb_set_gate_stage0(khb_ctx* c, uint32_t log2_bytes) {
  if (!c || (log2_bytes && log2_bytes != KHB_GATE_STAGE0_AUTO && (log2_bytes < 10 || log2_bytes > 30)))
    return KHB_EINVAL;
  if (c->queued) return KHB_EBUSY;
  c->gate0_log2 = log2_bytes;
  return KHB_OK;
}

int khb_set_gate_stage1(khb_ctx* c, uint32_t log2_bytes) {
  if (!c || (log2_bytes && log2_bytes != KHB_GATE_STAGE1_AUTO && (log2_bytes < 10 || log2_bytes > 31)))
    return KHB_EINVAL;
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
  c->geom = bloom_geom(bytes_per_sub, bits_per_sub, hashes);
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
  const uint32_t blocks = c->lanes / kBlock;
  if ((rc = prepare_host_launch(c, S, A, blocks))) return rc;
  KHB_TRY(c, hipEventRecord(S.ev0, S.stream));
  launch_bsgs(c->d_gate0 ? kScanG2 : c->d_gate1 ? kScanG1 : c->d_gate ? kScanG : kScan, blocks, S.stream, A);
  KHB_TRY(c, hipGetLastError());
  KHB_TRY(c, hipEventRecord(S.ev1, S.stream));
  S.total_waves = A.total_waves;
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
  KHB_TRY(c, hipEventSynchronize(S.ev1));
  if (!host_counters_ok(c, S)) return KHB_EHANDOFF;   // the launch's epilogue did not complete
  S.counters_zero = true;
  const uint32_t nc = S.h_counters[0], nd = S.h_counters[1];
  uint32_t take = nc < c->cand_cap ? nc : c->cand_cap;
  if (take > cap) take = cap;
  if (take && cand) memcpy(cand, S.h_cand, sizeof(khb_cand) * take);
  uint32_t dt = nd < kDegenCap ? nd : kDegenCap;
  if (dt > degen_cap) dt = degen_cap;
  if (dt && degen) memcpy(degen, S.h_degen, sizeof(khb_degenerate) * dt);
  const uint64_t steps = walked_groups(S) * KHB_GROUP;
  if (st) {
    st->n_cand = nc;
    st->n_degenerate = nd;
    st->giant_steps = steps;
    launch_times(c, S, st, true);
  }
  return steps == S.pending_steps ? KHB_OK : KHB_EINCOMPLETE;
}

int khb_scan(khb_ctx* c, const uint8_t* centres, uint32_t n_jobs, uint32_t group_begin, uint32_t group_count,
             khb_cand* cand, uint32_t cap, khb_stats* st) {
  if (c && c->queued) return KHB_EBUSY;   // khb_collect would retire the older submission, not this one
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
  S.counters_zero = false;
  if (e == hipSuccess) {
    ScanArgs A = make_args(c, S, 1, group_begin, group_count, kBatch);
    A.xdump = d_x;
    const uint32_t blocks = (uint32_t)((A.n_items + kBlock - 1) / kBlock);
    launch_bsgs(kDump, blocks < c->lanes / kBlock ? blocks : c->lanes / kBlock, S.stream, A);
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
  c->ageom = bloom_geom(bytes, bits, hashes);
  return KHB_OK;
}

int khb_addr_submit(khb_ctx* c, const uint8_t* centres, uint32_t n_jobs, uint32_t group_begin, uint32_t group_count,
                    int search) {
  int rc = check_scan_args(c, centres, n_jobs, group_begin, group_count, false);
  if (rc) return rc;
  const bool endo = search >= 0 && (search & KHB_SEARCH_ENDOMORPHISM);
  if (endo) search &= ~KHB_SEARCH_ENDOMORPHISM;
  if (search < 0 || search > 2) return KHB_EINVAL;
  if (!c->d_abloom) return KHB_ESTATE;
  if (c->queued && c->slot[c->head].kind != 2) return KHB_EBUSY;     // an -m bsgs scan is in flight
  KHB_TRY(c, hipSetDevice(c->device));
  Slot* Sp = next_slot(c, rc);
  if (!Sp) return rc;
  Slot& S = *Sp;
  if ((rc = ensure_centres(c, S, n_jobs))) return rc;
  if (!S.h_ahits)
    KHB_TRY(c, hipHostMalloc((void**)&S.h_ahits, sizeof(khb_addr_hit) * kAddrHitCap, hipHostMallocCoherent));
  pts_from_be(S.h_centres, centres, n_jobs);
  ScanArgs A = make_args(c, S, n_jobs, group_begin, group_count);
  A.bloom = c->d_abloom;
  A.geom = c->ageom;
  A.ahits = S.h_ahits;
  A.ahit_cap = khb_addr_hit_capacity(c);
  const uint32_t blocks = c->lanes / kBlock;
  if ((rc = prepare_host_launch(c, S, A, blocks))) return rc;
  KHB_TRY(c, hipEventRecord(S.ev0, S.stream));
  if (endo)
    launch_addr_e(search == 0 ? kAddrUE : search == 1 ? kAddrCE : kAddrBE, blocks, S.stream, A);
  else
    launch_addr(search == 0 ? kAddrU : search == 1 ? kAddrC : kAddrB, blocks, S.stream, A);
  KHB_TRY(c, hipGetLastError());
  KHB_TRY(c, hipEventRecord(S.ev1, S.stream));
  S.total_waves = A.total_waves;
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
  KHB_TRY(c, hipEventSynchronize(S.ev1));
  if (!host_counters_ok(c, S)) return KHB_EHANDOFF;   // the launch's epilogue did not complete
  S.counters_zero = true;
  const uint32_t nh = S.h_counters[0], nd = S.h_counters[1];
  const uint32_t acap = khb_addr_hit_capacity(c);
  uint32_t take = nh < acap ? nh : acap;
  if (take > cap) take = cap;
  if (take && hits) memcpy(hits, S.h_ahits, sizeof(khb_addr_hit) * take);
  const uint64_t steps = walked_groups(S) * KHB_GROUP;
  if (st) {
    st->n_cand = nh;
    st->n_degenerate = nd;
    st->giant_steps = steps;
    launch_times(c, S, st, true);
  }
  return steps == S.pending_steps ? KHB_OK : KHB_EINCOMPLETE;
}

int khb_addr_scan(khb_ctx* c, const uint8_t* centres, uint32_t n_jobs, uint32_t group_begin, uint32_t group_count,
                  int search, khb_addr_hit* hits, uint32_t cap, khb_stats* st) {
  if (c && c->queued) return KHB_EBUSY;   // as khb_scan
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
  S.counters_zero = false;
  if (e == hipSuccess) {
    ScanArgs A = make_args(c, S, 1, group_begin, group_count);
    A.xdump = d_xy;
    const uint32_t blocks = (uint32_t)((A.n_items + kBlock - 1) / kBlock);
    launch_addr(kAddrDump, blocks < c->lanes / kBlock ? blocks : c->lanes / kBlock, S.stream, A);
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
// ------------------------------------------------------------------- second / third check (§8(f)3)
namespace {

void cpts_from_be(khb::CPt* dst, const uint8_t* src, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) {
    fe_from_be(dst[i].x, src + 64 * (size_t)i);
    fe_from_be(dst[i].y, src + 64 * (size_t)i + 32);
  }
}

khb::U8 u8_from_be(const uint8_t* be) {
  Fe f;
  fe_from_be(f, be);
  khb::U8 r;
  memcpy(r.v, f.v, sizeof r.v);
  return r;
}

bool bloom_args_ok(const uint8_t* bf, uint64_t bytes, uint64_t bits, uint32_t hashes) {
  return bf && bytes && bits >= 2 && (bits + 7) / 8 == bytes && hashes && hashes <= 255;   // bloom.cpp:110-113
}

int ensure_check_buffers(khb_ctx* c, uint32_t n, uint32_t n_targets) {
  if (n > c->ck_cap) {
    hipFree(c->d_ck_in);
    hipFree(c->d_ck_out);
    c->d_ck_in = nullptr;
    c->d_ck_out = nullptr;
    c->ck_cap = 0;
    const uint32_t cap = n < 4096 ? 4096 : n;
    KHB_TRY(c, hipMalloc(&c->d_ck_in, sizeof(CheckIn) * cap));
    KHB_TRY(c, hipMalloc(&c->d_ck_out, sizeof(CheckOut) * cap));
    c->ck_cap = cap;
  }
  if (n_targets > c->ck_tcap) {
    c->ck_targets_be.clear();
    hipFree(c->d_ck_targets);
    c->d_ck_targets = nullptr;
    c->ck_tcap = 0;
    const uint32_t cap = n_targets < 256 ? 256 : n_targets;
    KHB_TRY(c, hipMalloc(&c->d_ck_targets, sizeof(khb::CPt) * cap));
    c->ck_tcap = cap;
  }
  return KHB_OK;
}

}  // namespace

int khb_load_check_tables(khb_ctx* c, const khb_check_tables* t) {
  if (!c || !t || !t->gtable || !t->amp2 || !t->amp3 || !t->bptable || t->m3 == 0 || t->m3 > (1ull << 40))
    return KHB_EINVAL;
  if (!bloom_args_ok(t->l2, t->l2_bytes_per_sub, t->l2_bits_per_sub, t->l2_hashes) ||
      !bloom_args_ok(t->l3, t->l3_bytes_per_sub, t->l3_bits_per_sub, t->l3_hashes))
    return KHB_EINVAL;
  KHB_TRY(c, hipSetDevice(c->device));
  auto up = [](size_t v) { return (v + 255) & ~(size_t)255; };
  const size_t n_g = 32 * 256, o_g = 0, o_a2 = up(o_g + sizeof(khb::CPt) * n_g), o_a3 = up(o_a2 + sizeof(khb::CPt) * 32);
  const size_t b2 = 256 * (size_t)t->l2_bytes_per_sub, b3 = 256 * (size_t)t->l3_bytes_per_sub;
  const size_t o_l2 = up(o_a3 + sizeof(khb::CPt) * 32), o_l3 = up(o_l2 + b2), o_bp = up(o_l3 + b3);
  const size_t total = o_bp + 16 * (size_t)t->m3;
  std::vector<uint8_t> h;
  try {
    h.assign(total, 0);
  } catch (const std::bad_alloc&) {
    return KHB_ENOMEM;
  }
  cpts_from_be((khb::CPt*)(h.data() + o_g), t->gtable, (uint32_t)n_g);
  cpts_from_be((khb::CPt*)(h.data() + o_a2), t->amp2, 32);
  cpts_from_be((khb::CPt*)(h.data() + o_a3), t->amp3, 32);
  memcpy(h.data() + o_l2, t->l2, b2);
  memcpy(h.data() + o_l3, t->l3, b3);
  memcpy(h.data() + o_bp, t->bptable, 16 * (size_t)t->m3);
  if (c->ck_stream) KHB_TRY(c, hipStreamSynchronize(c->ck_stream));
  hipFree(c->d_ck);
  c->d_ck = nullptr;
  c->ck_loaded = false;
  KHB_TRY(c, hipMalloc(&c->d_ck, total));
  KHB_TRY(c, hipMemcpy(c->d_ck, h.data(), total, hipMemcpyHostToDevice));
  uint8_t* d = (uint8_t*)c->d_ck;
  khb::CheckTables& T = c->ck;
  T.gtab = (const khb::CPt*)(d + o_g);
  T.amp2 = (const khb::CPt*)(d + o_a2);
  T.amp3 = (const khb::CPt*)(d + o_a3);
  T.l2 = d + o_l2;
  T.l3 = d + o_l3;
  T.bp = d + o_bp;
  T.g2 = bloom_geom(t->l2_bytes_per_sub, t->l2_bits_per_sub, t->l2_hashes);
  T.g3 = bloom_geom(t->l3_bytes_per_sub, t->l3_bits_per_sub, t->l3_hashes);
  T.n_bp = t->m3;
  T.m_double = u8_from_be(t->m_double_be);
  T.m2_double = u8_from_be(t->m2_double_be);
  T.m3 = u8_from_be(t->m3_be);
  T.m3_double = u8_from_be(t->m3_double_be);
  c->ck_loaded = true;
  return KHB_OK;
}

int khb_check(khb_ctx* c, const uint8_t* targets_xy, uint32_t n_targets, const khb_check_in* in, uint32_t n,
              khb_check_out* out) {
  if (!c || (n && (!in || !out)) || (n_targets && !targets_xy)) return KHB_EINVAL;
  if (!c->ck_loaded) return KHB_ESTATE;
  if (n == 0) return KHB_OK;
  for (uint32_t i = 0; i < n; ++i)
    if (in[i].target >= n_targets) return KHB_EINVAL;
  KHB_TRY(c, hipSetDevice(c->device));
  if (!c->ck_stream) {
    int lo = 0, hi = 0;
    KHB_TRY(c, hipDeviceGetStreamPriorityRange(&lo, &hi));
    KHB_TRY(c, hipStreamCreateWithPriority(&c->ck_stream, hipStreamNonBlocking, hi));
  }
  int rc = ensure_check_buffers(c, n, n_targets);
  if (rc) return rc;
  std::vector<CheckIn> hin(n);
  std::vector<CheckOut> hout(n);
  for (uint32_t i = 0; i < n; ++i) {
    hin[i].start = u8_from_be(in[i].start_be);
    hin[i].a = in[i].a;
    hin[i].target = in[i].target;
  }
  KHB_TRY(c, hipMemcpyAsync(c->d_ck_in, hin.data(), sizeof(CheckIn) * n, hipMemcpyHostToDevice, c->ck_stream));
  const size_t tbytes = 64 * (size_t)n_targets;
  const bool same = c->ck_targets_be.size() == tbytes && (tbytes == 0 || !memcmp(c->ck_targets_be.data(), targets_xy, tbytes));
  std::vector<khb::CPt> ht;
  if (!same) {
    ht.resize(n_targets);
    cpts_from_be(ht.data(), targets_xy, n_targets);
    c->ck_targets_be.clear();            // invalid until the upload below has been issued
    KHB_TRY(c, hipMemcpyAsync(c->d_ck_targets, ht.data(), sizeof(khb::CPt) * n_targets, hipMemcpyHostToDevice,
                              c->ck_stream));
    c->ck_targets_be.assign(targets_xy, targets_xy + tbytes);
  }
  launch_check(c->ck_stream, c->ck, c->d_ck_in, c->d_ck_targets, n_targets, c->d_ck_out, n);
  KHB_TRY(c, hipGetLastError());
  KHB_TRY(c, hipMemcpyAsync(hout.data(), c->d_ck_out, sizeof(CheckOut) * n, hipMemcpyDeviceToHost, c->ck_stream));
  KHB_TRY(c, hipStreamSynchronize(c->ck_stream));
  for (uint32_t i = 0; i < n; ++i) {
    Fe k;
    memcpy(k.v, hout[i].key.v, sizeof k.v);
    fe_to_be(out[i].key_be, k);
    out[i].found = hout[i].found;
    out[i].l2_hits = hout[i].l2_hits;
    out[i].l3_hits = hout[i].l3_hits;
    out[i].bp_hits = hout[i].bp_hits;
  }
  return KHB_OK;
}

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
    A.bgeom[l] = bloom_geom(bytes_per_sub[l], bits_per_sub[l], hashes[l]);
  }
  if (e == hipSuccess && bp && m3) {
    e = hipMalloc(&dbp, 16 * m3);
    A.bp = dbp;
  }
  if (e == hipSuccess)
    e = hipMemcpyAsync(S.d_centres, S.h_centres, sizeof(AffPt) * n_jobs, hipMemcpyHostToDevice, S.stream);
  if (e == hipSuccess) e = hipMemsetAsync(S.d_counters, 0, kCounterBytes, S.stream);
  S.counters_zero = false;
  if (e == hipSuccess) e = hipEventRecord(S.ev0, S.stream);
  if (e == hipSuccess) {
    launch_baby(c->lanes / kBlock, S.stream, A);
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
