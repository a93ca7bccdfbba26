/*
 * khbsgs.h — C ABI of the MI355X (gfx950) BSGS giant-step library, libkhbsgs.so.
 *
 * This is the drop-in boundary for keyhunt's GPU path.  It replaces the reference's unwired
 * CUDA surface (cuda/bsgs_kernel.cu:230-319: cudaInit, cudaAllocateBSGSMemory,
 * cudaCopyToDevice, cudaLaunchBSGS, cudaCopyFromDevice, cudaFreeMemory) and takes over exactly
 * the CPU work of keyhunt.cpp:3867-4004 — the per-(chunk, target) giant-step group loop of
 * thread_process_bsgs with its level-1 bloom probe.  Candidates it returns feed the host's
 * bsgs_secondcheck (keyhunt.cpp:3948 -> 4271-4368), unchanged.
 *
 * Conventions
 *   - Every function returns 0 (KHB_OK) or a negative KHB_E* code; khb_strerror() names it.
 *     The library never prints.
 *   - One context per device; a context is used by one host thread at a time.  Distinct
 *     contexts are independent (thread-safe across devices).
 *   - 256-bit field elements and points cross the boundary big-endian: a point is x||y, 64 bytes,
 *     each coordinate Int::Get32Bytes order (secp256k1/Int.cpp:308-316).
 *   - The caller keeps ownership of every host buffer; tables are copied into device memory.
 *   - Missing or non-gfx950 GPU: khb_open fails with KHB_ENODEV.  There is no CPU fallback.
 */
#ifndef KHBSGS_H
#define KHBSGS_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KHB_OK 0
#define KHB_EINVAL -1     /* bad argument / shape */
#define KHB_ENODEV -2     /* no usable gfx950 device */
#define KHB_ENOMEM -3     /* device or pinned allocation failed */
#define KHB_EHIP -4       /* HIP runtime error (khb_last_hip_error() has the hipError_t) */
#define KHB_ESTATE -5     /* call order violated (e.g. scan before tables are loaded) */
#define KHB_EBUSY -6      /* a submission is still in flight */
#define KHB_EINCOMPLETE -7 /* collect: the groups the kernel counted as walked differ from the submitted
                             n_jobs x group_count (a work-item bookkeeping fault; results incomplete) */
#define KHB_EHANDOFF -8    /* collect: the launch's end-of-launch hand-off (the last wave's copy of the counters
                             to pinned host memory) did not count every wave; khb_last_handoff has the counts */

#define KHB_GROUP 1024         /* giant steps per group: CPU_GRP_SIZE, keyhunt.cpp:127 */
#define KHB_GIANT_TABLE 513    /* GSn[0..511] + _2GSn, keyhunt.cpp:1318-1338 */

/* ABI version of this header (entry points, khb_stats and the other structs); bumped whenever one of
 * them changes.  A binding checks khb_abi_version() == the KHB_ABI_VERSION it was written for before
 * any other call (khb_stats gained launch_begin_ms/launch_end_ms/shader_mhz in ABI 3 and 4; ABI 5 added
 * khb_load_check_tables / khb_check; ABI 6 added khb_stats.event_ms; ABI 7 added khb_build_info,
 * khb_set_gate_stage0 / khb_gate_stages, KHB_EHANDOFF / khb_last_handoff and the -m address endomorphism
 * (KHB_SEARCH_ENDOMORPHISM, khb_addr_hit.kind = form | e << 2)). */
#define KHB_ABI_VERSION 7
int khb_abi_version(void);
/* What this library was built as, one line of `key=value` words: abi, arch, variant ("product" for the in-tree
 * build; tools/build_variant.sh names its timing builds), the kernel's build defines (waves per SIMD, groups per
 * work item, gate stages, half prefix stream, extra -D flags) and the compiler.  A bench line records it, so a
 * number can always be traced to the kernel that produced it. */
const char* khb_build_info(void);

typedef struct khb_ctx khb_ctx;

/* One level-1 bloom hit: giant step `a` (= group*1024 + t, keyhunt.cpp:3948) of job `job`. */
typedef struct {
  uint32_t job;
  uint32_t a;
} khb_cand;

/* A group whose batch inverse collapsed (some dx == 0: the target sits exactly on a window
 * centre, SURVEY.md §8a quirk ii).  Reported so the host can mirror the reference. */
typedef struct {
  uint32_t job;
  uint32_t group;
} khb_degenerate;

typedef struct {
  uint32_t n_cand;         /* total hits (may exceed the capacity given to khb_collect, and the ring's
                              capacity khb_candidate_capacity(): then only that many were kept, and the
                              caller rescans the submission in parts -- SURVEY.md §8b) */
  uint32_t n_degenerate;
  uint64_t giant_steps;    /* giant steps the device walked (counted on the device: groups x 1024) */
  float kernel_ms;         /* the scan kernel's execution span: from its first workgroup's start to its last
                              wave's exit on the device's 100 MHz clock (s_memrealtime; khb_submit /
                              khb_addr_submit), capped by the submission's HIP events, which also count the
                              time a queued launch waits for CUs behind the other slot's launch */
  double launch_begin_ms;  /* the launch's begin and end on the context's clock: ms since the last
                              khb_reset_epoch (or khb_open); end = the submission's end event, begin = end -
                              kernel_ms; -1 if unavailable.  Two submissions in flight */
  double launch_end_ms;    /* overlap, so the union of these intervals is the device-busy time. */
  float shader_mhz;        /* average shader clock of block 0's first wave over its lifetime (s_memtime /
                              s_memrealtime at its start and at its exit; s_memtime counts per XCD, so one
                              wave's own interval is the one that can be timed), 0 if unavailable */
  float event_ms;          /* the submission's HIP-event time, dispatch to end: the launch duration
                              rocprofv3 --kernel-trace reports (>= kernel_ms; with two submissions in flight
                              it includes the wait behind the other slot's launch), -1 if unavailable */
} khb_stats;

/* ---- device / context ---- */
int khb_device_count(int* n);
/* lanes: persistent-grid size in work lanes (0 = auto: one full residency of the kernel,
 * CUs x 4 SIMDs x waves-per-SIMD x 64).  Sizes the scratch. */
int khb_open(int device, uint32_t lanes, khb_ctx** out);
int khb_close(khb_ctx* ctx);
const char* khb_strerror(int code);
int khb_last_hip_error(const khb_ctx* ctx);
/* After KHB_EHANDOFF: the waves the last collected launch's epilogue counted, and the launch's wave total. */
int khb_last_handoff(const khb_ctx* ctx, uint32_t* waves_seen, uint32_t* waves_total);
/* The hipStream_t the context launches on (for external HIP events / synchronisation). */
void* khb_stream(khb_ctx* ctx);
/* Persistent-grid size of the context in work lanes (one lane = one work item at a time). */
uint32_t khb_lanes(const khb_ctx* ctx);
/* The auto lane count khb_open(device, 0, ...) would choose (0 if the device is unusable). */
uint32_t khb_default_lanes(int device);
/* Groups per work item of the -m bsgs scan (khb_submit / khb_dump_x): a lane walks this many
 * consecutive groups of one job with two field inversions in total, so a launch fills the device
 * when n_jobs * ceil(group_count / khb_groups_per_item()) >= khb_lanes(ctx). */
uint32_t khb_groups_per_item(void);
/* Allocate the device state of the first `depth` submission slots now (1 or 2; a slot's prefix scratch
 * is 4,120 x 32 B x khb_lanes(ctx): ~35 GB at the auto 262,144 lanes on MI355X) instead of on the first queued submission.  KHB_ENOMEM leaves the
 * extra slot empty and the context usable with one submission in flight (the caller's queue depth 1). */
int khb_reserve_slots(khb_ctx* ctx, int depth);
/* Candidate ring entries a -m bsgs launch keeps (default and maximum 2^20).  Lowering it is for tests
 * of the caller's overflow path (stats.n_cand > capacity -> rescan in parts). */
int khb_set_candidate_capacity(khb_ctx* ctx, uint32_t cap);
uint32_t khb_candidate_capacity(const khb_ctx* ctx);
/* Bloom-hit ring entries a -m address launch keeps: min(khb_candidate_capacity, 2^18).  As for the
 * candidates, stats.n_cand > capacity means "rescan the submission in parts" (every hit must reach
 * the host's searchbinary, keyhunt.cpp:2716-2937). */
uint32_t khb_addr_hit_capacity(const khb_ctx* ctx);
/* Restart the context's clock (khb_stats.launch_begin_ms / launch_end_ms); KHB_EBUSY while a
 * submission is in flight. */
int khb_reset_epoch(khb_ctx* ctx);

/* ---- tables (bsgs setup, keyhunt.cpp:1185-1364) ---- */
/* Level-1 bloom: 256 sub-blooms of identical geometry concatenated in sub-bloom order
 * (bloom_bP[0..255].bf, bloom.h:26-45).  bits/hashes as in struct bloom. */
int khb_load_bloom(khb_ctx* ctx, const uint8_t* bf_concat, uint64_t bytes_per_sub, uint64_t bits_per_sub,
                   uint32_t hashes);
/* Level-0 gate in front of the level-1 probe (no reference counterpart; a superset filter): a
 * blocked bloom filter of 2^log2_bits bits in 64-bit blocks (block i = bytes 8i..8i+7, bit b of
 * the block = bit b%8 of byte 8i + b/8).  With x the canonical x-coordinate as an integer,
 * w0 = x mod 2^32 and w1 = (x >> 32) mod 2^32, x selects block w0 mod 2^(log2_bits-6) and within
 * it, for p < probes, bit 32 (p mod 2) + ((w1 >> 5p) mod 32) (probes 0 and 2 in the block's low
 * word, probe 1 in its high word); every baby-step x of the level-1 set has its bits set
 * (khb_build_baby writes one).  With a gate, the giant-step probe reads x's block (one 8-byte
 * load) and runs the level-1 check (both XXH64, all bits) only when all its bits are set: every
 * level-1 candidate that passes the gate is still reported, so no baby-step hit is lost.
 * gate NULL removes it; log2_bits in [13, 32]; probes in [1, KHB_GATE_MAX_PROBES]. */
#define KHB_GATE_MAX_PROBES 3
int khb_load_gate(khb_ctx* ctx, const uint8_t* gate, uint32_t log2_bits, uint32_t probes);
/* Stage-1 fold for gates loaded after this call: a gate larger than 2^log2_bytes bytes is also kept
 * OR-folded to 2^log2_bytes bytes (block i of the fold = OR of the gate's blocks j with
 * j mod (2^log2_bytes / 8) == i).  x tests its block of the fold first and reads its block of the
 * full gate only when those bits are all set: the same candidates, and most tests served by a fold
 * small enough for the L2 (k = 1) or by one that fits the Infinity Cache beside the level-1 bloom
 * (k >= 4).  0 = no stage 1; otherwise log2_bytes in [10, 31], or KHB_GATE_STAGE1_AUTO (the default):
 * 2 MiB for a gate of up to 32 MiB (k = 1), 32 MiB for a larger one (k >= 4). */
#define KHB_GATE_STAGE1_AUTO 1
int khb_set_gate_stage1(khb_ctx* ctx, uint32_t log2_bytes);
/* Stage-0 filter for gates loaded after this call, in front of a stage-1 fold: the hi words of the gate's blocks
 * (probe 1's bit of every member) OR-folded to 2^log2_bytes bytes of 32-bit words (word i = OR of the hi words of
 * blocks j with j mod (2^log2_bytes / 4) == i).  x tests bit (w1 >> 5) mod 32 of word w0 mod (2^log2_bytes / 4)
 * and reads its block of the fold only when it is set: one bit per member, so the same candidates.  Built only
 * with probes >= 2 and a fold larger than the filter.  0 (the default) = no stage 0; otherwise log2_bytes in
 * [10, 30], or KHB_GATE_STAGE0_AUTO: 2 MiB in front of a fold larger than 2 MiB (k >= 4), none otherwise.  The
 * default is off because the filter measured 4.6 % slower on config C (k = 4): the extra per-x load costs more
 * memory-pipeline cycles than the fold reads it saves. */
#define KHB_GATE_STAGE0_AUTO 1
int khb_set_gate_stage0(khb_ctx* ctx, uint32_t log2_bytes);
/* The gate stages the loaded gate runs with: bit 2 the gate, bit 1 its stage-1 fold, bit 0 the stage-0 filter. */
int khb_gate_stages(const khb_ctx* ctx);
/* GSn[0..511] and _2GSn (keyhunt.cpp:1325-1338), 513 affine points x||y BE. */
int khb_load_giant_table(khb_ctx* ctx, const uint8_t* gsn_xy_be);
/* Lane start offsets: offs[m] = (m*groups_per_lane) * _2GSn, m in [0, n) (offs[0] unused: the
 * identity).  A lane owns groups [m*groups_per_lane, (m+1)*groups_per_lane) of a job. */
int khb_load_lane_offsets(khb_ctx* ctx, const uint8_t* offs_xy_be, uint32_t n, uint32_t groups_per_lane);

/* ---- scan ---- */
/* Enqueue the group loop for n_jobs jobs.  centres[k] (x||y BE) is startP of job k, i.e.
 * target + (order - base - (2M*512 + M))*G (keyhunt.cpp:3861-3869), the centre of group 0.
 * Every job scans groups [group_begin, group_begin + group_count); group_begin must be a
 * multiple of groups_per_lane.  Returns immediately (stream-ordered).  A context has two submission
 * slots, each on its own stream: two submissions may be in flight (their launches overlap), a third
 * returns KHB_EBUSY until khb_collect retires one. */
int khb_submit(khb_ctx* ctx, const uint8_t* centres_xy_be, uint32_t n_jobs, uint32_t group_begin,
               uint32_t group_count);
/* Wait for the OLDEST submission in flight (FIFO) and retire it; copy up to cap of its candidates
 * (unordered) and degenerate-group records.  stats may be NULL.  KHB_EINCOMPLETE: the device's count of
 * walked groups differs from the submission. */
int khb_collect(khb_ctx* ctx, khb_cand* cand, uint32_t cap, khb_degenerate* degen, uint32_t degen_cap,
                khb_stats* stats);
/* Convenience: submit + collect.  KHB_EBUSY if any submission is in flight (the collect would retire
 * that one, not this). */
int khb_scan(khb_ctx* ctx, const uint8_t* centres_xy_be, uint32_t n_jobs, uint32_t group_begin,
             uint32_t group_count, khb_cand* cand, uint32_t cap, khb_stats* stats);

/* ---- second / third check on the device ----
 * bsgs_secondcheck + bsgs_thirdcheck (keyhunt.cpp:4271-4368) for a batch of level-1 candidates, one
 * device lane each: base = start + a*BSGS_M_double, Q = target - base*G, the 32 points Q + BSGS_AMP2[i]
 * into the level-2 bloom; for each hit i the third check on base + i*BSGS_M2_double with BSGS_AMP3, the
 * level-3 bloom, bsgs_searchbinary over bPtable (3748-3773, its exact probe order) and the key
 * verification by ComputePublicKey; calcualteindex (6680-6689).  It replaces the host loop the
 * candidates feed at keyhunt.cpp:3947-3982; the found key equals the reference's.
 * Tables are copied to the device by khb_load_check_tables: */
typedef struct {
  const uint8_t* gtable;            /* 32*256 points x||y BE, secp->GTable of Secp256K1::Init
                                       (secp256k1/SECP256K1.cpp:43-54): entry 256*i + b - 1 = b * 2^(8i) * G,
                                       b in 1..255 (entry 256*i + 255 is not read) */
  const uint8_t* amp2;              /* BSGS_AMP2[0..31] x||y BE (keyhunt.cpp:1339-1350) */
  const uint8_t* amp3;              /* BSGS_AMP3[0..31] x||y BE (keyhunt.cpp:1352-1363) */
  const uint8_t* l2;                /* bloom_bPx2nd[0..255].bf concatenated (one geometry, as khb_load_bloom) */
  uint64_t l2_bytes_per_sub, l2_bits_per_sub;
  uint32_t l2_hashes;
  const uint8_t* l3;                /* bloom_bPx3rd[0..255].bf concatenated */
  uint64_t l3_bytes_per_sub, l3_bits_per_sub;
  uint32_t l3_hashes;
  const uint8_t* bptable;           /* bPtable: m3 x struct bsgs_xvalue (16 B: value[6], 2 pad, uint64 index LE),
                                       sorted as bsgs_sort leaves it */
  uint64_t m3;                      /* bsgs_m3 */
  uint8_t m_double_be[32];          /* BSGS_M_double */
  uint8_t m2_double_be[32];         /* BSGS_M2_double */
  uint8_t m3_be[32];                /* BSGS_M3 */
  uint8_t m3_double_be[32];         /* BSGS_M3_double */
} khb_check_tables;
int khb_load_check_tables(khb_ctx* ctx, const khb_check_tables* tables);

typedef struct {
  uint8_t start_be[32];             /* start_range of bsgs_secondcheck: the chunk's base (BSGS_CURRENT) */
  uint32_t a;                       /* the candidate's giant step (khb_cand.a) */
  uint32_t target;                  /* index into targets_xy */
} khb_check_in;
typedef struct {
  uint8_t key_be[32];               /* the private key when found */
  uint32_t found;                   /* bsgs_secondcheck's return value (0 or 1) */
  uint32_t l2_hits;                 /* level-2 bloom hits (third checks run) */
  uint32_t l3_hits;                 /* level-3 bloom hits in those third checks */
  uint32_t bp_hits;                 /* bPtable matches (each verified by ComputePublicKey) */
} khb_check_out;
/* Synchronous; runs on the context's own check stream (high priority), so it may be called while scan
 * submissions are in flight: its lanes take the CU slots the running launch's last waves free.
 * targets_xy: n_targets points x||y BE (OriginalPointsBSGS).  KHB_ESTATE before khb_load_check_tables. */
int khb_check(khb_ctx* ctx, const uint8_t* targets_xy, uint32_t n_targets, const khb_check_in* in, uint32_t n,
              khb_check_out* out);

/* ---- parity / debug ---- */
/* x-coordinates (BE, probe order t = 0..1023 per group) of groups [group_begin,
 * group_begin+group_count) of ONE job; xs must hold group_count*1024*32 bytes, canonical. */
int khb_dump_x(khb_ctx* ctx, const uint8_t* centre_xy_be, uint32_t group_begin, uint32_t group_count,
               uint8_t* xs);
/* Field self-test kernel: r[i] = op(a[i], b[i]) mod p, canonical, for op 0=mul 1=sqr 2=add 3=sub
 * 4=inv 5=lazy add (a < p, b < 2^256) 6=a^2 + b (the fused squaring, a, b < 2^256); 32-byte BE
 * values. */
int khb_field_op(khb_ctx* ctx, int op, const uint8_t* a, const uint8_t* b, uint8_t* r, uint32_t n);
/* Bloom self-test kernel: hit[i] = bloom_check(level-1, x[i]) for 32-byte BE x values. */
int khb_probe(khb_ctx* ctx, const uint8_t* xs, uint8_t* hit, uint32_t n);

/* ---- -m address / -m rmd160 (keyhunt.cpp:2586-2937, BTC P2PKH, with or without -e) ----
 * The same group walk with the table Gn[i] = (i+1)*stride*G, _2Gn = 1024*stride*G loaded through
 * khb_load_giant_table (init_generator, keyhunt.cpp:4386-4399), lane offsets as above.  A job is
 * one claimed chunk; centres[k] = pubkey(chunk_base_k + 512*stride) (keyhunt.cpp:2587-2589), so
 * point t of group j of job k is the key chunk_base_k + (1024*j + t)*stride. */
typedef struct {
  uint32_t job;
  uint32_t group;
  uint32_t t;
  uint32_t kind;     /* form | e << 2.  form: 0 = compressed prefix 02, 1 = compressed prefix 03, 2 = uncompressed
                        (x, y), 3 = uncompressed (x, p - y), the negated point (-e only).  e: the point itself (0),
                        or with -e (beta*x, y) = lambda*P (1) and (beta^2*x, y) = lambda^2*P (2), keyhunt.cpp:2646-2763.
                        Without -e kind is 0, 1 or 2 as before. */
} khb_addr_hit;

/* The single target bloom of -m address (bloom over 20-byte hash160 values, initBloomFilter,
 * keyhunt.cpp:6559-6576). */
int khb_load_addr_bloom(khb_ctx* ctx, const uint8_t* bf, uint64_t bytes, uint64_t bits, uint32_t hashes);
/* search: 0 = uncompress, 1 = compress, 2 = both (keyhunt.cpp:59-61, -l), optionally OR'ed with
 * KHB_SEARCH_ENDOMORPHISM (-e, keyhunt.cpp:579-585, 2646-2763): per point also beta*x and beta^2*x (compressed:
 * 6 hashes per point) and, for uncompressed keys, the negated points (6 hashes per point).  Every point's
 * hash160(s) are probed in the bloom; bloom hits are returned (the host runs searchbinary and the key
 * recovery: lambda^e * key, negated as the hit's form says).  group_begin must be a multiple of groups_per_lane.
 * Submissions share the context's two slots with khb_submit (two in flight, FIFO collect, a third returns
 * KHB_EBUSY). */
#define KHB_SEARCH_ENDOMORPHISM 4
int khb_addr_submit(khb_ctx* ctx, const uint8_t* centres_xy_be, uint32_t n_jobs, uint32_t group_begin,
                    uint32_t group_count, int search);
/* stats->n_cand = number of bloom hits (may exceed cap); giant_steps = keys scanned. */
int khb_addr_collect(khb_ctx* ctx, khb_addr_hit* hits, uint32_t cap, khb_stats* stats);
int khb_addr_scan(khb_ctx* ctx, const uint8_t* centres_xy_be, uint32_t n_jobs, uint32_t group_begin,
                  uint32_t group_count, int search, khb_addr_hit* hits, uint32_t cap, khb_stats* stats);
/* parity: x||y (64 bytes BE per point, t = 0..1023 per group) of ONE job. */
int khb_addr_dump(khb_ctx* ctx, const uint8_t* centre_xy_be, uint32_t group_begin, uint32_t group_count,
                  uint8_t* xy);
/* self-test: out[21*i] = hash160 (20 bytes) of point i (x||y BE) for kind 0/1/2, then one byte =
 * bloom_check20 result against the loaded address bloom (0 when none is loaded). */
int khb_hash160(khb_ctx* ctx, int kind, const uint8_t* xy_be, uint8_t* out, uint32_t n);

/* ---- baby-step tables on the GPU (thread_bPload, keyhunt.cpp:4404-4592; orchestration 1615-1880) ----
 * Uses the loaded giant table as Gn[i] = (i+1)*G, _2Gn = 1024*G and the lane offsets for jobs of
 * groups_per_job groups.  Job k covers baby steps ic = k*groups_per_job*1024 + [0, groups_per_job*1024)
 * (key ic + 1); centres[k] = pubkey(k*groups_per_job*1024 + 513).  Every x with ic < l1ext is added
 * to the level-1 bloom, ic < m2 to level 2, ic < m3 to level 3 and written to bp as struct
 * bsgs_xvalue {x bytes 16..21, 2 zero bytes, u64 ic} (unsorted).  l1/l2/l3 receive 256 concatenated
 * sub-blooms of bytes_per_sub[level] bytes (NULL skips a level, e.g. one read from -S files);
 * bp receives m3*16 bytes (NULL skips it).  gate (NULL skips it) receives the level-0 gate of
 * khb_load_gate for every ic < l1ext, 2^gate_log2 bits, gate_probes bits per x. */
int khb_build_baby(khb_ctx* ctx, const uint8_t* centres_xy_be, uint32_t n_jobs, uint32_t groups_per_job,
                   uint64_t l1ext, uint64_t m2, uint64_t m3, const uint64_t bytes_per_sub[3],
                   const uint64_t bits_per_sub[3], const uint32_t hashes[3], uint8_t* l1, uint8_t* l2, uint8_t* l3,
                   uint8_t* bp, uint8_t* gate, uint32_t gate_log2, uint32_t gate_probes, float* kernel_ms);

#ifdef __cplusplus
}
#endif
#endif
