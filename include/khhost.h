/*
 * khhost.h — C ABI of the host half of the engine, libkhhost.so: keyhunt's BSGS setup and
 * confirmation (keyhunt.cpp:962-1880, 4271-4368) plus the multi-GPU search driver that calls
 * libkhbsgs.so.  The keyhunt_amd CLI is built from the same sources; this ABI exists so tests and
 * bench.py can drive exactly the code the CLI runs.
 *
 * Points and 256-bit values cross as big-endian bytes (x||y for points), like include/khbsgs.h.
 * Functions return 0 on success or a negative KHB_E* code (include/khbsgs.h).
 */
#ifndef KHHOST_H
#define KHHOST_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version of this header; bumped whenever a signature, a struct or an output array changes.
 * A binding checks khh_abi_version() == the KHH_ABI_VERSION it was written for before any other call. */
#define KHH_ABI_VERSION 6
int khh_abi_version(void);

typedef struct khh_tables khh_tables;

/* Geometry + all tables.  n_str: -n value ("0x.." or decimal) or NULL (2^44); k: -k factor;
 * threads: builder threads; gpl: GPU groups per lane (lane-offset table).  NULL on error (err). */
khh_tables* khh_tables_new(const char* n_str, int k, int threads, uint32_t gpl, char* err, size_t errlen);
void khh_tables_free(khh_tables* t);
/* Like khh_tables_new, with -S semantics (keyhunt.cpp:1373-1613, 1881-2025): the reference's table
 * files keyhunt_bsgs_{4,6,2,7}_*.{blm,tbl} are read from dir when present (checksums verified
 * unless skip_checksum), only the missing tables are computed, and with save != 0 the missing ones
 * are written back.  *have receives the mask of files read (1 L1, 2 L2, 4 bPtable, 8 L3). */
khh_tables* khh_tables_new_files(const char* n_str, int k, int threads, uint32_t gpl, const char* dir,
                                 int skip_checksum, int save, uint32_t* have, char* err, size_t errlen);
/* Like khh_tables_new with the baby-step walk on GPU `device` (khb_build_baby); identical tables.
 * *kernel_ms (nullable) receives the build kernel's time. */
khh_tables* khh_tables_new_gpu(const char* n_str, int k, int threads, uint32_t gpl, int device, double* kernel_ms,
                               char* err, size_t errlen);
/* Write all four table files into dir. */
int khh_tables_save(const khh_tables* t, const char* dir, char* err, size_t errlen);
/* out: [0]=m [1]=m2 [2]=m3 [3]=aux [4]=cycles [5]=N(low64) [6]=l1 extent [7..9]=bloom entries L1..L3 */
void khh_params(const khh_tables* t, uint64_t out[10]);
/* level 1..3, sub-bloom idx 0..255: pointer to the bit array; geometry through the out params */
const uint8_t* khh_bloom(const khh_tables* t, int level, int idx, uint64_t* bytes, uint64_t* bits, uint32_t* hashes);
void khh_giant_table(const khh_tables* t, uint8_t out[513 * 64]);
void khh_amp_table(const khh_tables* t, int level, uint8_t out[32 * 64]);
uint32_t khh_lane_offsets(const khh_tables* t, uint8_t* out /* n*64, may be NULL */, uint32_t* gpl);
/* Level-0 gate (khb_load_gate): pointer to 2^log2 / 8 bytes, or NULL with *log2 = 0 when none */
const uint8_t* khh_gate(const khh_tables* t, uint32_t* log2);
/* Gate probes (bits per x, khb_load_gate's probes); 0 when the tables have no gate */
uint32_t khh_gate_probes(const khh_tables* t);
/* bPtable (sorted): m3 records of {6-byte value, 2 pad, u64 index} */
const uint8_t* khh_bptable(const khh_tables* t, uint64_t* n);

/* startP of (chunk base, target): keyhunt.cpp:3861-3869 */
int khh_chunk_centre(const khh_tables* t, const uint8_t base_be[32], const uint8_t target_xy[64], uint8_t out_xy[64]);
/* The search engine's batched centres (engine.cpp job_centres) of n_chunks x n_targets jobs:
 * out[64 * (c * n_targets + j)] = centre of chunk bases[c] for target j (what khh_chunk_centre gives
 * one at a time); consecutive bases (2N apart) take the batched auxiliary walk. */
int khh_job_centres(const khh_tables* t, const uint8_t* bases_be, uint32_t n_chunks, const uint8_t* targets_xy,
                    uint32_t n_targets, uint8_t* out_xy, int threads);
/* bsgs_secondcheck: 1 found (key_be filled), 0 not found */
int khh_secondcheck(const khh_tables* t, const uint8_t base_be[32], uint32_t a, const uint8_t target_xy[64],
                    uint8_t key_be[32]);

/* Multi-GPU search over [start, end): found[k] (0/1) and keys[k] (32 B BE) per target.
 * devices: n_devices device ordinals.  stats_out (nullable): [0]=chunks [1]=giant steps
 * [2]=candidates [3]=degenerate groups [4]=kernel microseconds [5]=scan launches (stats_out holds 6). */
int khh_search(const khh_tables* t, const uint8_t* targets_xy, int n_targets, const uint8_t start_be[32],
               const uint8_t end_be[32], const int* devices, int n_devices, uint32_t lanes,
               uint32_t chunks_per_batch, uint64_t max_chunks, int* found, uint8_t* keys_be, uint64_t* stats_out,
               char* err, size_t errlen);

/* Persistent multi-GPU session: contexts opened and tables resident in HBM once, then any number
 * of searches.  khh_session_run writes the 6 stats entries of khh_search (stats_out holds 6).
 * khh_session_run_ex writes the first min(stats_len, KHH_SESSION_STATS) of: those 6, [6]=launches
 * rescanned in parts after a candidate-ring overflow, [7]=device-busy microseconds (union of each
 * device's launch intervals, summed over devices; two launches in flight overlap, so [7] <= [4]),
 * [8]=average shader clock of the launches in kHz, [9]=candidates confirmed on the GPU (khb_check),
 * [10]=microseconds spent in those khb_check calls, [11]=the launches' summed HIP-event microseconds
 * (khb_stats.event_ms: dispatch to end, what rocprofv3's kernel trace reports; [4] sums their execution
 * spans, khb_stats.kernel_ms). */
#define KHH_SESSION_STATS 12
typedef struct khh_session khh_session;
khh_session* khh_session_open(const khh_tables* t, const int* devices, int n_devices, uint32_t lanes,
                              uint32_t chunks_per_batch, int check_threads, char* err, size_t errlen);
int khh_session_run(khh_session* s, const uint8_t* targets_xy, int n_targets, const uint8_t start_be[32],
                    const uint8_t end_be[32], uint64_t max_chunks, int random_chunks, int* found, uint8_t* keys_be,
                    uint64_t* stats_out, char* err, size_t errlen);
int khh_session_run_ex(khh_session* s, const uint8_t* targets_xy, int n_targets, const uint8_t start_be[32],
                       const uint8_t end_be[32], uint64_t max_chunks, int random_chunks, int* found, uint8_t* keys_be,
                       uint64_t* stats_out, uint32_t stats_len, char* err, size_t errlen);
void khh_session_close(khh_session* s);
/* Test hooks: candidate ring capacity per launch (0 = default 2^20; small values drive the
 * split-and-rescan path), the level-0 gate on/off, recording of every level-1 candidate of the next
 * runs (khh_session_recorded), and optionally a replacement level-1 bloom of the tables' geometry
 * (256 sub-blooms concatenated; NULL keeps the tables'). */
int khh_session_set_test_hooks(khh_session* s, uint32_t cand_cap, int use_gate, int record, const uint8_t* l1_concat);
/* Where later runs confirm their level-1 candidates (bsgs_secondcheck/thirdcheck, keyhunt.cpp:4271-4368):
 * 0 = the host's CPU pool (default), 1 = the GPU that scanned them (khb_check; the check tables are
 * loaded into every context), 2 = the GPU for batches of more than 4096 candidates, else the host. */
#define KHH_CHECK_HOST 0
#define KHH_CHECK_DEVICE 1
#define KHH_CHECK_AUTO 2
int khh_session_set_check_mode(khh_session* s, int mode);
/* keyhunt's -B mode for later runs (keyhunt.cpp:227): 0 sequential, 1 backward, 2 both, 3 random, 4 dance
 * (the thread_process_bsgs* variants, 3778-5700; engine.hpp ChunkCursor).  A run's random_chunks != 0
 * still selects random. */
int khh_session_set_chunk_mode(khh_session* s, int mode);
/* The chunk bases a -B mode claims from [start, end) with chunks of two_n keys, in claim order, up to cap
 * (out: 32 B BE each); the seed drives both / dance.  Returns the count (the whole sequence unless cap is
 * reached or the mode is random).  Host only: the claim order the search uses. */
uint64_t khh_chunk_sequence(int mode, const uint8_t start_be[32], const uint8_t end_be[32], const uint8_t two_n_be[32],
                            uint64_t seed, uint8_t* out_be, uint64_t cap);
/* Secp256K1::Init's GTable (secp256k1/SECP256K1.cpp:43-54), 32*256 points x||y BE (khb_check_tables.gtable). */
void khh_gtable(uint8_t out[32 * 256 * 64]);
/* Candidates recorded in the last run: chunk base (32 B BE), target index, giant step a; returns the
 * count (may exceed cap). */
uint64_t khh_session_recorded(const khh_session* s, uint8_t* bases_be, uint32_t* targets, uint32_t* a, uint64_t cap);

/* helpers */
int khh_pubkey(const uint8_t key_be[32], uint8_t out_xy[64]);
int khh_parse_pubkey(const char* hex, uint8_t out_xy[64], int* compressed);

/* ---- -m address / -m rmd160 (BTC P2PKH) ----
 * Targets from a target file's text (base58 addresses or 40-hex rmd160 lines, keyhunt.cpp:6300-6358).
 * The generator (Gn table + lane offsets for chunks of n_seq keys) is built for stride and gpl. */
typedef struct khh_addr khh_addr;
khh_addr* khh_addr_new(const char* text, int bloom_multiplier, const uint8_t stride_be[32], uint64_t n_seq,
                       uint32_t gpl, int threads, char* err, size_t errlen);
void khh_addr_free(khh_addr* a);
/* sorted 20-byte table (n entries) and the target bloom */
const uint8_t* khh_addr_table(const khh_addr* a, uint64_t* n);
const uint8_t* khh_addr_bloom(const khh_addr* a, uint64_t* bytes, uint64_t* bits, uint32_t* hashes);
void khh_addr_giant_table(const khh_addr* a, uint8_t out[513 * 64]);
uint32_t khh_addr_lane_offsets(const khh_addr* a, uint8_t* out /* n*64, may be NULL */, uint32_t* gpl);
/* Sequential (random_chunks = 0) or -R search of [start, end) with search 0/1/2 (-l), OR'ed with
 * KHB_SEARCH_ENDOMORPHISM (4, include/khbsgs.h) for -e: the found keys are then lambda^e multiples too.  Found keys
 * (32 B BE each) with compressed flags and rmd160s, in discovery order; *n_found may exceed cap.
 * Discovery order is batch order, and (chunk, key) order inside a batch, except after an overflow: a batch
 * whose bloom hits overflowed khb_addr_hit_capacity is rescanned in parts queued behind the batch already
 * submitted after it, so its keys are reported after that later batch's (the bsgs session reorders its
 * candidates the same way).  Callers that need range order sort the keys.
 * stats_out (nullable): [0]=chunks [1]=keys [2]=bloom hits [3]=degenerate groups [4]=kernel us
 * [5]=launches; khh_addr_search writes these 6.  khh_addr_search_ex writes the first
 * min(stats_len, KHH_ADDR_STATS) of them and [6]=average shader clock of the launches in kHz,
 * [7]=rescans (launches whose bloom hits overflowed khb_addr_hit_capacity and were rescanned in parts). */
#define KHH_ADDR_STATS 8
int khh_addr_search(const khh_addr* a, const uint8_t start_be[32], const uint8_t end_be[32], int search,
                    int random_chunks, const int* devices, int n_devices, uint32_t lanes, uint64_t max_chunks,
                    uint8_t* keys_be, uint8_t* compressed, uint8_t* rmd, uint32_t cap, uint32_t* n_found,
                    uint64_t* stats_out, char* err, size_t errlen);
int khh_addr_search_ex(const khh_addr* a, const uint8_t start_be[32], const uint8_t end_be[32], int search,
                       int random_chunks, const int* devices, int n_devices, uint32_t lanes, uint64_t max_chunks,
                       uint8_t* keys_be, uint8_t* compressed, uint8_t* rmd, uint32_t cap, uint32_t* n_found,
                       uint64_t* stats_out, uint32_t stats_len, char* err, size_t errlen);
/* Tests: bloom-hit ring capacity of the search's launches (0 = the library default, 2^18). */
int khh_addr_set_hit_capacity(khh_addr* a, uint32_t cap);
/* The host confirmation of one GPU bloom hit (khb_addr_hit.kind = form | e << 2) of the point with key key_be:
 * searchbinary of the hash the kind names, then the reference's key recovery (keyhunt.cpp:2789-2937; lambda^e * key,
 * negated for the other point of a compressed x or for form 3).  Returns 1 and the key / compressed flag when the
 * hash is a target, 0 when it is not. */
int khh_addr_confirm(const khh_addr* a, const uint8_t key_be[32], uint32_t kind, uint8_t out_key_be[32],
                     int* compressed);
/* hash160 of a public key (x||y BE) and its P2PKH address (out_addr >= 36 bytes) */
void khh_hash160(const uint8_t xy[64], int compressed, uint8_t out[20]);
void khh_rmd_to_address(const uint8_t rmd[20], char* out_addr);

#ifdef __cplusplus
}
#endif
#endif
