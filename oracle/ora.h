/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference keyhunt `-m bsgs` hot path, used as the parity checker
 * for the MI355X engine. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this code; the product (libkhbsgs.so, keyhunt_amd, libkhhost.so) never links it.
 *
 * Every function cites the reference file:line it restates (paths relative to the reference
 * checkout consigcody94/keyhuntM1CPU).  Parity pins: SURVEY.md §8c — BSGSD.md:35-36/80 (puzzle 63
 * -> 7cce5efdaccf6808), the puzzle-30 smoke known answer (3d94cd64), self-certifying puzzle keys
 * from tests/1to63_65.txt, published XXH64 vectors.  Running the compiled reference was denied
 * (SURVEY.md §8c), so the oracle is pinned by those fixtures, not by reference binaries.
 */
#ifndef ORA_H
#define ORA_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 256-bit unsigned integer, little-endian 64-bit limbs (restates the low four limbs of Int,
 * secp256k1/Int.h:178-181; the hot path never sets the fifth limb). */
typedef struct { uint64_t w[4]; } ora_u256;
typedef struct { ora_u256 x, y, z; } ora_point;

/* ---- 256-bit integer helpers ---- */
int      ora_u256_cmp(const ora_u256* a, const ora_u256* b);
uint64_t ora_u256_add(ora_u256* r, const ora_u256* a, const ora_u256* b);   /* returns carry  */
uint64_t ora_u256_sub(ora_u256* r, const ora_u256* a, const ora_u256* b);   /* returns borrow */
void     ora_u256_set64(ora_u256* r, uint64_t v);
int      ora_u256_is_zero(const ora_u256* a);
void     ora_u256_mul64(ora_u256* r, const ora_u256* a, uint64_t m);        /* mod 2^256      */
int      ora_u256_from_hex(ora_u256* r, const char* hex);                   /* 0 ok           */
void     ora_u256_to_hex(const ora_u256* a, char out[65]);                  /* lowercase, no leading zeros (Int.cpp:1019-1057) */
void     ora_u256_to_be(const ora_u256* a, uint8_t out[32]);                /* Int::Get32Bytes (Int.cpp:308-316) */
void     ora_u256_from_be(ora_u256* r, const uint8_t in[32]);

/* ---- field Fp, reference semantics (secp256k1/IntMod.cpp) ---- */
void ora_fe_add(ora_u256* r, const ora_u256* a, const ora_u256* b);   /* IntMod.cpp:51-57   */
void ora_fe_sub(ora_u256* r, const ora_u256* a, const ora_u256* b);   /* IntMod.cpp:97-101  */
void ora_fe_neg(ora_u256* r, const ora_u256* a);                      /* IntMod.cpp:105-108 */
void ora_fe_mulK1(ora_u256* r, const ora_u256* a, const ora_u256* b); /* IntMod.cpp:855-915 */
void ora_fe_sqrK1(ora_u256* r, const ora_u256* a);                    /* IntMod.cpp:977-1093 */
void ora_fe_inv(ora_u256* r, const ora_u256* a);                      /* IntMod.cpp:112-513 (result: canonical inverse, 0 if none) */
void ora_fe_mul_exact(ora_u256* r, const ora_u256* a, const ora_u256* b); /* canonical a*b mod p (Montgomery ModMul, IntMod.cpp:655+) */
void ora_fe_pow(ora_u256* r, const ora_u256* a, const ora_u256* e);
int  ora_fe_has_sqrt(const ora_u256* a);                              /* Int::HasSqrt IntMod.cpp:563-574 */
void ora_fe_sqrt(ora_u256* r, const ora_u256* a);                     /* Int::ModSqrt IntMod.cpp:578-652 (p = 3 mod 4 branch) */

/* ---- secp256k1 group (secp256k1/SECP256K1.cpp) ---- */
void ora_secp_init(void);                                             /* SECP256K1.cpp:29-56 */
void ora_compute_pubkey(ora_point* r, const ora_u256* k);             /* SECP256K1.cpp:61-82 */
void ora_add_direct(ora_point* r, const ora_point* p1, const ora_point* p2); /* SECP256K1.cpp:242-265 */
void ora_double_direct(ora_point* r, const ora_point* p);             /* SECP256K1.cpp:376-401 */
void ora_negation(ora_point* r, const ora_point* p);                   /* SECP256K1.cpp:103-111 */
int  ora_parse_pubkey_hex(const char* s, ora_point* r, int* compressed); /* SECP256K1.cpp:114-170 */
void ora_pubkey_hex(const ora_point* p, int compressed, char* out);   /* SECP256K1.cpp:172-189 */
const ora_u256* ora_order(void);
const ora_u256* ora_prime(void);

/* ---- XXH64 (xxhash/xxhash.h:2304-2527, vendored v0.8.0) ---- */
uint64_t ora_xxh64(const void* buf, size_t len, uint64_t seed);

/* ---- bloom (bloom/bloom.cpp) ---- */
typedef struct {
  uint64_t entries, bits, bytes;
  uint8_t hashes;
  long double error;
  uint8_t ready, major, minor;
  double bpe;
  uint8_t* bf;
} ora_bloom;                                                          /* bloom.h:26-45 */
int  ora_bloom_init2(ora_bloom* b, uint64_t entries, long double error); /* bloom.cpp:93-126 */
int  ora_bloom_check(const ora_bloom* b, const void* buf, int len);   /* bloom.cpp:128-156 */
int  ora_bloom_add(ora_bloom* b, const void* buf, int len);           /* bloom.cpp:61-85,159-162 */
void ora_bloom_free(ora_bloom* b);

/* ---- BSGS engine (keyhunt.cpp) ---- */
typedef struct { uint8_t value[6]; uint8_t pad[2]; uint64_t index; } ora_xvalue; /* keyhunt.cpp:70-73 */

typedef struct ora_bsgs ora_bsgs;

/* Geometry + all tables (keyhunt.cpp:1045-1364, 1615-1880, 4386-4592).  n_hex: "-n" value as
 * the reference parses it ("0x..." hex or decimal), NULL for the default 2^44.  Returns NULL and
 * writes a reference-style message into err on a rejected geometry. */
ora_bsgs* ora_bsgs_new(const char* n_str, int kfactor, int nthreads, char* err, size_t errlen);
void      ora_bsgs_free(ora_bsgs* c);
/* out: [0]=bsgs_m [1]=bsgs_m2 [2]=bsgs_m3 [3]=bsgs_aux [4]=cycles [5]=N(low64) [6]=L1 extent
 *      [7]=itemsbloom [8]=itemsbloom2 [9]=itemsbloom3 */
void ora_bsgs_params(const ora_bsgs* c, uint64_t out[10]);
const ora_bloom* ora_bsgs_bloom(const ora_bsgs* c, int level, int idx);  /* level 1,2,3 */
const ora_xvalue* ora_bsgs_bptable(const ora_bsgs* c);
void ora_bsgs_giant_table(const ora_bsgs* c, uint8_t out[513 * 64]);   /* GSn[0..511], _2GSn as x||y BE */
void ora_bsgs_amp_table(const ora_bsgs* c, int level, uint8_t out[32 * 64]);

/* startP of (base, target): keyhunt.cpp:3861-3869 */
void ora_bsgs_chunk_start(const ora_bsgs* c, const ora_u256* base, const ora_point* target, ora_point* startP);
/* Group loop of thread_process_bsgs (keyhunt.cpp:3871-4002) starting from centre startP (group j0),
 * for nj groups.  xdump (nullable) receives nj*1024 32-byte BE x values in probe order; cand
 * receives the giant-step indices a = j*1024+t whose L1 bloom probe hit (up to cap). *ncand is the
 * total number of hits (may exceed cap).  next (nullable) gets the centre after the last group. */
void ora_bsgs_scan(const ora_bsgs* c, const ora_point* startP, uint32_t j0, uint32_t nj,
                   uint8_t* xdump, uint64_t* cand, uint32_t cap, uint32_t* ncand, ora_point* next);
/* keyhunt.cpp:4271-4304 (+4306-4368, 3748-3773, 6680-6689). 1 = found, key in *key. */
int ora_bsgs_secondcheck(const ora_bsgs* c, const ora_u256* base, uint32_t a, const ora_point* target, ora_u256* key);
/* Sequential -t 1 search (keyhunt.cpp:3819-4006): chunks from start until end (or max_chunks),
 * targets in file order.  found[k] set to 1 and keys[k] filled for each found target.  Returns
 * the number of chunks processed. */
uint64_t ora_bsgs_search(const ora_bsgs* c, const ora_point* targets, int ntargets, const ora_u256* start,
                         const ora_u256* end, uint64_t max_chunks, int* found, ora_u256* keys);
/* CPU baseline: nthreads threads each scan consecutive groups of the chunk(s) starting at base for
 * `seconds` seconds; returns the number of giant steps (groups*1024) completed. */
uint64_t ora_bsgs_bench(const ora_bsgs* c, const ora_point* target, const ora_u256* base, int nthreads,
                        double seconds, double* elapsed);

/* ---- -m address / -m rmd160 (ora_addr.c) ---- */
void ora_sha256(const uint8_t* msg, size_t len, uint8_t out[32]);
void ora_ripemd160(const uint8_t* msg, size_t len, uint8_t out[20]);
void ora_hash160(const uint8_t* msg, size_t len, uint8_t out[20]);
void ora_pub_hash160(const ora_point* p, int compressed, uint8_t out[20]);   /* SECP256K1.cpp:671-705 */
void ora_x_hash160(uint8_t prefix, const ora_u256* x, uint8_t out[20]);     /* SECP256K1.cpp:707-789 */
int  ora_b58decode(const char* s, uint8_t* bin, size_t binsz, size_t* outsz); /* base58.c:39-112 */
void ora_rmd_to_address(const uint8_t rmd[20], char* out);                  /* keyhunt.cpp:2274-2284 */

typedef struct ora_addr ora_addr;
typedef struct ora_addr_gen ora_addr_gen;
/* forceReadFileAddress (keyhunt.cpp:6300-6358) over a target file's text; bloom per
 * initBloomFilter (keyhunt.cpp:6559-6576); table sorted (_sort). */
ora_addr* ora_addr_new(const char* text, int bloom_multiplier);
void      ora_addr_free(ora_addr* A);
uint64_t  ora_addr_count(const ora_addr* A);
const uint8_t* ora_addr_table(const ora_addr* A);
const ora_bloom* ora_addr_bloom(const ora_addr* A);
int       ora_addr_searchbinary(const ora_addr* A, const uint8_t data[20]);   /* keyhunt.cpp:2311-2335 */
/* init_generator (keyhunt.cpp:4386-4399): Gn[i] = (i+1)*stride*G, _2Gn = 1024*stride*G */
ora_addr_gen* ora_addr_gen_new(const ora_u256* stride);
void      ora_addr_gen_free(ora_addr_gen* g);
void      ora_addr_gen_table(const ora_addr_gen* g, uint8_t out[513 * 64]);
/* one thread_process group (keyhunt.cpp:2586-2711, checks 2789-2937); see ora_addr.c */
#define ORA_SEARCH_ENDO 4
void ora_mulmod_n(ora_u256* r, const ora_u256* a, const ora_u256* b);
void ora_endo_constants(int i, ora_u256* lambda, ora_u256* beta);   /* i = 0: lambda, beta; 1: lambda^2, beta^2 */
void ora_addr_group(const ora_addr* A, const ora_addr_gen* g, const ora_u256* key, int search, uint8_t* xy,
                    uint32_t* hits, uint32_t hcap, uint32_t* nhits, ora_u256* keys, uint32_t kcap,
                    uint32_t* nkeys);

/* ---- flat C-ABI helpers for ctypes (hex/byte strings only) ---- */
int ora_h_pubkey(const char* khex, char* out_hex, int compressed);       /* pubkey of key */
int ora_h_parse_target(const char* line, uint8_t xy_be[64], int* compressed);

#ifdef __cplusplus
}
#endif
#endif
