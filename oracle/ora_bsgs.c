/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see ora.h).
 * The BSGS engine of keyhunt.cpp restated in C: geometry (1045-1213), blooms (1215-1303), giant
 * tables (1309-1364), baby-step table build (thread_bPload 4404-4592 + orchestration 1615-1880),
 * the giant-step group loop (thread_process_bsgs 3778-4009) and candidate confirmation
 * (bsgs_secondcheck/thirdcheck 4271-4368, bsgs_searchbinary 3748-3773, calcualteindex 6680-6689).
 */
#include "ora.h"
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define GRP 1024            /* CPU_GRP_SIZE keyhunt.cpp:127 */
#define HALF (GRP / 2)
#define BLOOM_SEED_ERR 0.000001   /* keyhunt.cpp:1238, 1267, 1296 */
#define THREADBPWORKLOAD_DEFAULT 1048576ULL   /* keyhunt.cpp:63 */

struct ora_bsgs {
  uint64_t bsgs_m, bsgs_m2, bsgs_m3, bsgs_aux, cycles, l1ext;
  uint64_t items1, items2, items3;
  ora_u256 N, M, M2, M3, M_double, M2_double, M3_double, N_double, intaux;
  ora_bloom l1[256], l2[256], l3[256];
  ora_xvalue* bp;
  ora_point gsn[HALF], g2sn, amp2[32], amp3[32];
  ora_point gn[HALF], g2n;   /* baby-step stride table (init_generator keyhunt.cpp:4386-4399) */
};

/* ---------- small 256-bit helpers ---------- */
static void u256_shl1(ora_u256* a) {
  for (int i = 3; i > 0; --i) a->w[i] = (a->w[i] << 1) | (a->w[i - 1] >> 63);
  a->w[0] <<= 1;
}
static int u256_bit(const ora_u256* a, int i) { return (int)((a->w[i / 64] >> (i % 64)) & 1); }

/* q = a / b, r = a % b (b != 0); shift-subtract (one-off geometry arithmetic). */
static void u256_divmod(ora_u256* q, ora_u256* r, const ora_u256* a, const ora_u256* b) {
  ora_u256 qq = {{0, 0, 0, 0}}, rr = {{0, 0, 0, 0}};
  for (int i = 255; i >= 0; --i) {
    int top = (int)(rr.w[3] >> 63);
    u256_shl1(&rr);
    rr.w[0] |= (uint64_t)u256_bit(a, i);
    if (top || ora_u256_cmp(&rr, b) >= 0) {
      ora_u256_sub(&rr, &rr, b);
      qq.w[i / 64] |= 1ULL << (i % 64);
    }
  }
  if (q) *q = qq;
  if (r) *r = rr;
}

static void u256_mul(ora_u256* r, const ora_u256* a, const ora_u256* b) {   /* mod 2^256 */
  ora_u256 acc = {{0, 0, 0, 0}};
  for (int i = 0; i < 4; ++i) {
    unsigned __int128 c = 0;
    for (int j = 0; i + j < 4; ++j) {
      c += (unsigned __int128)a->w[j] * b->w[i] + acc.w[i + j];
      acc.w[i + j] = (uint64_t)c;
      c >>= 64;
    }
  }
  *r = acc;
}

/* Int::SetBase10 */
static int u256_from_dec(ora_u256* r, const char* s) {
  ora_u256 v = {{0, 0, 0, 0}}, d;
  if (!*s) return -1;
  for (; *s; ++s) {
    if (*s < '0' || *s > '9') return -1;
    ora_u256_mul64(&v, &v, 10);
    ora_u256_set64(&d, (uint64_t)(*s - '0'));
    ora_u256_add(&v, &v, &d);
  }
  *r = v;
  return 0;
}

/* ---------- geometry ---------- */
static uint64_t items_for(uint64_t m, uint64_t floor_limit, uint64_t minimum) {
  /* keyhunt.cpp:1185-1213 */
  if (m / 256 > floor_limit) {
    uint64_t it = m / 256;
    if (m % 256) it++;
    return it;
  }
  return minimum;
}

static int setup_geometry(ora_bsgs* c, const char* n_str, int kfactor, char* err, size_t errlen) {
  ora_u256 aux, r, k32, k1024, kk, two;
  /* keyhunt.cpp:1052-1067 */
  if (n_str) {
    int rc = (n_str[0] == '0' && n_str[1] == 'x') ? ora_u256_from_hex(&c->N, n_str + 2) : u256_from_dec(&c->N, n_str);
    if (rc) { snprintf(err, errlen, "[E] invalid -n value"); return -1; }
  } else {
    ora_u256_set64(&c->N, 0x100000000000ULL);
  }
  /* keyhunt.cpp:1069-1076: "exact root" is decided by Euler's criterion mod p and the root is
   * Int::ModSqrt mod p. */
  if (!ora_fe_has_sqrt(&c->N)) { snprintf(err, errlen, "[E] -n param doesn't have exact square root"); return -1; }
  ora_fe_sqrt(&c->M, &c->N);
  ora_u256_set64(&k1024, GRP);
  u256_divmod(NULL, &r, &c->M, &k1024);
  if (!ora_u256_is_zero(&r)) { snprintf(err, errlen, "[E] M value is not divisible by 1024"); return -1; }
  /* keyhunt.cpp:1129-1179 */
  ora_u256_set64(&kk, (uint64_t)(kfactor <= 0 ? 1 : kfactor));
  u256_mul(&c->M, &c->M, &kk);
  ora_u256_set64(&k32, 32);
  ora_u256_set64(&two, 2);
  u256_divmod(&c->M2, &r, &c->M, &k32);
  if (!ora_u256_is_zero(&r)) { ora_u256 one; ora_u256_set64(&one, 1); ora_u256_add(&c->M2, &c->M2, &one); }
  u256_mul(&c->M_double, &c->M, &two);
  u256_mul(&c->M2_double, &c->M2, &two);
  u256_divmod(&c->M3, &r, &c->M2, &k32);
  if (!ora_u256_is_zero(&r)) { ora_u256 one; ora_u256_set64(&one, 1); ora_u256_add(&c->M3, &c->M3, &one); }
  u256_mul(&c->M3_double, &c->M3, &two);
  c->bsgs_m2 = c->M2.w[0];
  c->bsgs_m3 = c->M3.w[0];
  u256_divmod(&aux, &r, &c->N, &c->M);
  if (!ora_u256_is_zero(&r)) u256_mul(&c->N, &c->M, &aux);
  c->bsgs_m = c->M.w[0];
  c->bsgs_aux = aux.w[0];
  u256_mul(&c->N_double, &c->N, &two);
  if (c->M.w[1] | c->M.w[2] | c->M.w[3] || c->bsgs_m > (1ULL << 36)) {
    snprintf(err, errlen, "[E] baby-step table too large for the oracle");
    return -1;
  }
  c->items1 = items_for(c->bsgs_m, 10000, 1000);
  c->items2 = items_for(c->bsgs_m2, 1000, 1000);
  c->items3 = items_for(c->bsgs_m3, 1000, 1000);
  /* cycles, intaux: keyhunt.cpp:3810-3817 */
  c->cycles = c->bsgs_aux / GRP + ((c->bsgs_aux % GRP) ? 1 : 0);
  ora_u256 half; ora_u256_set64(&half, HALF);
  u256_mul(&c->intaux, &c->M_double, &half);
  ora_u256_add(&c->intaux, &c->intaux, &c->M);
  /* L1 extent, keyhunt.cpp:1739-1793 + thread_bPload's "i_counter < to" (quirk vi): when m is not a
   * multiple of the 2^20 job size the last job's `to` overshoots m by one job. */
  uint64_t W = THREADBPWORKLOAD_DEFAULT;
  if (W >= c->bsgs_m) W = c->bsgs_m;
  uint64_t R = c->bsgs_m % W;
  c->l1ext = R ? (c->bsgs_m / W) * W + W + R : c->bsgs_m;
  return 0;
}

/* ---------- giant tables, keyhunt.cpp:1309-1364 ---------- */
static void setup_giant_tables(ora_bsgs* c) {
  ora_point mp2d, mp2, mp3, mp3d, bsP, g, tmp;
  ora_compute_pubkey(&mp2d, &c->M_double);   /* BSGS_MP_double */
  ora_negation(&bsP, &mp2d);
  g = bsP;
  c->gsn[0] = g;
  ora_double_direct(&g, &g);
  c->gsn[1] = g;
  for (int i = 2; i < HALF; ++i) { ora_add_direct(&g, &g, &bsP); c->gsn[i] = g; }
  ora_double_direct(&c->g2sn, &c->gsn[HALF - 1]);
  ora_compute_pubkey(&mp2, &c->M2);
  ora_compute_pubkey(&mp2d, &c->M2_double);
  ora_compute_pubkey(&mp3, &c->M3);
  ora_compute_pubkey(&mp3d, &c->M3_double);
  /* Negation + Reduce: z == 1 so Reduce leaves canonical coordinates unchanged */
  ora_negation(&c->amp2[0], &mp2);
  ora_negation(&tmp, &mp2d);
  for (int i = 1; i < 32; ++i) ora_add_direct(&c->amp2[i], &c->amp2[i - 1], &tmp);
  ora_negation(&c->amp3[0], &mp3);
  ora_negation(&tmp, &mp3d);
  for (int i = 1; i < 32; ++i) ora_add_direct(&c->amp3[i], &c->amp3[i - 1], &tmp);
  /* init_generator (keyhunt.cpp:4386-4399), stride 1 */
  ora_u256 one; ora_u256_set64(&one, 1);
  ora_point G1;
  ora_compute_pubkey(&G1, &one);
  g = G1;
  c->gn[0] = g;
  ora_double_direct(&g, &g);
  c->gn[1] = g;
  for (int i = 2; i < HALF; ++i) { ora_add_direct(&g, &g, &G1); c->gn[i] = g; }
  ora_double_direct(&c->g2n, &c->gn[HALF - 1]);
}

/* ---------- the shared 1024-point group step ---------- */
/* Computes the 1024 x-coordinates of the group centred on *centre (pts order of keyhunt.cpp
 * 3885-3943 / 4450-4513) and advances *centre by tab2 (3986-3999 / 4565-4578). */
static void group_step(ora_point* centre, const ora_point* tab, const ora_point* tab2, ora_u256* dx,
                       ora_u256* subp, ora_u256* xs) {
  ora_u256 dy, dyn, s, p, inverse, nv;
  int i;
  for (i = 0; i < HALF - 1; ++i) ora_fe_sub(&dx[i], &tab[i].x, &centre->x);
  ora_fe_sub(&dx[i], &tab[i].x, &centre->x);
  ora_fe_sub(&dx[i + 1], &tab2->x, &centre->x);
  /* IntGroup::ModInv (IntGroup.cpp:36-58) over HALF+1 elements */
  subp[0] = dx[0];
  for (int k = 1; k < HALF + 1; ++k) ora_fe_mulK1(&subp[k], &subp[k - 1], &dx[k]);
  inverse = subp[HALF];
  ora_fe_inv(&inverse, &inverse);
  for (int k = HALF; k > 0; --k) {
    ora_fe_mulK1(&nv, &subp[k - 1], &inverse);
    ora_fe_mulK1(&inverse, &inverse, &dx[k]);
    dx[k] = nv;
  }
  dx[0] = inverse;
  xs[HALF] = centre->x;
  for (i = 0; i < HALF - 1; ++i) {
    ora_u256 x;
    ora_fe_sub(&dy, &tab[i].y, &centre->y);
    ora_fe_mulK1(&s, &dy, &dx[i]);
    ora_fe_sqrK1(&p, &s);
    ora_fe_neg(&x, &centre->x);
    ora_fe_add(&x, &x, &p);
    ora_fe_sub(&x, &x, &tab[i].x);
    xs[HALF + (i + 1)] = x;
    ora_fe_neg(&dyn, &tab[i].y);
    ora_fe_sub(&dyn, &dyn, &centre->y);
    ora_fe_mulK1(&s, &dyn, &dx[i]);
    ora_fe_sqrK1(&p, &s);
    ora_fe_neg(&x, &centre->x);
    ora_fe_add(&x, &x, &p);
    ora_fe_sub(&x, &x, &tab[i].x);
    xs[HALF - (i + 1)] = x;
  }
  {
    ora_u256 x;
    ora_fe_neg(&dyn, &tab[i].y);
    ora_fe_sub(&dyn, &dyn, &centre->y);
    ora_fe_mulK1(&s, &dyn, &dx[i]);
    ora_fe_sqrK1(&p, &s);
    ora_fe_neg(&x, &centre->x);
    ora_fe_add(&x, &x, &p);
    ora_fe_sub(&x, &x, &tab[i].x);
    xs[0] = x;
  }
  /* next centre */
  {
    ora_point n;
    ora_fe_sub(&dy, &tab2->y, &centre->y);
    ora_fe_mulK1(&s, &dy, &dx[i + 1]);
    ora_fe_sqrK1(&p, &s);
    ora_fe_neg(&n.x, &centre->x);
    ora_fe_add(&n.x, &n.x, &p);
    ora_fe_sub(&n.x, &n.x, &tab2->x);
    ora_fe_sub(&n.y, &tab2->x, &n.x);
    ora_fe_mulK1(&n.y, &n.y, &s);
    ora_fe_sub(&n.y, &n.y, &tab2->y);
    ora_u256_set64(&n.z, 1);
    *centre = n;
  }
}

/* ---------- baby-step table build ---------- */
typedef struct {
  ora_bsgs* c;
  uint64_t from, to;
} bp_job;

static void bloom_add_atomic(ora_bloom* b, const uint8_t* xb) {
  /* bloom_add under the per-sub-bloom mutex (keyhunt.cpp:4529-4560); OR-ing bits is
   * order-independent, so an atomic OR gives the identical bit array. */
  uint64_t a = ora_xxh64(xb, 32, 0x59f2815b16f81798ULL);
  uint64_t bb = ora_xxh64(xb, 32, a);
  for (uint8_t i = 0; i < b->hashes; ++i) {
    uint64_t x = (a + bb * i) % b->bits;
    __atomic_fetch_or(&b->bf[x >> 3], (uint8_t)(1u << (x % 8)), __ATOMIC_RELAXED);
  }
}

/* thread_bPload (keyhunt.cpp:4404-4592) for one job [from, to) */
static void bp_run_job(ora_bsgs* c, uint64_t from, uint64_t to) {
  ora_u256* dx = (ora_u256*)malloc(sizeof(ora_u256) * (HALF + 1));
  ora_u256* subp = (ora_u256*)malloc(sizeof(ora_u256) * (HALF + 1));
  ora_u256* xs = (ora_u256*)malloc(sizeof(ora_u256) * GRP);
  uint64_t nb = (to - from) / GRP + (((to - from) % GRP) ? 1 : 0);
  ora_u256 km;
  ora_u256_set64(&km, from + 1 + HALF);
  ora_point centre;
  ora_compute_pubkey(&centre, &km);
  uint64_t ic = from;
  uint8_t xb[32];
  for (uint64_t s = 0; s < nb; ++s) {
    group_step(&centre, c->gn, &c->g2n, dx, subp, xs);
    for (int j = 0; j < GRP; ++j, ++ic) {
      ora_u256_to_be(&xs[j], xb);
      int idx = xb[0];
      if (ic < c->bsgs_m3) {
        memcpy(c->bp[ic].value, xb + 16, 6);
        c->bp[ic].index = ic;
        bloom_add_atomic(&c->l3[idx], xb);
      }
      if (ic < c->bsgs_m2) bloom_add_atomic(&c->l2[idx], xb);
      if (ic < to) bloom_add_atomic(&c->l1[idx], xb);
    }
  }
  free(dx); free(subp); free(xs);
}

typedef struct {
  ora_bsgs* c;
  bp_job* jobs;
  int njobs;
  int* next;
  pthread_mutex_t* mu;
} bp_pool;

static void* bp_worker(void* arg) {
  bp_pool* pl = (bp_pool*)arg;
  for (;;) {
    pthread_mutex_lock(pl->mu);
    int j = (*pl->next)++;
    pthread_mutex_unlock(pl->mu);
    if (j >= pl->njobs) break;
    bp_run_job(pl->c, pl->jobs[j].from, pl->jobs[j].to);
  }
  return NULL;
}

static int xv_cmp(const void* a, const void* b) {
  const ora_xvalue* x = (const ora_xvalue*)a;
  const ora_xvalue* y = (const ora_xvalue*)b;
  int r = memcmp(x->value, y->value, 6);
  if (r) return r;
  return x->index < y->index ? -1 : (x->index > y->index);
}

static int build_tables(ora_bsgs* c, int nthreads) {
  for (int i = 0; i < 256; ++i) {
    if (ora_bloom_init2(&c->l1[i], c->items1, BLOOM_SEED_ERR)) return -1;
    if (ora_bloom_init2(&c->l2[i], c->items2, BLOOM_SEED_ERR)) return -1;
    if (ora_bloom_init2(&c->l3[i], c->items3, BLOOM_SEED_ERR)) return -1;
  }
  c->bp = (ora_xvalue*)calloc(c->bsgs_m3, sizeof(ora_xvalue));
  if (!c->bp) return -1;
  /* job list, keyhunt.cpp:1733-1807 */
  uint64_t W = THREADBPWORKLOAD_DEFAULT;
  if (W >= c->bsgs_m) W = c->bsgs_m;
  uint64_t cyc = c->bsgs_m / W, R = c->bsgs_m % W;
  if (R) cyc++;
  bp_job* jobs = (bp_job*)calloc(cyc, sizeof(bp_job));
  uint64_t base = 0;
  for (uint64_t j = 0; j < cyc; ++j) {
    jobs[j].c = c;
    jobs[j].from = base;
    jobs[j].to = (j < cyc - 1) ? base + W : base + W + R;
    base += W;
  }
  int next = 0;
  pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
  bp_pool pl = {c, jobs, (int)cyc, &next, &mu};
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, bp_worker, &pl);
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
  /* bsgs_sort (keyhunt.cpp:3657-3746): introsort by 6-byte memcmp.  For distinct keys every
   * correct sort yields the same array; equal 6-byte keys (quirk v) are ordered by index here. */
  qsort(c->bp, c->bsgs_m3, sizeof(ora_xvalue), xv_cmp);
  return 0;
}

ora_bsgs* ora_bsgs_new(const char* n_str, int kfactor, int nthreads, char* err, size_t errlen) {
  ora_secp_init();
  ora_bsgs* c = (ora_bsgs*)calloc(1, sizeof(ora_bsgs));
  if (!c) return NULL;
  if (setup_geometry(c, n_str, kfactor, err, errlen)) { free(c); return NULL; }
  setup_giant_tables(c);
  if (build_tables(c, nthreads)) {
    snprintf(err, errlen, "[E] table allocation failed");
    ora_bsgs_free(c);
    return NULL;
  }
  return c;
}

void ora_bsgs_free(ora_bsgs* c) {
  if (!c) return;
  for (int i = 0; i < 256; ++i) { ora_bloom_free(&c->l1[i]); ora_bloom_free(&c->l2[i]); ora_bloom_free(&c->l3[i]); }
  free(c->bp);
  free(c);
}

void ora_bsgs_params(const ora_bsgs* c, uint64_t out[10]) {
  out[0] = c->bsgs_m; out[1] = c->bsgs_m2; out[2] = c->bsgs_m3; out[3] = c->bsgs_aux;
  out[4] = c->cycles; out[5] = c->N.w[0]; out[6] = c->l1ext;
  out[7] = c->items1; out[8] = c->items2; out[9] = c->items3;
}

const ora_bloom* ora_bsgs_bloom(const ora_bsgs* c, int level, int idx) {
  if (idx < 0 || idx > 255) return NULL;
  return level == 1 ? &c->l1[idx] : level == 2 ? &c->l2[idx] : level == 3 ? &c->l3[idx] : NULL;
}

const ora_xvalue* ora_bsgs_bptable(const ora_bsgs* c) { return c->bp; }

static void pt_be(const ora_point* p, uint8_t* out) { ora_u256_to_be(&p->x, out); ora_u256_to_be(&p->y, out + 32); }

void ora_bsgs_giant_table(const ora_bsgs* c, uint8_t out[513 * 64]) {
  for (int i = 0; i < HALF; ++i) pt_be(&c->gsn[i], out + 64 * i);
  pt_be(&c->g2sn, out + 64 * HALF);
}

void ora_bsgs_amp_table(const ora_bsgs* c, int level, uint8_t out[32 * 64]) {
  const ora_point* t = level == 2 ? c->amp2 : c->amp3;
  for (int i = 0; i < 32; ++i) pt_be(&t[i], out + 64 * i);
}

/* keyhunt.cpp:3861-3869: point_aux = G*(order - base - intaux); startP = target + point_aux */
void ora_bsgs_chunk_start(const ora_bsgs* c, const ora_u256* base, const ora_point* target, ora_point* startP) {
  ora_u256 km;
  ora_point aux;
  ora_u256_sub(&km, ora_order(), base);
  ora_u256_sub(&km, &km, &c->intaux);
  ora_compute_pubkey(&aux, &km);
  ora_add_direct(startP, target, &aux);
}

void ora_bsgs_scan(const ora_bsgs* c, const ora_point* startP, uint32_t j0, uint32_t nj, uint8_t* xdump,
                   uint64_t* cand, uint32_t cap, uint32_t* ncand, ora_point* next) {
  ora_u256* dx = (ora_u256*)malloc(sizeof(ora_u256) * (HALF + 1));
  ora_u256* subp = (ora_u256*)malloc(sizeof(ora_u256) * (HALF + 1));
  ora_u256* xs = (ora_u256*)malloc(sizeof(ora_u256) * GRP);
  ora_point centre = *startP;
  uint32_t n = 0;
  uint8_t xb[32];
  for (uint32_t jj = 0; jj < nj; ++jj) {
    uint64_t j = (uint64_t)j0 + jj;
    group_step(&centre, c->gsn, &c->g2sn, dx, subp, xs);
    for (int t = 0; t < GRP; ++t) {
      ora_u256_to_be(&xs[t], xb);
      if (xdump) memcpy(xdump + ((uint64_t)jj * GRP + t) * 32, xb, 32);
      if (ora_bloom_check(&c->l1[xb[0]], xb, 32)) {   /* keyhunt.cpp:3945-3947 */
        if (n < cap && cand) cand[n] = j * GRP + (uint64_t)t;
        n++;
      }
    }
  }
  if (ncand) *ncand = n;
  if (next) *next = centre;
  free(dx); free(subp); free(xs);
}

/* bsgs_searchbinary (keyhunt.cpp:3748-3773) */
static int searchbinary(const ora_xvalue* buf, const uint8_t* data, int64_t n, uint64_t* rv) {
  int64_t min = 0, max = n, half = n, current = 0;
  int r = 0;
  while (!r && half >= 1) {
    half = (max - min) / 2;
    int rc = memcmp(data + 16, buf[current + half].value, 6);
    if (rc == 0) { *rv = buf[current + half].index; r = 1; }
    else {
      if (rc < 0) max = max - half;
      else min = min + half;
      current = min;
    }
  }
  return r;
}

/* calcualteindex (keyhunt.cpp:6680-6689): (2i+1)*M3 */
static void calc_index(const ora_bsgs* c, int i, ora_u256* key) {
  if (i == 0) { *key = c->M3; return; }
  ora_u256 ii;
  ora_u256_set64(&ii, (uint64_t)i);
  u256_mul(key, &ii, &c->M3_double);
  ora_u256_add(key, key, &c->M3);
}

/* bsgs_thirdcheck (keyhunt.cpp:4306-4368) */
static int thirdcheck(const ora_bsgs* c, const ora_u256* start, uint32_t a, const ora_point* target, ora_u256* key) {
  ora_u256 base, ai, ck;
  ora_point bp, aux, S, Q, QA;
  uint8_t xb[32];
  ora_u256_set64(&ai, a);
  u256_mul(&base, &ai, &c->M2_double);
  ora_u256_add(&base, &base, start);
  ora_compute_pubkey(&bp, &base);
  ora_negation(&aux, &bp);
  ora_add_direct(&S, target, &aux);
  Q = S;
  for (int i = 0; i < 32; ++i) {
    ora_add_direct(&QA, &Q, &c->amp3[i]);
    S = QA;
    ora_u256_to_be(&S.x, xb);
    if (ora_bloom_check(&c->l3[xb[0]], xb, 32)) {
      uint64_t j = 0;
      if (searchbinary(c->bp, xb, (int64_t)c->bsgs_m3, &j)) {
        ora_u256 jj;
        ora_point pa;
        calc_index(c, i, &ck);
        ora_u256_set64(&jj, j + 1);
        ora_u256_add(key, &ck, &jj);
        ora_u256_add(key, key, &base);
        ora_compute_pubkey(&pa, key);
        if (ora_u256_cmp(&pa.x, &target->x) == 0) return 1;
        calc_index(c, i, &ck);
        ora_u256_sub(key, &ck, &jj);
        ora_u256_add(key, key, &base);
        ora_compute_pubkey(&pa, key);
        if (ora_u256_cmp(&pa.x, &target->x) == 0) return 1;
      }
    } else {
      /* keyhunt.cpp:4352-4364: AddDirect(P,-P) special case */
      if (ora_u256_cmp(&Q.x, &c->amp3[i].x) == 0) {
        calc_index(c, i, &ck);
        ora_u256_add(key, &ck, &base);
        return 1;
      }
    }
  }
  return 0;
}

/* bsgs_secondcheck (keyhunt.cpp:4271-4304) */
int ora_bsgs_secondcheck(const ora_bsgs* c, const ora_u256* start, uint32_t a, const ora_point* target, ora_u256* key) {
  ora_u256 base, ai;
  ora_point bp, aux, S, Q, QA;
  uint8_t xb[32];
  ora_u256_set64(&ai, a);
  u256_mul(&base, &c->M_double, &ai);
  ora_u256_add(&base, &base, start);
  ora_compute_pubkey(&bp, &base);
  ora_negation(&aux, &bp);
  ora_add_direct(&S, target, &aux);
  Q = S;
  for (int i = 0; i < 32; ++i) {
    ora_add_direct(&QA, &Q, &c->amp2[i]);
    S = QA;
    ora_u256_to_be(&S.x, xb);
    if (ora_bloom_check(&c->l2[xb[0]], xb, 32)) {
      if (thirdcheck(c, &base, (uint32_t)i, target, key)) return 1;
    }
  }
  return 0;
}

/* thread_process_bsgs (keyhunt.cpp:3819-4006), single thread. */
uint64_t ora_bsgs_search(const ora_bsgs* c, const ora_point* targets, int ntargets, const ora_u256* start,
                         const ora_u256* end, uint64_t max_chunks, int* found, ora_u256* keys) {
  ora_u256* dx = (ora_u256*)malloc(sizeof(ora_u256) * (HALF + 1));
  ora_u256* subp = (ora_u256*)malloc(sizeof(ora_u256) * (HALF + 1));
  ora_u256* xs = (ora_u256*)malloc(sizeof(ora_u256) * GRP);
  ora_u256 cur = *start;
  uint64_t chunks = 0;
  uint8_t xb[32];
  for (int k = 0; k < ntargets; ++k) found[k] = 0;
  for (;;) {
    if (max_chunks && chunks >= max_chunks) break;
    ora_u256 base = cur;
    ora_u256_add(&cur, &cur, &c->N_double);
    if (ora_u256_cmp(&base, end) >= 0) break;
    chunks++;
    ora_u256 km;
    ora_point aux;
    ora_u256_sub(&km, ora_order(), &base);
    ora_u256_sub(&km, &km, &c->intaux);
    ora_compute_pubkey(&aux, &km);
    for (int k = 0; k < ntargets; ++k) {
      if (found[k]) continue;
      ora_point centre;
      ora_add_direct(&centre, &targets[k], &aux);
      for (uint64_t j = 0; j < c->cycles && !found[k]; ++j) {
        group_step(&centre, c->gsn, &c->g2sn, dx, subp, xs);
        for (int t = 0; t < GRP && !found[k]; ++t) {
          ora_u256_to_be(&xs[t], xb);
          if (ora_bloom_check(&c->l1[xb[0]], xb, 32)) {
            ora_u256 key;
            if (ora_bsgs_secondcheck(c, &base, (uint32_t)(j * GRP + (uint64_t)t), &targets[k], &key)) {
              found[k] = 1;
              keys[k] = key;
            }
          }
        }
      }
    }
    int all = 1;
    for (int k = 0; k < ntargets; ++k) all &= found[k];
    if (all) break;   /* "All points were found" (keyhunt.cpp:3975-3981) */
  }
  free(dx); free(subp); free(xs);
  return chunks;
}

/* ---------- CPU baseline timing ---------- */
typedef struct {
  const ora_bsgs* c;
  ora_point target;
  ora_u256 base;
  double seconds;
  volatile int* stop;
  uint64_t steps;
} bench_arg;

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void* bench_worker(void* p) {
  bench_arg* a = (bench_arg*)p;
  const ora_bsgs* c = a->c;
  ora_u256* dx = (ora_u256*)malloc(sizeof(ora_u256) * (HALF + 1));
  ora_u256* subp = (ora_u256*)malloc(sizeof(ora_u256) * (HALF + 1));
  ora_u256* xs = (ora_u256*)malloc(sizeof(ora_u256) * GRP);
  uint8_t xb[32];
  ora_u256 base = a->base;
  uint64_t steps = 0;
  while (!*a->stop) {
    ora_point centre;
    ora_bsgs_chunk_start(c, &base, &a->target, &centre);
    for (uint64_t j = 0; j < c->cycles && !*a->stop; ++j) {
      group_step(&centre, c->gsn, &c->g2sn, dx, subp, xs);
      for (int t = 0; t < GRP; ++t) {
        ora_u256_to_be(&xs[t], xb);
        if (ora_bloom_check(&c->l1[xb[0]], xb, 32)) {
          ora_u256 key;
          ora_bsgs_secondcheck(c, &base, (uint32_t)(j * GRP + (uint64_t)t), &a->target, &key);
        }
      }
      steps += GRP;
    }
    ora_u256_add(&base, &base, &c->N_double);
  }
  a->steps = steps;
  free(dx); free(subp); free(xs);
  return NULL;
}

uint64_t ora_bsgs_bench(const ora_bsgs* c, const ora_point* target, const ora_u256* base, int nthreads,
                        double seconds, double* elapsed) {
  if (nthreads < 1) nthreads = 1;
  volatile int stop = 0;
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  bench_arg* args = (bench_arg*)calloc((size_t)nthreads, sizeof(bench_arg));
  double t0 = now_s();
  for (int t = 0; t < nthreads; ++t) {
    args[t].c = c;
    args[t].target = *target;
    /* thread t starts t chunks (of 2N keys) after base, like threads claiming BSGS_CURRENT */
    ora_u256 off, tt;
    ora_u256_set64(&tt, (uint64_t)t);
    u256_mul(&off, &c->N_double, &tt);
    ora_u256_add(&args[t].base, base, &off);
    args[t].seconds = seconds;
    args[t].stop = &stop;
    pthread_create(&th[t], NULL, bench_worker, &args[t]);
  }
  while (now_s() - t0 < seconds) {
    struct timespec ts = {0, 20 * 1000 * 1000};
    nanosleep(&ts, NULL);
  }
  stop = 1;
  uint64_t total = 0;
  for (int t = 0; t < nthreads; ++t) { pthread_join(th[t], NULL); total += args[t].steps; }
  if (elapsed) *elapsed = now_s() - t0;
  free(th);
  free(args);
  return total;
}
