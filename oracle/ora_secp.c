/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see ora.h).
 * secp256k1 group operations restated from secp256k1/SECP256K1.cpp and secp256k1/Point.cpp.
 */
#include "ora.h"
#include <stdio.h>
#include <string.h>
#include <stdlib.h>

static const ora_u256 ORDER = {{0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, 0xFFFFFFFFFFFFFFFFULL}};
static ora_point G;
static ora_point GTABLE[32 * 256];   /* SECP256K1.cpp:44-54: GTable[i*256+j] = (j+1)*256^i*G */
static int inited = 0;

const ora_u256* ora_order(void) { return &ORDER; }

/* Point::Reduce (Point.cpp:65-73): divide x, y by z (canonical). */
static void point_reduce(ora_point* p) {
  ora_u256 iz;
  ora_fe_inv(&iz, &p->z);
  ora_fe_mul_exact(&p->x, &p->x, &iz);
  ora_fe_mul_exact(&p->y, &p->y, &iz);
  ora_u256_set64(&p->z, 1);
}

/* Secp256K1::Add2 (SECP256K1.cpp:268-306): projective + affine (p2.z == 1). */
static void add2(ora_point* r, const ora_point* p1, const ora_point* p2) {
  ora_u256 u, v, u1, v1, vs2, vs3, us2, a, us2w, vs2v2, vs3u2, _2vs2v2;
  ora_point o;
  ora_fe_mulK1(&u1, &p2->y, &p1->z);
  ora_fe_mulK1(&v1, &p2->x, &p1->z);
  ora_fe_sub(&u, &u1, &p1->y);
  ora_fe_sub(&v, &v1, &p1->x);
  ora_fe_sqrK1(&us2, &u);
  ora_fe_sqrK1(&vs2, &v);
  ora_fe_mulK1(&vs3, &vs2, &v);
  ora_fe_mulK1(&us2w, &us2, &p1->z);
  ora_fe_mulK1(&vs2v2, &vs2, &p1->x);
  ora_fe_add(&_2vs2v2, &vs2v2, &vs2v2);
  ora_fe_sub(&a, &us2w, &vs3);
  ora_fe_sub(&a, &a, &_2vs2v2);
  ora_fe_mulK1(&o.x, &v, &a);
  ora_fe_mulK1(&vs3u2, &vs3, &p1->y);
  ora_fe_sub(&o.y, &vs2v2, &a);
  ora_fe_mulK1(&o.y, &o.y, &u);
  ora_fe_sub(&o.y, &o.y, &vs3u2);
  ora_fe_mulK1(&o.z, &vs3, &p1->z);
  *r = o;
}

/* Secp256K1::AddDirect (SECP256K1.cpp:242-265).  dx == 0 gives ModInv == 0 and therefore s == 0,
 * exactly as the reference (the special case bsgs_thirdcheck works around, keyhunt.cpp:4352-4364). */
void ora_add_direct(ora_point* r, const ora_point* p1, const ora_point* p2) {
  ora_u256 s, p, dy, dx;
  ora_point o;
  ora_u256_set64(&o.z, 1);
  ora_fe_sub(&dy, &p2->y, &p1->y);
  ora_fe_sub(&dx, &p2->x, &p1->x);
  ora_fe_inv(&dx, &dx);
  ora_fe_mulK1(&s, &dy, &dx);
  ora_fe_sqrK1(&p, &s);
  ora_fe_sub(&o.x, &p, &p1->x);
  ora_fe_sub(&o.x, &o.x, &p2->x);
  ora_fe_sub(&o.y, &p2->x, &o.x);
  ora_fe_mulK1(&o.y, &o.y, &s);
  ora_fe_sub(&o.y, &o.y, &p2->y);
  *r = o;
}

/* Secp256K1::DoubleDirect (SECP256K1.cpp:376-401). */
void ora_double_direct(ora_point* r, const ora_point* pt) {
  ora_u256 s, p, a;
  ora_point o;
  ora_u256_set64(&o.z, 1);
  ora_fe_mulK1(&s, &pt->x, &pt->x);
  ora_fe_add(&p, &s, &s);
  ora_fe_add(&p, &p, &s);
  ora_fe_add(&a, &pt->y, &pt->y);
  ora_fe_inv(&a, &a);
  ora_fe_mulK1(&s, &p, &a);
  ora_fe_mulK1(&p, &s, &s);
  ora_fe_add(&a, &pt->x, &pt->x);
  ora_fe_neg(&a, &a);
  ora_fe_add(&o.x, &a, &p);
  ora_fe_sub(&a, &o.x, &pt->x);
  ora_fe_mulK1(&p, &a, &s);
  ora_fe_add(&o.y, &p, &pt->y);
  ora_fe_neg(&o.y, &o.y);
  *r = o;
}

/* Secp256K1::Negation (SECP256K1.cpp:103-111): y = P - y (plain subtraction). */
void ora_negation(ora_point* r, const ora_point* p) {
  ora_point o;
  o.x = p->x;
  ora_u256_sub(&o.y, ora_prime(), &p->y);
  ora_u256_set64(&o.z, 1);
  *r = o;
}

void ora_secp_init(void) {
  if (inited) return;
  /* SECP256K1.cpp:37-39 */
  ora_u256_from_hex(&G.x, "79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798");
  ora_u256_from_hex(&G.y, "483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8");
  ora_u256_set64(&G.z, 1);
  /* SECP256K1.cpp:44-54 */
  ora_point n = G;
  for (int i = 0; i < 32; ++i) {
    GTABLE[i * 256] = n;
    ora_double_direct(&n, &n);
    for (int j = 1; j < 255; ++j) {
      GTABLE[i * 256 + j] = n;
      ora_add_direct(&n, &n, &GTABLE[i * 256]);
    }
    GTABLE[i * 256 + 255] = n;
  }
  inited = 1;
}

static uint8_t le_byte(const ora_u256* k, int i) { return (uint8_t)(k->w[i / 8] >> (8 * (i % 8))); }

/* Secp256K1::ComputePublicKey (SECP256K1.cpp:61-82): byte windows from the least significant byte,
 * projective Add2 accumulation, then Reduce.  k must be in [1, n). */
void ora_compute_pubkey(ora_point* r, const ora_u256* k) {
  ora_secp_init();
  int i;
  uint8_t b = 0;
  for (i = 0; i < 32; ++i) {
    b = le_byte(k, i);
    if (b) break;
  }
  if (i == 32) { memset(r, 0, sizeof(*r)); return; }  /* reference indexes out of bounds here */
  ora_point q = GTABLE[256 * i + (b - 1)];
  ++i;
  for (; i < 32; ++i) {
    b = le_byte(k, i);
    if (b) add2(&q, &q, &GTABLE[256 * i + (b - 1)]);
  }
  point_reduce(&q);
  *r = q;
}

/* Secp256K1::EC (SECP256K1.cpp:478-487) */
static int on_curve(const ora_point* p) {
  ora_u256 s, t, seven;
  ora_u256_set64(&seven, 7);
  ora_fe_sqrK1(&s, &p->x);
  ora_fe_mulK1(&t, &s, &p->x);
  ora_fe_add(&t, &t, &seven);
  ora_fe_mulK1(&s, &p->y, &p->y);
  ora_fe_sub(&s, &s, &t);
  return ora_u256_is_zero(&s);
}

/* Secp256K1::GetY (SECP256K1.cpp:462-476) */
static void get_y(ora_u256* y, const ora_u256* x, int want_even) {
  ora_u256 s, p, seven;
  ora_u256_set64(&seven, 7);
  ora_fe_sqrK1(&s, x);
  ora_fe_mulK1(&p, &s, x);
  ora_fe_add(&p, &p, &seven);
  ora_fe_sqrt(&p, &p);
  int even = (p.w[0] & 1) == 0;
  if ((!even && want_even) || (even && !want_even)) ora_fe_neg(&p, &p);
  *y = p;
}

static int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

/* Secp256K1::GetByte (SECP256K1.cpp:90-101) for well-formed hex pairs. */
static int get_byte(const char* s, int idx) {
  int h = hexval(s[2 * idx]), l = hexval(s[2 * idx + 1]);
  if (h < 0 || l < 0) return -1;
  return h * 16 + l;
}

/* Secp256K1::ParsePublicKeyHex (SECP256K1.cpp:114-170).  Returns 1 on success. */
int ora_parse_pubkey_hex(const char* s, ora_point* r, int* compressed) {
  ora_secp_init();
  memset(r, 0, sizeof(*r));
  int len = (int)strlen(s);
  if (len < 2) return 0;
  int type = get_byte(s, 0);
  uint8_t xb[32], yb[32];
  switch (type) {
    case 0x02:
    case 0x03:
      if (len != 66) return 0;
      for (int i = 0; i < 32; ++i) { int v = get_byte(s, i + 1); if (v < 0) return 0; xb[i] = (uint8_t)v; }
      ora_u256_from_be(&r->x, xb);
      get_y(&r->y, &r->x, type == 0x02);
      *compressed = 1;
      break;
    case 0x04:
      if (len != 130) return 0;
      for (int i = 0; i < 32; ++i) { int v = get_byte(s, i + 1); if (v < 0) return 0; xb[i] = (uint8_t)v; }
      for (int i = 0; i < 32; ++i) { int v = get_byte(s, i + 33); if (v < 0) return 0; yb[i] = (uint8_t)v; }
      ora_u256_from_be(&r->x, xb);
      ora_u256_from_be(&r->y, yb);
      *compressed = 0;
      break;
    default:
      return 0;
  }
  ora_u256_set64(&r->z, 1);
  return on_curve(r);
}

/* Secp256K1::GetPublicKeyHex (SECP256K1.cpp:172-189): lowercase (util.c tohex "%.2x"). */
void ora_pubkey_hex(const ora_point* p, int compressed, char* out) {
  static const char* dg = "0123456789abcdef";
  uint8_t b[65];
  int n;
  if (!compressed) {
    b[0] = 4;
    ora_u256_to_be(&p->x, b + 1);
    ora_u256_to_be(&p->y, b + 33);
    n = 65;
  } else {
    b[0] = (p->y.w[0] & 1) ? 3 : 2;
    ora_u256_to_be(&p->x, b + 1);
    n = 33;
  }
  for (int i = 0; i < n; ++i) { out[2 * i] = dg[b[i] >> 4]; out[2 * i + 1] = dg[b[i] & 15]; }
  out[2 * n] = 0;
}

int ora_h_pubkey(const char* khex, char* out_hex, int compressed) {
  ora_u256 k;
  if (ora_u256_from_hex(&k, khex)) return -1;
  ora_point p;
  ora_compute_pubkey(&p, &k);
  ora_pubkey_hex(&p, compressed, out_hex);
  return 0;
}

int ora_h_parse_target(const char* line, uint8_t xy_be[64], int* compressed) {
  ora_point p;
  if (!ora_parse_pubkey_hex(line, &p, compressed)) return 0;
  ora_u256_to_be(&p.x, xy_be);
  ora_u256_to_be(&p.y, xy_be + 32);
  return 1;
}
