#include "secp_host.hpp"

#include <mutex>
#include <string.h>
#include <vector>

namespace khb {

namespace {

const U256 kOrder = [] {
  U256 v;
  U256::from_hex("FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141", v);
  return v;
}();
const U256 kPrime = [] {
  U256 v;
  U256::from_hex("FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2F", v);
  return v;
}();
const Pt kG = [] {
  U256 x, y;
  U256::from_hex("79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798", x);
  U256::from_hex("483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8", y);
  Pt g;
  g.x = fe_of(x);
  g.y = fe_of(y);
  return g;
}();

// Jacobian point for scalar multiplication; inf marks the identity.
struct Jac {
  Fh X, Y, Z;
  bool inf = true;
};

void jac_double(Jac& r, const Jac& p) {
  if (p.inf || fe_is_zero(p.Y)) { r.inf = true; return; }
  Fh A, B, C, D, E, F, t;
  fe_sqr(A, p.X);
  fe_sqr(B, p.Y);
  fe_sqr(C, B);
  fe_add(t, p.X, B);
  fe_sqr(t, t);
  fe_sub(t, t, A);
  fe_sub(t, t, C);
  fe_add(D, t, t);
  fe_add(E, A, A);
  fe_add(E, E, A);
  fe_sqr(F, E);
  Jac o;
  o.inf = false;
  fe_sub(o.X, F, D);
  fe_sub(o.X, o.X, D);
  fe_sub(t, D, o.X);
  fe_mul(o.Y, E, t);
  Fh c8;
  fe_add(c8, C, C);
  fe_add(c8, c8, c8);
  fe_add(c8, c8, c8);
  fe_sub(o.Y, o.Y, c8);
  fe_mul(o.Z, p.Y, p.Z);
  fe_add(o.Z, o.Z, o.Z);
  r = o;
}

void jac_add_aff(Jac& r, const Jac& p, const Pt& q) {
  if (p.inf) {
    r.X = q.x; r.Y = q.y;
    r.Z = fh_one();
    r.inf = false;
    return;
  }
  Fh z2, u2, s2, H, R, HH, HHH, V, t;
  fe_sqr(z2, p.Z);
  fe_mul(u2, q.x, z2);
  fe_mul(s2, q.y, z2);
  fe_mul(s2, s2, p.Z);
  fe_sub(H, u2, p.X);
  fe_sub(R, s2, p.Y);
  if (fe_is_zero(H)) {
    if (fe_is_zero(R)) { jac_double(r, p); return; }
    r.inf = true;
    return;
  }
  fe_sqr(HH, H);
  fe_mul(HHH, H, HH);
  fe_mul(V, p.X, HH);
  Jac o;
  o.inf = false;
  fe_sqr(o.X, R);
  fe_sub(o.X, o.X, HHH);
  fe_sub(o.X, o.X, V);
  fe_sub(o.X, o.X, V);
  fe_sub(t, V, o.X);
  fe_mul(o.Y, R, t);
  fe_mul(t, p.Y, HHH);
  fe_sub(o.Y, o.Y, t);
  fe_mul(o.Z, p.Z, H);
  r = o;
}

// Fixed-base table: kTab[i][d-1] = d * 16^i * G, 64 windows x 15 digits, built once.
std::vector<Pt> g_tab;
std::once_flag g_tab_once;

void build_tab() {
  g_tab.resize(64 * 15);
  Pt base = kG;
  for (int i = 0; i < 64; ++i) {
    Pt acc = base;
    g_tab[i * 15] = acc;
    acc = double_direct(base);
    g_tab[i * 15 + 1] = acc;
    for (int d = 3; d <= 15; ++d) {
      acc = add_direct(acc, base);
      g_tab[i * 15 + d - 1] = acc;
    }
    base = add_direct(acc, base);   // 16 * base
  }
}

}  // namespace

Fh fe_of(const U256& v) {
  uint8_t b[32];
  v.to_be(b);
  Fh f;
  fe_from_be(f, b);
  return f;
}

U256 u256_of(const Fh& f) {
  uint8_t b[32];
  fe_to_be(b, f);
  return U256::from_be(b);
}

void fe_pow(Fh& r, const Fh& a, const U256& e) {
  Fh acc = fh_one();
  for (int i = e.bit_length() - 1; i >= 0; --i) {
    fe_sqr(acc, acc);
    if (e.bit(i)) fe_mul(acc, acc, a);
  }
  r = acc;
}

bool fe_has_sqrt(const Fh& a) {
  U256 e = (kPrime - U256(1)).shr(1);
  Fh t;
  fe_pow(t, a, e);
  return fe_eq(t, fh_one());
}

void fe_sqrt(Fh& r, const Fh& a) {
  if (!fe_has_sqrt(a)) { r = Fh{}; return; }
  U256 e = (kPrime + U256(1)).shr(2);
  fe_pow(r, a, e);
}

void fe_batch_inv(Fh* v, size_t n, Fh* pre) {
  Fh acc = fh_one();
  for (size_t i = 0; i < n; ++i) {
    pre[i] = acc;
    if (!fe_is_zero(v[i])) fe_mul(acc, acc, v[i]);
  }
  Fh inv;
  fe_inv(inv, acc);
  for (size_t i = n; i-- > 0;) {
    if (fe_is_zero(v[i])) continue;
    Fh vi = v[i];
    fe_mul(v[i], inv, pre[i]);
    fe_mul(inv, inv, vi);
  }
}

const U256& secp_order() { return kOrder; }
const U256& secp_prime() { return kPrime; }
const Pt& secp_g() { return kG; }

Pt add_direct(const Pt& p1, const Pt& p2) {
  Fh dy, dx, s, p;
  Pt r;
  fe_sub(dy, p2.y, p1.y);
  fe_sub(dx, p2.x, p1.x);
  fe_inv(dx, dx);                 // 0 when p1.x == p2.x (Int::ModInv CLEAR)
  fe_mul(s, dy, dx);
  fe_sqr(p, s);
  fe_sub(r.x, p, p1.x);
  fe_sub(r.x, r.x, p2.x);
  fe_sub(r.y, p2.x, r.x);
  fe_mul(r.y, r.y, s);
  fe_sub(r.y, r.y, p2.y);
  return r;
}

Pt double_direct(const Pt& pt) {
  Fh s, p, a;
  Pt r;
  fe_sqr(s, pt.x);
  fe_add(p, s, s);
  fe_add(p, p, s);
  fe_add(a, pt.y, pt.y);
  fe_inv(a, a);
  fe_mul(s, p, a);
  fe_sqr(p, s);
  fe_add(a, pt.x, pt.x);
  fe_sub(r.x, p, a);
  fe_sub(a, r.x, pt.x);
  fe_mul(p, a, s);
  fe_add(r.y, p, pt.y);
  Fh zero{};
  fe_sub(r.y, zero, r.y);
  return r;
}

Pt negation(const Pt& p) {
  Pt r;
  r.x = p.x;
  Fh zero{};
  fe_sub(r.y, zero, p.y);
  return r;
}

Pt mul_g(const U256& k) {
  std::call_once(g_tab_once, build_tab);
  Jac q;
  for (int i = 0; i < 64; ++i) {
    int d = (int)((k.w[i / 16] >> ((i % 16) * 4)) & 15);
    if (d) jac_add_aff(q, q, g_tab[i * 15 + d - 1]);
  }
  Pt r{};
  if (q.inf) return r;
  Fh zi, zi2, zi3;
  fe_inv(zi, q.Z);
  fe_sqr(zi2, zi);
  fe_mul(zi3, zi2, zi);
  fe_mul(r.x, q.X, zi2);
  fe_mul(r.y, q.Y, zi3);
  return r;
}

bool on_curve(const Pt& p) {
  Fh s, t, seven = fh_small(7);
  fe_sqr(s, p.x);
  fe_mul(t, s, p.x);
  fe_add(t, t, seven);
  fe_sqr(s, p.y);
  return fe_eq(s, t);
}

static int hv(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

bool parse_pubkey_hex(const char* s, Pt& out, bool& compressed, std::string* err) {
  const size_t len = strlen(s);
  auto fail = [&](const char* m) { if (err) *err = m; return false; };
  if (len < 2) return fail("ParsePublicKeyHex: Error invalid public key specified (66 or 130 character length)");
  uint8_t b[65];
  size_t nb = len / 2 < 65 ? len / 2 : 65;
  for (size_t i = 0; i < nb; ++i) {
    int h = hv(s[2 * i]), l = hv(s[2 * i + 1]);
    if (h < 0 || l < 0)
      return fail("ParsePublicKeyHex: Error invalid public key specified (unexpected hexadecimal digit)");
    b[i] = (uint8_t)(h * 16 + l);
  }
  Fh x, y;
  switch (b[0]) {
    case 0x02:
    case 0x03: {
      if (len != 66) return fail("ParsePublicKeyHex: Error invalid public key specified (66 character length)");
      fe_from_be(x, b + 1);
      Fh s3, t, seven = fh_small(7);
      fe_sqr(s3, x);
      fe_mul(t, s3, x);
      fe_add(t, t, seven);
      fe_sqrt(y, t);
      const bool odd = y.w[0] & 1;
      if (odd == (b[0] == 0x02)) { Fh zero{}; fe_sub(y, zero, y); }
      compressed = true;
      break;
    }
    case 0x04:
      if (len != 130) return fail("ParsePublicKeyHex: Error invalid public key specified (130 character length)");
      fe_from_be(x, b + 1);
      fe_from_be(y, b + 33);
      compressed = false;
      break;
    default:
      return fail("ParsePublicKeyHex: Error invalid public key specified (Unexpected prefix (only 02,03 or 04 allowed)");
  }
  out.x = x;
  out.y = y;
  if (!on_curve(out)) return fail("ParsePublicKeyHex: Error invalid public key specified (Not lie on elliptic curve)");
  return true;
}

std::string pubkey_hex(const Pt& p, bool compressed) {
  static const char* dg = "0123456789abcdef";
  uint8_t b[65];
  size_t n;
  if (compressed) {
    b[0] = (p.y.w[0] & 1) ? 3 : 2;
    fe_to_be(b + 1, p.x);
    n = 33;
  } else {
    b[0] = 4;
    fe_to_be(b + 1, p.x);
    fe_to_be(b + 33, p.y);
    n = 65;
  }
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; ++i) { s[2 * i] = dg[b[i] >> 4]; s[2 * i + 1] = dg[b[i] & 15]; }
  return s;
}

void pt_to_be(uint8_t out[64], const Pt& p) {
  fe_to_be(out, p.x);
  fe_to_be(out + 32, p.y);
}

Pt pt_from_be(const uint8_t in[64]) {
  Pt p;
  fe_from_be(p.x, in);
  fe_from_be(p.y, in + 32);
  return p;
}

// Secp256K1::Init (SECP256K1.cpp:43-54): N = G; per window i: GTable[256i] = N, N = 2N, then
// GTable[256i + j] = N, N += GTable[256i] for j < 255, GTable[256i + 255] = N.  The same chain of
// DoubleDirect / AddDirect, so every entry is the reference's point.
const std::vector<uint8_t>& gtable_be() {
  static std::once_flag once;
  static std::vector<uint8_t> tab;
  std::call_once(once, [] {
    tab.assign(32 * 256 * 64, 0);
    Pt n = secp_g();
    for (int i = 0; i < 32; ++i) {
      const Pt w = n;
      pt_to_be(tab.data() + 64 * (256 * i), w);
      n = double_direct(n);
      for (int j = 1; j < 255; ++j) {
        pt_to_be(tab.data() + 64 * (256 * i + j), n);
        n = add_direct(n, w);
      }
      pt_to_be(tab.data() + 64 * (256 * i + 255), n);
    }
  });
  return tab;
}

}  // namespace khb
