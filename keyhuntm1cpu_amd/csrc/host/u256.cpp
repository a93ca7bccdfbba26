#include "u256.hpp"

#include <string.h>
#include <sys/random.h>

namespace khb {

typedef unsigned __int128 u128;

int U256::bit_length() const {
  for (int i = 3; i >= 0; --i)
    if (w[i]) return 64 * i + (64 - __builtin_clzll(w[i]));
  return 0;
}

int U256::cmp(const U256& a, const U256& b) {
  for (int i = 3; i >= 0; --i)
    if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
  return 0;
}

uint64_t U256::add(U256& r, const U256& a, const U256& b) {
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c += (u128)a.w[i] + b.w[i];
    r.w[i] = (uint64_t)c;
    c >>= 64;
  }
  return (uint64_t)c;
}

uint64_t U256::sub(U256& r, const U256& a, const U256& b) {
  uint64_t br = 0;
  for (int i = 0; i < 4; ++i) {
    u128 d = (u128)a.w[i] - b.w[i] - br;
    r.w[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  return br;
}

U256 operator*(const U256& a, const U256& b) {
  U256 r;
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; i + j < 4; ++j) {
      c += (u128)a.w[j] * b.w[i] + r.w[i + j];
      r.w[i + j] = (uint64_t)c;
      c >>= 64;
    }
  }
  return r;
}

U256 operator*(const U256& a, uint64_t m) {
  U256 r;
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c += (u128)a.w[i] * m;
    r.w[i] = (uint64_t)c;
    c >>= 64;
  }
  return r;
}

U256 U256::shl(int n) const {
  U256 r;
  if (n >= 256) return r;
  int q = n / 64, s = n % 64;
  for (int i = 3; i >= q; --i) {
    uint64_t v = w[i - q] << s;
    if (s && i - q - 1 >= 0) v |= w[i - q - 1] >> (64 - s);
    r.w[i] = v;
  }
  return r;
}

U256 U256::shr(int n) const {
  U256 r;
  if (n >= 256) return r;
  int q = n / 64, s = n % 64;
  for (int i = 0; i + q < 4; ++i) {
    uint64_t v = w[i + q] >> s;
    if (s && i + q + 1 < 4) v |= w[i + q + 1] << (64 - s);
    r.w[i] = v;
  }
  return r;
}

void U256::divmod(const U256& a, const U256& b, U256* q, U256* r) {
  U256 qq, rr;
  for (int i = a.bit_length() - 1; i >= 0; --i) {
    uint64_t top = rr.w[3] >> 63;
    rr = rr.shl(1);
    rr.w[0] |= (uint64_t)a.bit(i);
    if (top || rr >= b) {
      sub(rr, rr, b);
      qq.w[i >> 6] |= 1ull << (i & 63);
    }
  }
  if (q) *q = qq;
  if (r) *r = rr;
}

static int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

bool U256::from_hex(const char* s, U256& out) {
  U256 v;
  if (!s || !*s) return false;
  for (; *s; ++s) {
    int d = hexval(*s);
    if (d < 0) return false;
    if (v.w[3] >> 60) return false;   // overflow
    v = v.shl(4);
    v.w[0] |= (uint64_t)d;
  }
  out = v;
  return true;
}

bool U256::from_dec(const char* s, U256& out) {
  U256 v;
  if (!s || !*s) return false;
  for (; *s; ++s) {
    if (*s < '0' || *s > '9') return false;
    v = v * 10ull;
    add(v, v, U256((uint64_t)(*s - '0')));
  }
  out = v;
  return true;
}

std::string U256::hex() const {
  static const char* dg = "0123456789abcdef";
  std::string s;
  for (int i = 63; i >= 0; --i) {
    int nib = (int)((w[i / 16] >> ((i % 16) * 4)) & 15);
    if (s.empty() && nib == 0) continue;
    s.push_back(dg[nib]);
  }
  if (s.empty()) s = "0";
  return s;
}

std::string U256::dec() const {
  if (is_zero()) return "0";
  std::string s;
  U256 v = *this, q, r;
  const U256 ten(10);
  while (!v.is_zero()) {
    divmod(v, ten, &q, &r);
    s.insert(s.begin(), (char)('0' + r.w[0]));
    v = q;
  }
  return s;
}

void U256::to_be(uint8_t out[32]) const {
  for (int i = 0; i < 32; ++i) out[i] = (uint8_t)(w[3 - i / 8] >> (56 - 8 * (i % 8)));
}

U256 U256::from_be(const uint8_t in[32]) {
  U256 r;
  for (int i = 0; i < 4; ++i) {
    uint64_t v = 0;
    for (int j = 0; j < 8; ++j) v = (v << 8) | in[(3 - i) * 8 + j];
    r.w[i] = v;
  }
  return r;
}

U256 random_in(const U256& lo, const U256& hi) {
  U256 span = hi - lo, v, r;
  uint8_t b[32];
  if (getrandom(b, sizeof b, 0) != (ssize_t)sizeof b) memset(b, 0x5a, sizeof b);
  v = U256::from_be(b);
  if (span.is_zero()) return lo;
  U256::divmod(v, span, nullptr, &r);
  return lo + r;
}

U256 mulmod(const U256& a0, const U256& b, const U256& m) {
  U256 a, acc;
  U256::divmod(a0, m, nullptr, &a);
  for (int i = 255; i >= 0; --i) {
    uint64_t c = U256::add(acc, acc, acc);
    if (c || acc >= m) U256::sub(acc, acc, m);
    if (b.bit(i)) {
      c = U256::add(acc, acc, a);
      if (c || acc >= m) U256::sub(acc, acc, m);
    }
  }
  return acc;
}

}  // namespace khb
