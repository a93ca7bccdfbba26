// 256-bit unsigned integers for the host side of the engine: keys, ranges and BSGS geometry
// (the roles of the reference's Int, secp256k1/Int.h:40-194, restricted to non-negative values).
#pragma once
#include <stdint.h>
#include <string>

namespace khb {

struct U256 {
  uint64_t w[4] = {0, 0, 0, 0};   // little-endian limbs

  U256() = default;
  explicit U256(uint64_t v) { w[0] = v; }

  bool is_zero() const { return (w[0] | w[1] | w[2] | w[3]) == 0; }
  bool fits64() const { return (w[1] | w[2] | w[3]) == 0; }
  int bit(int i) const { return (int)((w[i >> 6] >> (i & 63)) & 1); }
  int bit_length() const;

  static int cmp(const U256& a, const U256& b);
  friend bool operator<(const U256& a, const U256& b) { return cmp(a, b) < 0; }
  friend bool operator<=(const U256& a, const U256& b) { return cmp(a, b) <= 0; }
  friend bool operator>(const U256& a, const U256& b) { return cmp(a, b) > 0; }
  friend bool operator>=(const U256& a, const U256& b) { return cmp(a, b) >= 0; }
  friend bool operator==(const U256& a, const U256& b) { return cmp(a, b) == 0; }
  friend bool operator!=(const U256& a, const U256& b) { return cmp(a, b) != 0; }

  // arithmetic mod 2^256; the carry/borrow out is returned where it matters
  static uint64_t add(U256& r, const U256& a, const U256& b);
  static uint64_t sub(U256& r, const U256& a, const U256& b);
  friend U256 operator+(const U256& a, const U256& b) { U256 r; add(r, a, b); return r; }
  friend U256 operator-(const U256& a, const U256& b) { U256 r; sub(r, a, b); return r; }
  friend U256 operator*(const U256& a, const U256& b);
  friend U256 operator*(const U256& a, uint64_t m);
  U256 shl(int n) const;
  U256 shr(int n) const;
  // q = a / b, r = a % b (b != 0)
  static void divmod(const U256& a, const U256& b, U256* q, U256* r);

  // parsing / printing (Int::SetBase16/SetBase10, Int::GetBase16 — lowercase, no leading zeros)
  static bool from_hex(const char* s, U256& out);
  static bool from_dec(const char* s, U256& out);
  std::string hex() const;
  std::string dec() const;
  void to_be(uint8_t out[32]) const;
  static U256 from_be(const uint8_t in[32]);
};

// a * b mod m (m != 0; a, b any): shift-and-add, for the rare key recoveries (keyhunt's ModMulK1order, -e).
U256 mulmod(const U256& a, const U256& b, const U256& m);

// Uniform random value in [lo, hi) from getrandom (Int::Rand, Int.cpp:751-765 / Random.cpp:133-145:
// the -R / -B random policies, non-deterministic like the reference's).
U256 random_in(const U256& lo, const U256& hi);

}  // namespace khb
