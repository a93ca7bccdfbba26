// Host-side secp256k1 group arithmetic for the engine's setup and confirmation work
// (secp256k1/SECP256K1.cpp: ComputePublicKey :61-82, AddDirect :242-265, DoubleDirect :376-401,
// Negation :103-111, ParsePublicKeyHex :114-170, GetPublicKeyHex :172-189).
//
// Field operations use the 4 x 64-bit host field of fh.hpp (canonical, like device/fe.hpp).
#pragma once
#include <stdint.h>
#include <string>
#include <vector>

#include "fh.hpp"
#include "u256.hpp"

namespace khb {

struct Pt {   // affine point, z == 1 (the reference's Point after Reduce)
  Fh x, y;
};

Fh fe_of(const U256& v);      // v < p
U256 u256_of(const Fh& f);
void fe_pow(Fh& r, const Fh& a, const U256& e);
bool fe_has_sqrt(const Fh& a);               // Int::HasSqrt (IntMod.cpp:563-574)
void fe_sqrt(Fh& r, const Fh& a);            // Int::ModSqrt, 0 when a is not a square (IntMod.cpp:578-596)
// In-place Montgomery batch inversion; zero elements stay zero (the product skips them).
void fe_batch_inv(Fh* v, size_t n, Fh* scratch);

const U256& secp_order();
const U256& secp_prime();
const Pt& secp_g();

Pt add_direct(const Pt& p1, const Pt& p2);   // reference semantics incl. dx == 0 -> s == 0
Pt double_direct(const Pt& p);
Pt negation(const Pt& p);                     // y = P - y
Pt mul_g(const U256& k);                      // k*G for 0 < k < n (ComputePublicKey)
bool on_curve(const Pt& p);

// Parse a 02/03 (66 chars) or 04 (130 chars) hex public key.  On failure returns false and sets
// err to the reference's message text.
bool parse_pubkey_hex(const char* s, Pt& out, bool& compressed, std::string* err);
std::string pubkey_hex(const Pt& p, bool compressed);
void pt_to_be(uint8_t out[64], const Pt& p);
// Secp256K1::Init's GTable (SECP256K1.cpp:43-54) as 32*256 points x||y BE: entry 256*i + j = (j+1)*2^(8i)*G
// for j < 255, entry 256*i + 255 = 2^(8(i+1))*G (the reference's "dummy" point).  Built once, cached.
const std::vector<uint8_t>& gtable_be();
Pt pt_from_be(const uint8_t in[64]);

}  // namespace khb
