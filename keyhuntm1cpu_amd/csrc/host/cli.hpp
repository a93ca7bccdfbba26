// Shared pieces of the keyhunt_amd CLI (keyhunt_main.cpp: option parsing and -m bsgs;
// keyhunt_address.cpp: -m address / -m rmd160).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "u256.hpp"

namespace khb {

// "[+] Total %s keys in %s seconds: ..." (keyhunt.cpp:2194-2238)
std::string speed_line(const U256& total, uint64_t seconds);

struct AddressCli {
  int mode = 1;                       // 1 address, 3 rmd160 (keyhunt.cpp:51-57)
  int search = 2;                     // -l (keyhunt.cpp:300: both)
  bool endomorphism = false;          // -e (keyhunt.cpp:579-585)
  bool crypto_set = false;            // -c given
  const char* stride = nullptr;       // -I
  bool random = false;                // -R
  bool quiet = false;                 // -q
  bool have_range = false;            // -r accepted
  U256 start, end;
  bool flag_bits = false;             // -b
  int bitrange = 0;
  std::string bits_min, bits_max;
  const char* file = nullptr;         // -f
  const char* str_n = nullptr;        // -n
  std::vector<int> devices{0};
  uint32_t lanes = 0;
  uint64_t max_chunks = 0;
  uint64_t out_seconds = 30;
  int bloom_multiplier = 1;
  int threads = 16;
};

int run_address_mode(const AddressCli& o);

}  // namespace khb
