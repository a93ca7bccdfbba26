// keyhunt_amd — keyhunt-compatible CLI for the `-m bsgs` path on MI355X.
//
// Flags, target-file rules and output follow keyhunt.cpp main() (415-2259): getopt string
// (489), -b (508-527), -r (678-712, 816-838), -k (595-601), -n (665-668, 1052-1067), -t, -q,
// -s, -R/-B (498-507, 673-677), target file (962-1044), geometry/bloom prints (1045-1303),
// found-key output (3950-3981) and the stats line (2145-2252).  GPU selection follows the
// reference README's documented interface (README.md:115-122): --gpu, -g <ids>, --gpu-blocks.
#include <getopt.h>
#include <math.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/random.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/khbsgs.h"
#include "bsgs_host.hpp"
#include "cli.hpp"
#include "engine.hpp"

using namespace khb;

namespace {

const char* kVersion = "1.0.0 keyhunt_amd (MI355X BSGS engine)";
const char* kBsgsModes[5] = {"sequential", "backward", "both", "random", "dance"};   // keyhunt.cpp:227
const char* kModes[7] = {"xpoint", "address", "bsgs", "rmd160", "pub2rmd", "minikeys", "vanity"};
const char* kLimitPrefix[7] = {"Mkeys/s", "Gkeys/s", "Tkeys/s", "Pkeys/s", "Ekeys/s", "Zkeys/s", "Ykeys/s"};

void menu() {
  printf("\nUsage:\n");
  printf("-h          show this help\n");
  printf("-B Mode     BSGS now have some modes <sequential, backward, both, random, dance>\n");
  printf("-b bits     For some puzzles you only need some numbers of bits in the test keys.\n");
  printf("-f file     Specify file name with public keys (02/03 compressed or 04 uncompressed hex)\n");
  printf("-k value    Use this only with bsgs mode, k value is factor for M, more speed but more RAM use wisely\n");
  printf("-m mode     mode of search for cryptos. (bsgs) default: bsgs\n");
  printf("-M          Matrix screen, feel like a h4x0r, but performance will dropped\n");
  printf("-n number   Use -n to set the N for the BSGS process. Bigger N more RAM needed\n");
  printf("-q          Quiet the thread output\n");
  printf("-r SR:EN    StarRange:EndRange, the end range can be omitted for search from start range to N-1 ECC value\n");
  printf("-R          Random, this is the default behavior\n");
  printf("-s ns       Number of seconds for the stats output, 0 to omit output.\n");
  printf("-t tn       CPU threads for table build and candidate confirmation\n");
  printf("--cpu-build build the baby-step tables on the CPU (default: on the first GPU)\n");
  printf("-6          to skip sha256 Checksum on data files\n");
  printf("--gpu       use the GPU path (always on: keyhunt_amd has no CPU giant-step path)\n");
  printf("-g ids      GPU device ids, comma separated (default 0)\n");
  printf("--gpu-blocks n   persistent workgroups per GPU (256 lanes each)\n");
  printf("--check where    confirm candidates (second/third check) on the host, the gpu, or auto (default host)\n");
  printf("--no-gate   probe every giant step in the level-1 bloom (no level-0 gate; same keys, more candidates)\n");
  printf("\nExample:\n\n./keyhunt_amd -m bsgs -f tests/63.pub -b 63 -q -g 0\n\n");
  exit(EXIT_FAILURE);
}

void trim(char* s) {   // trim(aux," \t\n\r") (util.c)
  size_t n = strlen(s);
  while (n && strchr(" \t\n\r", s[n - 1])) s[--n] = 0;
  size_t i = 0;
  while (s[i] && strchr(" \t\n\r", s[i])) ++i;
  if (i) memmove(s, s + i, strlen(s + i) + 1);
}

int index_of(const char* s, const char** arr, int n) {
  for (int i = 0; i < n; ++i)
    if (strcmp(s, arr[i]) == 0) return i;
  return -1;
}

bool valid_hex(const char* s) {   // isValidHex (util.c:169-178)
  if (!*s) return false;
  for (; *s; ++s)
    if (!isxdigit((unsigned char)*s)) return false;
  return true;
}

std::vector<std::string> tokens(const char* s) {   // stringtokenizer: split on " \t:"
  std::vector<std::string> out;
  std::string cur;
  for (const char* p = s; *p; ++p) {
    if (strchr(" \t:", *p)) {
      if (!cur.empty()) out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(*p);
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

U256 rand_range(const U256& lo, const U256& hi) {
  uint8_t b[32];
  if (getrandom(b, sizeof b, 0) != (ssize_t)sizeof b) {
    fprintf(stderr, "[E] Error getrandom() ?\n");
    exit(EXIT_FAILURE);
  }
  U256 v = U256::from_be(b), r;
  U256 span = hi - lo;
  if (span.is_zero()) return lo;
  U256::divmod(v, span, nullptr, &r);
  return lo + r;
}

}  // namespace

namespace khb {

std::string speed_line(const U256& total, uint64_t seconds) {   // keyhunt.cpp:2194-2238
  U256 per = total, q;
  U256::divmod(total, U256(seconds ? seconds : 1), &per, nullptr);
  U256 lim[7];
  const char* ls[7] = {"1000000", "1000000000", "1000000000000", "1000000000000000", "1000000000000000000",
                       "1000000000000000000000", "1000000000000000000000000"};
  for (int j = 0; j < 7; ++j) U256::from_dec(ls[j], lim[j]);
  char buf[512];
  if (per < lim[0]) {
    snprintf(buf, sizeof buf, "[+] Total %s keys in %llu seconds: %s keys/s", total.dec().c_str(),
             (unsigned long long)seconds, per.dec().c_str());
  } else {
    int i = 0;
    bool salir = false;
    while (i < 6 && !salir) {
      if (per < lim[i + 1]) salir = true; else i++;
    }
    const int idx = salir ? i : i - 1;
    U256::divmod(per, lim[idx], &q, nullptr);
    snprintf(buf, sizeof buf, "[+] Total %s keys in %llu seconds: ~%s %s (%s keys/s)", total.dec().c_str(),
             (unsigned long long)seconds, q.dec().c_str(), kLimitPrefix[idx], per.dec().c_str());
  }
  return buf;
}

}  // namespace khb

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  printf("[+] Version %s\n", kVersion);
  int mode = 2;   // bsgs
  int bsgs_mode = 0, kfactor = 1, nthreads = (int)std::thread::hardware_concurrency();
  bool quiet = false, matrix = false, flag_range = false, flag_bits = false;
  const char* file = nullptr;
  const char* str_n = nullptr;
  std::string range_start, range_end, bits_min, bits_max;
  uint64_t out_seconds = 30;
  int bitrange = 0;
  SearchConfig cfg;
  uint32_t gpu_blocks = 0;
  AddressCli ao;
  bool save_read_file = false, skip_checksum = false, cpu_build = false;
  bool endomorphism = false, eth = false;
  const char* kSearch[3] = {"uncompress", "compress", "both"};   // keyhunt.cpp:230
  if (nthreads > 16) nthreads = 16;
  static struct option longopts[] = {{"gpu", no_argument, nullptr, 1000},
                                     {"gpu-threads", required_argument, nullptr, 1001},
                                     {"gpu-blocks", required_argument, nullptr, 1002},
                                     {"max-chunks", required_argument, nullptr, 1003},
                                     {"cpu-build", no_argument, nullptr, 1004},
                                     {"check", required_argument, nullptr, 1005},
                                     {"no-gate", no_argument, nullptr, 1006},
                                     {nullptr, 0, nullptr, 0}};
  int c;
  while ((c = getopt_long(argc, argv, "deh6MqRSB:b:c:C:E:f:I:k:l:m:N:n:p:r:s:t:v:G:8:z:g:", longopts, nullptr)) != -1) {
    switch (c) {
      case 'h': menu(); break;
      case '6': skip_checksum = true; fprintf(stderr, "[W] Skipping checksums on files\n"); break;
      case 'B': {
        int v = index_of(optarg, kBsgsModes, 5);
        if (v >= 0) bsgs_mode = v; else fprintf(stderr, "[W] Ignoring unknow bsgs mode %s\n", optarg);
        break;
      }
      case 'b':
        bitrange = (int)strtol(optarg, nullptr, 10);
        if (bitrange > 0 && bitrange <= 256) {
          U256 mn = U256(1).shl(bitrange - 1), mx = U256(1).shl(bitrange);
          if (bitrange == 256 || mx > secp_order()) mx = secp_order();
          bits_min = mn.hex();
          bits_max = mx.hex();
          flag_bits = true;
        } else {
          fprintf(stderr, "[E] invalid bits param: %s.\n", optarg);
        }
        break;
      case 'd': printf("[+] Flag DEBUG enabled\n"); break;
      case 'e': endomorphism = true; printf("[+] Endomorphism enabled\n"); break;
      case 'c': {
        const char* cryptos[2] = {"btc", "eth"};
        const int v = index_of(optarg, cryptos, 2);
        if (v == 1) { eth = true; printf("[+] Setting search for ETH adddress.\n"); }
        if (v >= 0) ao.crypto_set = true;
        break;
      }
      case 'I': ao.stride = optarg; break;
      case 'l':
        switch (index_of(optarg, kSearch, 3)) {
          case 0: ao.search = 0; printf("[+] Search uncompress only\n"); break;
          case 1: ao.search = 1; printf("[+] Search compress only\n"); break;
          case 2: ao.search = 2; printf("[+] Search both compress and uncompress\n"); break;
        }
        break;
      case 'f': file = optarg; break;
      case 'k':
        kfactor = (int)strtol(optarg, nullptr, 10);
        if (kfactor <= 0) kfactor = 1;
        printf("[+] K factor %i\n", kfactor);
        break;
      case 'M': matrix = true; printf("[+] Matrix screen\n"); break;
      case 'm':
        mode = index_of(optarg, kModes, 7);
        if (mode < 0) { fprintf(stderr, "[E] Unknow mode value %s\n", optarg); exit(EXIT_FAILURE); }
        if (mode == 1) printf("[+] Mode address\n");
        if (mode == 3) printf("[+] Mode rmd160\n");
        break;
      case 'n': str_n = optarg; break;
      case 'q': quiet = true; printf("[+] Quiet thread output\n"); break;
      case 'R': printf("[+] Random mode\n"); bsgs_mode = 3; break;
      case 'r': {
        std::vector<std::string> t = tokens(optarg);
        if (t.size() == 1) {
          if (valid_hex(t[0].c_str())) { flag_range = true; range_start = t[0]; range_end = secp_order().hex(); }
          else fprintf(stderr, "[E] Invalid hexstring : %s.\n", t[0].c_str());
        } else if (t.size() == 2) {
          if (valid_hex(t[0].c_str()) && valid_hex(t[1].c_str())) { flag_range = true; range_start = t[0]; range_end = t[1]; }
          else fprintf(stderr, "[E] Invalid hexstring : %s\n", valid_hex(t[0].c_str()) ? t[1].c_str() : t[0].c_str());
        } else {
          printf("[E] Unknow number of Range Params: %i\n", (int)t.size());
        }
        break;
      }
      case 's':
        out_seconds = strtoull(optarg, nullptr, 10);
        if (out_seconds == 0) printf("[+] Turn off stats output\n");
        else printf("[+] Stats output every %llu seconds\n", (unsigned long long)out_seconds);
        break;
      case 'S': save_read_file = true; break;
      case 't':
        nthreads = (int)strtol(optarg, nullptr, 10);
        if (nthreads <= 0) nthreads = 1;
        printf(nthreads > 1 ? "[+] Threads : %u\n" : "[+] Thread : %u\n", nthreads);
        break;
      case 'g': {
        cfg.devices.clear();
        for (const std::string& s : tokens(std::string(optarg).c_str())) {
          std::string part;
          for (char ch : s + ",") {
            if (ch == ',') { if (!part.empty()) cfg.devices.push_back(atoi(part.c_str())); part.clear(); }
            else part.push_back(ch);
          }
        }
        if (cfg.devices.empty()) cfg.devices.push_back(0);
        break;
      }
      case 1000: break;                             // --gpu: the only path
      case 1001: break;                             // --gpu-threads: fixed 256-lane workgroups
      case 1002: gpu_blocks = (uint32_t)strtoul(optarg, nullptr, 10); break;
      case 1003: cfg.max_chunks = strtoull(optarg, nullptr, 10); break;
      case 1004: cpu_build = true; break;
      case 1005:                                    // where candidates are confirmed (engine.hpp check_mode)
        if ((cfg.check_mode = parse_check_mode(optarg)) < 0) {
          fprintf(stderr, "[E] --check: host, gpu or auto\n");
          exit(EXIT_FAILURE);
        }
        break;
      case 1006: cfg.use_gate = false; break;       // the reference's exact level-1 candidate stream
      case 'z':                                     // keyhunt.cpp:766-772 (used by initBloomFilter, 6559-6576)
        ao.bloom_multiplier = (int)strtol(optarg, nullptr, 10);
        if (ao.bloom_multiplier <= 0) ao.bloom_multiplier = 1;
        printf("[+] Bloom Size Multiplier %i\n", ao.bloom_multiplier);
        break;
      case 'C': case 'E': case 'N': case 'p': case 'v': case 'G': case '8':
        break;   // options of the other search modes
      default:
        fprintf(stderr, "[E] Unknow opcion -%c\n", c);
        exit(EXIT_FAILURE);
    }
  }
  // keyhunt.cpp:780-789: compared with MODE_BSGS (2), i.e. the -B sub-mode "both", whatever -m is
  if (bsgs_mode == 2 && endomorphism) {
    fprintf(stderr, "[E] Endomorphism doesn't work with BSGS\n");
    exit(EXIT_FAILURE);
  }
  if (bsgs_mode == 2 && ao.stride) {
    fprintf(stderr, "[E] Stride doesn't work with BSGS\n");
    exit(EXIT_FAILURE);
  }
  if (mode == 1 || mode == 3) {
    if (eth) {
      fprintf(stderr, "[E] keyhunt_amd searches BTC P2PKH addresses only (-c eth is not available)\n");
      exit(EXIT_FAILURE);
    }
    ao.endomorphism = endomorphism;   // keyhunt.cpp:2646-2937 (BTC)
    ao.mode = mode;
    ao.random = bsgs_mode == 3;
    ao.quiet = quiet;
    ao.file = file;
    ao.str_n = str_n;
    ao.devices = cfg.devices;
    ao.lanes = gpu_blocks * 256u;
    ao.max_chunks = cfg.max_chunks;
    ao.out_seconds = out_seconds;
    ao.threads = nthreads;
    ao.flag_bits = flag_bits;
    ao.bitrange = bitrange;
    ao.bits_min = bits_min;
    ao.bits_max = bits_max;
    if (flag_range) {   // keyhunt.cpp:816-838
      U256 a, b;
      U256::from_hex(range_start.c_str(), a);
      if (a.is_zero()) a = U256(1);
      U256::from_hex(range_end.c_str(), b);
      if (a != b) {
        if (a < secp_order() && b <= secp_order()) {
          if (a > b) {
            fprintf(stderr, "[W] Opps, start range can't be great than end range. Swapping them\n");
            std::swap(a, b);
          }
          ao.have_range = true;
          ao.start = a;
          ao.end = b;
        } else {
          fprintf(stderr, "[E] Start and End range can't be great than N\nFallback to random mode!\n");
        }
      } else {
        fprintf(stderr, "[E] Start and End range can't be the same\nFallback to random mode!\n");
      }
    }
    return run_address_mode(ao);
  }
  if (mode != 2) {
    fprintf(stderr, "[E] keyhunt_amd implements -m bsgs, -m address and -m rmd160 (mode %s is not available)\n",
            kModes[mode]);
    exit(EXIT_FAILURE);
  }
  // -e / -I outside the sub-mode "both" are ignored by -m bsgs, as there (keyhunt.cpp:780-789 above)
  printf("[+] Mode BSGS %s\n", kBsgsModes[bsgs_mode]);
  if (!file) file = "addresses.txt";   // default_fileName, keyhunt.cpp:231
  if (gpu_blocks) cfg.lanes = gpu_blocks * 256u;
  cfg.chunk_mode = bsgs_mode;                       // sequential, backward, both, random, dance
  cfg.random_chunks = bsgs_mode == 3;
  cfg.check_threads = nthreads;

  // ---- range (keyhunt.cpp:816-838, 1089-1119)
  U256 n_start, n_end;
  bool have_range = false;
  if (flag_range) {
    U256::from_hex(range_start.c_str(), n_start);
    if (n_start.is_zero()) n_start = U256(1);
    U256::from_hex(range_end.c_str(), n_end);
    if (n_start != n_end) {
      if (n_start < secp_order() && n_end <= secp_order()) {
        if (n_start > n_end) {
          fprintf(stderr, "[W] Opps, start range can't be great than end range. Swapping them\n");
          std::swap(n_start, n_end);
        }
        have_range = true;
      } else {
        fprintf(stderr, "[E] Start and End range can't be great than N\nFallback to random mode!\n");
      }
    } else {
      fprintf(stderr, "[E] Start and End range can't be the same\nFallback to random mode!\n");
    }
  }

  // ---- target file (keyhunt.cpp:962-1044)
  printf("[+] Opening file %s\n", file);
  FILE* fd = fopen(file, "rb");
  if (!fd) { fprintf(stderr, "[E] Can't open file %s\n", file); exit(EXIT_FAILURE); }
  std::vector<Target> targets;
  int counted = 0;
  char line[1024];
  while (fgets(line, 1022, fd)) {
    trim(line);
    if (strlen(line) >= 66) counted++;
  }
  if (counted == 0) { fprintf(stderr, "[E] There is no valid data in the file\n"); exit(EXIT_FAILURE); }
  fseek(fd, 0, SEEK_SET);
  while (fgets(line, 1022, fd)) {
    trim(line);
    if (strlen(line) < 66) continue;
    std::vector<std::string> t = tokens(line);
    if (t.empty()) continue;
    const std::string& tok = t[0];
    if (tok.size() == 66 || tok.size() == 130) {
      Target tg;
      std::string e;
      if (parse_pubkey_hex(tok.c_str(), tg.p, tg.compressed, &e)) targets.push_back(tg);
      else printf("%s\n", e.c_str());
    } else {
      printf("Invalid length: %s\n", tok.c_str());
    }
  }
  fclose(fd);
  if (targets.empty()) { fprintf(stderr, "[E] The file don't have any valid publickeys\n"); exit(EXIT_FAILURE); }
  printf("[+] Added %u points from file\n", (unsigned)targets.size());

  // ---- geometry (keyhunt.cpp:1045-1213)
  Geometry geo;
  std::string err;
  if (!make_geometry(str_n, kfactor, geo, err)) { fprintf(stderr, "%s\n", err.c_str()); exit(EXIT_FAILURE); }
  if (flag_bits && !have_range) {
    U256::from_hex(bits_min.c_str(), n_start);
    U256::from_hex(bits_max.c_str(), n_end);
    printf("[+] Bit Range %i\n", bitrange);
    printf("[+] -- from : 0x%s\n", bits_min.c_str());
    printf("[+] -- to   : 0x%s\n", bits_max.c_str());
    have_range = true;
  } else if (have_range) {
    printf("[+] Range \n");
    printf("[+] -- from : 0x%s\n", range_start.c_str());
    printf("[+] -- to   : 0x%s\n", range_end.c_str());
  }
  if (!have_range) {   // random start, keyhunt.cpp:1106-1112
    n_start = rand_range(U256(1), secp_order());
    n_end = secp_order();
  }
  if (n_end - n_start < geo.N) { fprintf(stderr, "[E] the given range is small\n"); exit(EXIT_FAILURE); }
  printf("[+] N = 0x%s\n", geo.N.hex().c_str());

  // ---- tables
  Tables T;
  auto mb = [](uint64_t bytes) { return (float)bytes / 1048576.0f; };
  {
    BloomFilter b;
    b.init2(geo.items1, 0.000001);
    printf("[+] Bloom filter for %llu elements : %.2f MB\n", (unsigned long long)geo.m, mb(b.bytes * 256));
    b.init2(geo.items2, 0.000001);
    printf("[+] Bloom filter for %llu elements : %.2f MB\n", (unsigned long long)geo.m2, mb(b.bytes * 256));
    b.init2(geo.items3, 0.000001);
    printf("[+] Bloom filter for %llu elements : %.2f MB\n", (unsigned long long)geo.m3, mb(b.bytes * 256));
    printf("[+] Allocating %.2f MB for %llu bP Points\n", (double)(geo.m3 * 16 / 1048576), (unsigned long long)geo.m3);
  }
  // -S: the reference's table files in the working directory (keyhunt.cpp:1373-1613)
  uint32_t have = 0;
  auto say = [](const std::string& m) { printf("%s", m.c_str()); fflush(stdout); };
  if (save_read_file) {
    T.prepare(geo);
    if (!T.load_files(".", skip_checksum, have, err, say)) {
      fprintf(stderr, "%s\n", err.c_str());
      exit(EXIT_FAILURE);
    }
    if (have && have != kFileAll && (have & kFileL1))
      printf("[I] We need to recalculate some files, don't worry this is only 3%% of the previous work\n");
  }
  if (have != kFileAll || !save_read_file) {
    // baby steps on the first GPU unless --cpu-build (identical tables; tests/test_gpu_tables.py)
    if (!T.build(geo, nthreads, 4, err, [&](uint64_t d, uint64_t tot) {
          printf("\r[+] processing %llu/%llu bP points : %i%%\r", (unsigned long long)d, (unsigned long long)tot,
                 (int)((double)d / (double)tot * 100));
          fflush(stdout);
        }, have, cpu_build ? -1 : cfg.devices[0])) {
      fprintf(stderr, "%s\n", err.c_str());
      exit(EXIT_FAILURE);
    }
    const uint64_t ext = (have & kFileL1) ? geo.m2 : geo.l1ext;
    printf("\r[+] processing %llu/%llu bP points : 100%%     \n", (unsigned long long)ext, (unsigned long long)ext);
    if (!(have & kFileBp)) printf("[+] Sorting %llu elements... Done!\n", (unsigned long long)geo.m3);
  } else if (!T.build(geo, nthreads, 4, err, nullptr, have)) {   // giant tables + lane offsets only
    fprintf(stderr, "%s\n", err.c_str());
    exit(EXIT_FAILURE);
  }
  if (save_read_file && have != kFileAll && !T.save_files(".", have, err, say)) {   // keyhunt.cpp:1881-2025
    fprintf(stderr, "%s\n", err.c_str());
    exit(EXIT_FAILURE);
  }

  // ---- search
  std::mutex out_mu;
  std::atomic<bool> finished{false};
  SearchCallbacks cb;
  cb.on_found = [&](int k, const U256& key) {   // keyhunt.cpp:3950-3971
    std::lock_guard<std::mutex> lk(out_mu);
    std::string kh = key.hex();
    printf("[+] Thread Key found privkey %s   \n", kh.c_str());
    std::string ph = pubkey_hex(mul_g(key), targets[k].compressed);
    printf("[+] Publickey %s\n", ph.c_str());
    FILE* f = fopen("KEYFOUNDKEYFOUND.txt", "a");
    if (f) {
      fprintf(f, "Key found privkey %s\nPublickey %s\n", kh.c_str(), ph.c_str());
      fclose(f);
    }
  };
  cb.on_chunk = [&](const U256& base) {             // keyhunt.cpp:3846-3860
    if (quiet) return;
    std::lock_guard<std::mutex> lk(out_mu);
    if (matrix) printf("[+] Thread 0x%s \n", base.hex().c_str());
    else { printf("\r[+] Thread 0x%s   \r", base.hex().c_str()); fflush(stdout); }
  };
  cb.on_warning = [&](const std::string& m) {
    std::lock_guard<std::mutex> lk(out_mu);
    fprintf(stderr, "%s\n", m.c_str());
  };
  std::vector<int> found;
  std::vector<U256> keys;
  SearchStats stats;
  auto t0 = std::chrono::steady_clock::now();
  std::thread stat_thread([&]() {                  // keyhunt.cpp:2154-2252
    uint64_t seconds = 0;
    while (!finished.load()) {
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
      auto el = std::chrono::duration_cast<std::chrono::seconds>(std::chrono::steady_clock::now() - t0).count();
      if ((uint64_t)el <= seconds) continue;
      seconds = (uint64_t)el;
      if (out_seconds == 0 || seconds % out_seconds) continue;
      uint64_t chunks;
      {
        std::lock_guard<std::mutex> lk(out_mu);
        chunks = __atomic_load_n(&stats.chunks, __ATOMIC_RELAXED);
        U256 total = geo.N_double * chunks;       // steps += 2 per chunk, keys = steps * N
        std::string s = speed_line(total, seconds);
        uint64_t gs = __atomic_load_n(&stats.giant_steps, __ATOMIC_RELAXED);
        if (matrix) printf("%s [%.3f G giant-steps/s]\n", s.c_str(), (double)gs / seconds / 1e9);
        else { printf("\r%s [%.3f G giant-steps/s]\r", s.c_str(), (double)gs / seconds / 1e9); fflush(stdout); }
      }
    }
  });
  int rc = run_search(T, targets, n_start, n_end, cfg, cb, found, keys, stats, err);
  finished = true;
  stat_thread.join();
  if (rc) { fprintf(stderr, "%s\n", err.c_str()); exit(EXIT_FAILURE); }
  int all = 1;
  for (int f : found) all &= f;
  if (all) {
    printf("All points were found\n");
    exit(EXIT_FAILURE);   // the reference exits with status 1 on success (keyhunt.cpp:3979-3980)
  }
  printf("\nEnd\n");
  return 0;
}
