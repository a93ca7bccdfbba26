// keyhunt_amd -m address / -m rmd160: keyhunt.cpp main() (800-960 setup and prints, 2145-2252 stats)
// and thread_process's output (writekey, keyhunt.cpp:5989-6030) over the libkhbsgs address scan.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>

#include "address_host.hpp"
#include "cli.hpp"

namespace khb {

namespace {

// writekey (keyhunt.cpp:5989-6030)
void writekey(const AddrFound& f, std::mutex& mu) {
  const Pt pub = mul_g(f.key);
  const std::string hexkey = f.key.hex();
  const std::string pubhex = pubkey_hex(pub, f.compressed);
  const std::string addr = rmd_to_address(f.rmd.data());
  char rmdhex[41];
  for (int i = 0; i < 20; ++i) snprintf(rmdhex + 2 * i, 3, "%02x", f.rmd[i]);
  std::lock_guard<std::mutex> lk(mu);
  FILE* keys = fopen("KEYFOUNDKEYFOUND.txt", "a+");
  if (keys) {
    fprintf(keys, "Private Key: %s\npubkey: %s\nAddress %s\nrmd160 %s\n", hexkey.c_str(), pubhex.c_str(), addr.c_str(),
            rmdhex);
    fclose(keys);
  }
  printf("\nHit! Private Key: %s\npubkey: %s\nAddress %s\nrmd160 %s\n", hexkey.c_str(), pubhex.c_str(), addr.c_str(),
         rmdhex);
  fflush(stdout);
}

}  // namespace

int run_address_mode(const AddressCli& o) {
  if (!o.crypto_set && o.mode == 1) printf("[+] Setting search for btc adddress\n");   // keyhunt.cpp:812-815
  U256 stride(1);
  if (o.stride) {   // keyhunt.cpp:790-797
    const bool ok = (o.stride[0] == '0' && o.stride[1] == 'x') ? U256::from_hex(o.stride + 2, stride)
                                                                : U256::from_dec(o.stride, stride);
    if (!ok || stride.is_zero()) {
      fprintf(stderr, "[E] invalid stride %s\n", o.stride);
      return EXIT_FAILURE;
    }
    printf("[+] Stride : %s\n", stride.dec().c_str());
  }
  const char* file = o.file ? o.file : "addresses.txt";   // default_fileName
  // range (keyhunt.cpp:844-864)
  U256 start(1), end = secp_order();
  if (o.have_range) {
    start = o.start;
    end = o.end;
  } else if (o.flag_bits) {
    U256::from_hex(o.bits_min.c_str(), start);
    U256::from_hex(o.bits_max.c_str(), end);
  }
  // -n (keyhunt.cpp:866-887)
  uint64_t n_seq = 0x100000000ull;
  if (o.str_n) {
    const uint64_t v = (o.str_n[0] == '0' && o.str_n[1] == 'x') ? strtoull(o.str_n, nullptr, 16)
                                                                 : strtoull(o.str_n, nullptr, 10);
    if (v < 1024) {
      fprintf(stderr, "[I] n value need to be equal or great than 1024, back to defaults\n");
    } else if (v % 1024 != 0) {
      fprintf(stderr, "[I] n value need to be multiplier of  1024\n");
    } else {
      n_seq = v;
    }
  }
  printf("[+] N = %p\n", (void*)n_seq);
  if (o.flag_bits) printf("[+] Bit Range %i\n", o.bitrange);
  else printf("[+] Range \n");
  printf("[+] -- from : 0x%s\n", start.hex().c_str());
  printf("[+] -- to   : 0x%s\n", end.hex().c_str());
  // targets (keyhunt.cpp:6300-6358, 6559-6576)
  AddrTargets T;
  std::string err;
  if (!AddrTargets::load_file(file, o.bloom_multiplier, T, &err)) {
    fprintf(stderr, "[E] %s\n[E] Unenexpected error\n", err.c_str());
    return EXIT_FAILURE;
  }
  printf("[+] Allocating memory for %llu elements: %.2f MB\n", (unsigned long long)T.counted,
         (double)(20.0 * (double)T.counted / 1048576.0));
  printf("[+] Bloom filter for %llu elements.\n", (unsigned long long)T.counted);
  printf("[+] Loading data to the bloomfilter total: %.2f MB\n", (double)T.bloom.bytes / 1048576.0);
  for (const std::string& s : T.skipped) fprintf(stderr, "[I] Ommiting invalid line %s\n", s.c_str());
  printf("[+] Sorting data ...");
  printf(" done! %llu values were loaded and sorted\n", (unsigned long long)T.table.size());
  // generator + lane offsets for one chunk of n_seq keys
  AddrGen G;
  const uint32_t gpl = 16;
  G.build(stride, (uint32_t)(n_seq / 1024), gpl, o.threads > 0 ? o.threads : 1);
  AddrConfig cfg;
  cfg.search = o.search;
  cfg.endomorphism = o.endomorphism;
  cfg.start = start;
  cfg.end = end;
  cfg.n_seq = n_seq;
  cfg.random = o.random;
  cfg.devices = o.devices;
  cfg.lanes = o.lanes;
  cfg.gpl = gpl;
  cfg.max_chunks = o.max_chunks;
  std::mutex out_mu;
  std::atomic<bool> done{false};
  AddrStats stats;
  std::atomic<uint64_t> keys_done{0};
  AddrCallbacks cb;
  cb.on_found = [&](const AddrFound& f) { writekey(f, out_mu); };
  cb.on_warning = [&](const std::string& m) {
    std::lock_guard<std::mutex> lk(out_mu);
    fprintf(stderr, "%s\n", m.c_str());
  };
  cb.on_chunk = [&](const U256& base, int device) {
    if (o.quiet) return;
    std::lock_guard<std::mutex> lk(out_mu);
    printf("\rBase key: %s     \r", base.hex().c_str());
    fflush(stdout);
  };
  // stats line every -s seconds (keyhunt.cpp:2145-2252): keys = groups * 1024, x6 with -e (keyhunt.cpp:2175-2180:
  // every -l mode), else x2 for -l compress
  std::thread stat_th([&] {
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t sec = 0;
    while (!done.load()) {
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
      const uint64_t s = (uint64_t)std::chrono::duration_cast<std::chrono::seconds>(
                             std::chrono::steady_clock::now() - t0).count();
      if (s == sec) continue;
      sec = s;
      if (o.out_seconds && s % o.out_seconds == 0) {
        U256 total(keys_done.load());
        if (o.endomorphism) total = total * 6u;
        else if (o.search == 1) total = total * 2u;
        std::lock_guard<std::mutex> lk(out_mu);
        printf("\r%s\r", speed_line(total, s).c_str());
        fflush(stdout);
      }
    }
  });
  AddrCallbacks cb2 = cb;
  cb2.on_chunk = [&](const U256& base, int device) {
    cb.on_chunk(base, device);
    keys_done.fetch_add(n_seq);
  };
  const int rc = addr_search(T, G, cfg, cb2, &stats, &err);
  done.store(true);
  stat_th.join();
  if (rc) {
    fprintf(stderr, "[E] %s\n", err.c_str());
    return EXIT_FAILURE;
  }
  printf("\nEnd\n");
  return 0;
}

}  // namespace khb
