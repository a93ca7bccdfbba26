// -S table files in the reference's on-disk format (keyhunt.cpp:1373-1613 read, 1881-2025 write),
// so tables built by keyhunt load here bit-exactly and the other way round:
//   keyhunt_bsgs_4_<m>.blm   L1: 256 x [struct bloom (80 B, x86-64) | bf bytes | sha256(bf) x 2]
//   keyhunt_bsgs_6_<m2>.blm  L2, same layout
//   keyhunt_bsgs_2_<m3>.tbl  bPtable: m3 x struct bsgs_xvalue (16 B) | sha256(table)
//   keyhunt_bsgs_7_<m3>.blm  L3, same layout as L1
// struct bloom (bloom/bloom.h:26-45) on x86-64: entries@0 bits@8 bytes@16 hashes@24 error@32
// (long double, 16 B) ready@48 major@49 minor@50 bpe@56 bf@64 (pointer, ignored), size 80.
#include <stdio.h>
#include <string.h>

#include "address_host.hpp"   // sha256
#include "bsgs_host.hpp"

namespace khb {

namespace {

constexpr size_t kBloomHdr = 80;
static_assert(sizeof(long double) == 16, "x86-64 long double layout expected");

void header_of(const BloomFilter& b, uint8_t h[kBloomHdr]) {
  memset(h, 0, kBloomHdr);
  memcpy(h + 0, &b.entries, 8);
  memcpy(h + 8, &b.bits, 8);
  memcpy(h + 16, &b.bytes, 8);
  h[24] = b.hashes;
  long double e = b.error;
  memcpy(h + 32, &e, 10);              // the 80-bit value; the 6 padding bytes stay zero
  h[48] = 1;                           // ready
  h[49] = 2;                           // BLOOM_VERSION_MAJOR (bloom.cpp:31)
  h[50] = 201;                         // BLOOM_VERSION_MINOR (bloom.cpp:32)
  memcpy(h + 56, &b.bpe, 8);
}

void bloom_of_header(BloomFilter& b, const uint8_t h[kBloomHdr]) {
  memcpy(&b.entries, h + 0, 8);
  memcpy(&b.bits, h + 8, 8);
  memcpy(&b.bytes, h + 16, 8);
  b.hashes = h[24];
  long double e = 0;
  memcpy(&e, h + 32, 10);
  b.error = e;
  b.ready = h[48] != 0;
  memcpy(&b.bpe, h + 56, 8);
}

bool read_blooms(const std::string& path, std::vector<BloomFilter>& v, bool skip_checksum, std::string& err,
                 const std::function<void(const std::string&)>& log) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  if (log) log("[+] Reading bloom filter from file " + path.substr(path.find_last_of('/') + 1) + " ");
  uint8_t hdr[kBloomHdr], ck[64], dg[32];
  for (int i = 0; i < 256; ++i) {
    if (fread(hdr, kBloomHdr, 1, f) != 1) { err = "[E] Error reading the file " + path; fclose(f); return false; }
    bloom_of_header(v[i], hdr);
    v[i].bf.assign(v[i].bytes, 0);
    if (v[i].bytes && fread(v[i].bf.data(), v[i].bytes, 1, f) != 1) {
      err = "[E] Error reading the file " + path;
      fclose(f);
      return false;
    }
    if (fread(ck, 64, 1, f) != 1) { err = "[E] Error reading the file " + path; fclose(f); return false; }
    if (!skip_checksum) {
      sha256(v[i].bf.data(), v[i].bytes, dg);
      if (memcmp(ck, dg, 32) || memcmp(ck + 32, dg, 32)) {
        err = "[E] Error checksum file mismatch! " + path;
        fclose(f);
        return false;
      }
    }
    if (i % 64 == 0 && log) log(".");
  }
  fclose(f);
  if (log) log(" Done!\n");
  return true;
}

bool write_blooms(const std::string& path, const std::vector<BloomFilter>& v, std::string& err,
                  const std::function<void(const std::string&)>& log) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) { err = "[E] Error can't create the file " + path; return false; }
  if (log) log("[+] Writing bloom filter to file " + path.substr(path.find_last_of('/') + 1) + " ");
  uint8_t hdr[kBloomHdr], dg[32];
  for (int i = 0; i < 256; ++i) {
    header_of(v[i], hdr);
    sha256(v[i].bf.data(), v[i].bytes, dg);
    if (fwrite(hdr, kBloomHdr, 1, f) != 1 || (v[i].bytes && fwrite(v[i].bf.data(), v[i].bytes, 1, f) != 1) ||
        fwrite(dg, 32, 1, f) != 1 || fwrite(dg, 32, 1, f) != 1) {
      err = "[E] Error writing the file " + path + " please delete it";
      fclose(f);
      return false;
    }
    if (i % 64 == 0 && log) log(".");
  }
  fclose(f);
  if (log) log(" Done!\n");
  return true;
}

std::string join(const std::string& dir, const std::string& name) {
  if (dir.empty() || dir == ".") return name;
  return dir.back() == '/' ? dir + name : dir + "/" + name;
}

}  // namespace

std::string Tables::file_name(const Geometry& g, uint32_t which) {
  char b[128];
  switch (which) {
    case kFileL1: snprintf(b, sizeof b, "keyhunt_bsgs_4_%llu.blm", (unsigned long long)g.m); break;
    case kFileL2: snprintf(b, sizeof b, "keyhunt_bsgs_6_%llu.blm", (unsigned long long)g.m2); break;
    case kFileBp: snprintf(b, sizeof b, "keyhunt_bsgs_2_%llu.tbl", (unsigned long long)g.m3); break;
    default: snprintf(b, sizeof b, "keyhunt_bsgs_7_%llu.blm", (unsigned long long)g.m3); break;
  }
  return b;
}

bool Tables::load_files(const std::string& dir, bool skip_checksum, uint32_t& have, std::string& err,
                        const std::function<void(const std::string&)>& log) {
  have = 0;
  err.clear();
  if (read_blooms(join(dir, file_name(geo, kFileL1)), l1, skip_checksum, err, log)) have |= kFileL1;
  if (!err.empty()) return false;
  if (read_blooms(join(dir, file_name(geo, kFileL2)), l2, skip_checksum, err, log)) have |= kFileL2;
  if (!err.empty()) return false;
  {
    const std::string path = join(dir, file_name(geo, kFileBp));
    FILE* f = fopen(path.c_str(), "rb");
    if (f) {
      if (log) log("[+] Reading bP Table from file " + file_name(geo, kFileBp) + " .");
      static_assert(sizeof(XValue) == 16, "struct bsgs_xvalue is 16 bytes");
      bp.assign(geo.m3, XValue());
      uint8_t ck[32], dg[32];
      const size_t bytes = sizeof(XValue) * geo.m3;
      if (fread(bp.data(), bytes, 1, f) != 1 || fread(ck, 32, 1, f) != 1) {
        err = "[E] Error reading the file " + path;
        fclose(f);
        return false;
      }
      fclose(f);
      if (!skip_checksum) {
        sha256((const uint8_t*)bp.data(), bytes, dg);
        if (memcmp(ck, dg, 32)) {
          err = "[E] Error checksum file mismatch! " + path;
          return false;
        }
      }
      if (log) log("... Done!\n");
      have |= kFileBp;
    }
  }
  if (read_blooms(join(dir, file_name(geo, kFileL3)), l3, skip_checksum, err, log)) have |= kFileL3;
  return err.empty();
}

bool Tables::save_files(const std::string& dir, uint32_t have, std::string& err,
                        const std::function<void(const std::string&)>& log) const {
  if (!(have & kFileL1) && !write_blooms(join(dir, file_name(geo, kFileL1)), l1, err, log)) return false;
  if (!(have & kFileL2) && !write_blooms(join(dir, file_name(geo, kFileL2)), l2, err, log)) return false;
  if (!(have & kFileBp)) {
    const std::string path = join(dir, file_name(geo, kFileBp));
    FILE* f = fopen(path.c_str(), "wb");
    if (!f) { err = "[E] Error can't create the file " + path; return false; }
    if (log) log("[+] Writing bP Table to file " + file_name(geo, kFileBp) + " .. ");
    const size_t bytes = sizeof(XValue) * bp.size();
    uint8_t dg[32];
    sha256((const uint8_t*)bp.data(), bytes, dg);
    if ((bytes && fwrite(bp.data(), bytes, 1, f) != 1) || fwrite(dg, 32, 1, f) != 1) {
      err = "[E] Error writing the file " + path;
      fclose(f);
      return false;
    }
    fclose(f);
    if (log) log("Done!\n");
  }
  if (!(have & kFileL3) && !write_blooms(join(dir, file_name(geo, kFileL3)), l3, err, log)) return false;
  return true;
}

}  // namespace khb
