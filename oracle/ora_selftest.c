/* ORACLE — TEST INFRASTRUCTURE ONLY.  Known-answer self test of the restatement. */
#include "ora.h"
#include <stdio.h>
#include <string.h>
#include <stdlib.h>

static int fails = 0;
#define EXPECT(c, ...) do { if (!(c)) { printf("FAIL: " __VA_ARGS__); printf("\n"); fails++; } } while (0)

int main(int argc, char** argv) {
  /* published XXH64 vectors */
  EXPECT(ora_xxh64("", 0, 0) == 0xEF46DB3751D8E999ULL, "xxh64 empty");
  EXPECT(ora_xxh64("abc", 3, 0) == 0x44BC2CF5AD770999ULL, "xxh64 abc = %016llx", (unsigned long long)ora_xxh64("abc", 3, 0));
  /* G and 3G (tests/1to63_65.txt lines 1-2) */
  char hex[140];
  ora_h_pubkey("1", hex, 1);
  EXPECT(!strcmp(hex, "0279be667ef9dcbbac55a06295ce870b07029bfcdb2dce28d959f2815b16f81798"), "G %s", hex);
  ora_h_pubkey("3", hex, 1);
  EXPECT(!strcmp(hex, "02f9308a019258c31049344f85f89d5229b531c845836f99b08601f113bce036f9"), "3G %s", hex);
  /* bloom sizing (16384 entries -> 471124 bits, 20 hashes) */
  ora_bloom b;
  ora_bloom_init2(&b, 16384, 0.000001);
  EXPECT(b.bits == 471124 && b.hashes == 20 && b.bytes == 58891, "bloom16384 bits=%llu hashes=%d bytes=%llu",
         (unsigned long long)b.bits, b.hashes, (unsigned long long)b.bytes);
  ora_bloom_free(&b);
  /* puzzle 30 smoke: -b 30 -n 0x100000 -> 3d94cd64 */
  char err[256] = "";
  ora_bsgs* c = ora_bsgs_new("0x100000", 1, 4, err, sizeof err);
  EXPECT(c != NULL, "bsgs_new %s", err);
  if (c) {
    ora_point t; int comp;
    int ok = ora_parse_pubkey_hex("030d282cf2ff536d2c42f105d0b8588821a915dc3f9a05bd98bb23af67a2e92a5b", &t, &comp);
    EXPECT(ok, "parse p30");
    ora_u256 s, e, key; int found = 0;
    ora_u256_from_hex(&s, "20000000");
    ora_u256_from_hex(&e, "40000000");
    uint64_t ch = ora_bsgs_search(c, &t, 1, &s, &e, 0, &found, &key);
    ora_u256_to_hex(&key, hex);
    printf("p30: chunks=%llu found=%d key=%s\n", (unsigned long long)ch, found, found ? hex : "-");
    EXPECT(found && !strcmp(hex, "3d94cd64"), "puzzle 30");
    ora_bsgs_free(c);
  }
  if (argc > 1 && !strcmp(argv[1], "p63")) {
    /* BSGSD.md:35-36,80: puzzle 63 in a 2^44-wide window around the key -> 7cce5efdaccf6808 */
    c = ora_bsgs_new(NULL, 1, 8, err, sizeof err);
    EXPECT(c != NULL, "bsgs_new %s", err);
    ora_point t; int comp;
    ora_parse_pubkey_hex("0365ec2994b8cc0a20d40dd69edfe55ca32a54bcbbaa6b0ddcff36049301a54579", &t, &comp);
    ora_u256 s, e, key; int found = 0;
    ora_u256_from_hex(&s, "7cce500000000000");
    ora_u256_from_hex(&e, "7cce600000000000");
    uint64_t ch = ora_bsgs_search(c, &t, 1, &s, &e, 0, &found, &key);
    ora_u256_to_hex(&key, hex);
    printf("p63: chunks=%llu found=%d key=%s\n", (unsigned long long)ch, found, found ? hex : "-");
    EXPECT(found && !strcmp(hex, "7cce5efdaccf6808"), "puzzle 63");
    ora_bsgs_free(c);
  }
  printf(fails ? "SELFTEST FAILED (%d)\n" : "SELFTEST OK\n", fails);
  return fails ? 1 : 0;
}
