"""Regenerate tests/golden/bloom_bits.json (test infrastructure).

The level-1 probe of keyhunt's BSGS hot loop is bloom_check(&bloom_bP[x[0]], x, 32)
(keyhunt.cpp:3948; bloom/bloom.cpp:128-156): a = XXH64(x, 32, 0x59f2815b16f81798),
b = XXH64(x, 32, a), bit i = (a + b*i) mod bits for i < hashes.  32-byte inputs take XXH64's
4-lane stripe loop and its mergeRounds (xxhash/xxhash.h:2469-2527), which the published
vectors of tests/test_oracle_pins.py (len < 32) do not reach.

This script computes the fixture with the Python `xxhash` package (libxxhash 0.8.2, an
implementation independent of this repository and of oracle/), never with the oracle, so the
oracle and the GPU are both checked against it:
  - x: 384 seeded 32-byte values (big-endian field-element bytes, as the device sees x), plus
    edge patterns (all-zero, all-0xff, one-hot words);
  - a, b per x;
  - the 20 bit positions for the k=1 (471,124 bits) and k=4 (1,884,499 bits) level-1 geometries
    (bloom_init2 of 16,384 / 65,536 entries at 1e-6).
Run from the repo root:  python tests/golden/make_bloom_bits.py
"""
import json
import os
import random

import xxhash

SEED = 0x59F2815B16F81798
GEOMETRIES = {"k1": (471124, 20), "k4": (1884499, 20)}
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bloom_bits.json")
M64 = (1 << 64) - 1


def bits_of(x: bytes, nbits: int, hashes: int) -> tuple[int, int, list[int]]:
    a = xxhash.xxh64_intdigest(x, seed=SEED)
    b = xxhash.xxh64_intdigest(x, seed=a)
    return a, b, [((a + b * i) & M64) % nbits for i in range(hashes)]


def inputs() -> list[bytes]:
    rng = random.Random(0x6B687536)
    xs = [bytes(32), b"\xff" * 32]
    for w in range(8):
        xs.append(bytes(4 * w) + b"\x00\x00\x00\x01" + bytes(28 - 4 * w))
        xs.append(bytes(4 * w) + b"\xff\xff\xff\xff" + bytes(28 - 4 * w))
    while len(xs) < 384:
        xs.append(rng.randbytes(32))
    return xs


def main():
    recs = []
    for x in inputs():
        r = {"x": x.hex()}
        for name, (nbits, hashes) in GEOMETRIES.items():
            a, b, bits = bits_of(x, nbits, hashes)
            r["a"], r["b"] = f"{a:016x}", f"{b:016x}"
            r[name] = bits
        recs.append(r)
    doc = {"generator": "tests/golden/make_bloom_bits.py", "xxhash": xxhash.XXHASH_VERSION,
           "seed": f"{SEED:016x}", "geometries": {k: {"bits": v[0], "hashes": v[1]} for k, v in GEOMETRIES.items()},
           "records": recs}
    with open(OUT, "w") as f:
        json.dump(doc, f, separators=(",", ":"))
        f.write("\n")
    print(f"wrote {OUT}: {len(recs)} records")


if __name__ == "__main__":
    main()
