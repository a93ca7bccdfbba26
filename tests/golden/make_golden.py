"""Regenerate tests/golden/*.json (test infrastructure; run from the repo root in the build
container, where the reference checkout is mounted read-only at /root/reference).

  puzzle_targets.json  data copied from the reference's fixture files (tests/1to63_65.txt,
                       tests/63.pub, tests/125.txt, tests/130.txt, tests/66.rmd): pubkeys / hash160
  puzzle_keys.json     keys of puzzles 1..45 found by the oracle BSGS search; each is
                       self-certifying: pubkey(key) equals the reference file's line
  scan_vectors.json    oracle candidate sets + x-dump digests for fixed (geometry, base, target)
  check_vectors.json   oracle bsgs_secondcheck results (keyhunt.cpp:4271-4368) for fixed candidates:
                       planted keys, the third check's AddDirect(P, -P) case, random candidates
                       (`python tests/golden/make_golden.py check` rewrites only this file)
"""
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from oracle import ora  # noqa: E402

REF = "/root/reference/tests"
OUT = os.path.dirname(os.path.abspath(__file__))


def read_lines(name):
    with open(os.path.join(REF, name)) as f:
        return [ln.strip() for ln in f if ln.strip()]


def main():
    targets = {
        "1to63_65": read_lines("1to63_65.txt"),
        "63.pub": read_lines("63.pub"),
        "125.txt": read_lines("125.txt"),
        "130.txt": read_lines("130.txt"),
        "66.rmd": read_lines("66.rmd"),
    }
    with open(os.path.join(OUT, "puzzle_targets.json"), "w") as f:
        json.dump(targets, f, indent=1)
    lines = targets["1to63_65"]
    keys = {}
    cache = {}
    # n <= 21: walk k*G over [1, 2^21) (BSGS cannot see a key equal to the chunk base: bsgs_secondcheck's
    # AddDirect(T, -base*G) hits dx == 0; e.g. puzzle 1 with -r 1:...)
    want = {ora.parse_pubkey(lines[n - 1])[0].x.value(): n for n in range(1, 22)}
    g = ora.pubkey(1)
    p = g
    for k in range(1, 1 << 21):
        n = want.get(p.x.value())
        if n is not None and ora.pubkey_hex(k, True) == lines[n - 1]:
            keys[str(n)] = {"key": hex(k)[2:], "pubkey": lines[n - 1], "method": "walk"}
        p = ora.add_direct(p, g) if k > 1 else ora.pubkey(2)
    for n in range(22, 46):
        pub = lines[n - 1]
        t, _ = ora.parse_pubkey(pub)
        nexp = 2 * ((n - 1) // 2)
        lo, hi = 1 << (n - 1), 1 << n
        if nexp not in cache:
            cache[nexp] = ora.Bsgs(hex(1 << nexp), 1)
        _, found = cache[nexp].search([t], lo, hi)
        k = found[0]
        assert k is not None, n
        assert ora.pubkey_hex(k, True) == pub
        keys[str(n)] = {"key": hex(k)[2:], "pubkey": pub, "method": "bsgs -n " + hex(1 << nexp)}
        print(n, hex(k), flush=True)
    assert len(keys) == 45, sorted(keys)
    with open(os.path.join(OUT, "puzzle_keys.json"), "w") as f:
        json.dump(keys, f, indent=1)
    # scan vectors
    bs = ora.Bsgs("0x100000000", 1)
    vec = []
    for key, base in [(0x2000000000123457, 0x2000000000000000), (0x1234567890ABCDEF, 0x1234560000000000),
                      (0x55AA55AA55AA, 0x550000000000)]:
        t = ora.pubkey(key)
        st = bs.chunk_start(base, t)
        cands, xs, _ = bs.scan(st, 0, bs.cycles, want_x=True)
        vec.append({"n": "0x100000000", "k": 1, "key": hex(key), "base": hex(base), "centre": st.be64().hex(),
                    "candidates": cands, "xdump_sha256": hashlib.sha256(xs).hexdigest(),
                    "x_first": xs[:64].hex(), "groups": bs.cycles})
    with open(os.path.join(OUT, "scan_vectors.json"), "w") as f:
        json.dump(vec, f, indent=1)


def splitmix(seed):
    s = seed
    while True:
        s = (s + 0x9E3779B97F4A7C15) & (2**64 - 1)
        z = s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        yield z ^ (z >> 31)


def check_vectors():
    n = "0x1000000000"
    bs = ora.Bsgs(n, 1)
    m, m2, m3 = bs.m, bs.m2, bs.m3
    r = splitmix(0x676f6c64656e)
    cases = []
    for _ in range(12):
        base = next(r) | ((next(r) & 0xFFFF) << 64)
        a = next(r) % 4096
        cases.append(("planted", base, a, base + a * 2 * m + next(r) % (2 * m + 64)))
    for _ in range(6):
        base, a, i2, i = next(r), next(r) % 4096, next(r) % 32, next(r) % 32
        cases.append(("special", base, a, base + a * 2 * m + i2 * 2 * m2 + i * 2 * m3 + m3))
    for _ in range(6):
        cases.append(("random", next(r) | (next(r) << 64), next(r) & 0xFFFFFFFF,
                      next(r) | (next(r) << 64) | (next(r) << 128)))
    vec = []
    for kind, base, a, key in cases:
        t = ora.pubkey(key)
        found = bs.secondcheck(base, a, t)
        vec.append({"kind": kind, "base": hex(base), "a": a, "target": t.be64().hex(),
                    "found": hex(found) if found is not None else None})
    with open(os.path.join(OUT, "check_vectors.json"), "w") as f:
        json.dump({"n": n, "k": 1, "cases": vec}, f, indent=1)


if __name__ == "__main__":
    if sys.argv[1:] == ["check"]:
        check_vectors()
    else:
        main()
        check_vectors()
