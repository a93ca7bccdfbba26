"""Regenerate tests/golden/*.json (test infrastructure; run from the repo root in the build
container, where the reference checkout is mounted read-only at /root/reference).

  puzzle_targets.json  data copied from the reference's fixture files (tests/1to63_65.txt,
                       tests/63.pub, tests/125.txt, tests/130.txt, tests/66.rmd): pubkeys / hash160
  puzzle_keys.json     keys of puzzles 1..45 found by the oracle BSGS search; each is
                       self-certifying: pubkey(key) equals the reference file's line
  scan_vectors.json    oracle candidate sets + x-dump digests for fixed (geometry, base, target)
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


if __name__ == "__main__":
    main()
