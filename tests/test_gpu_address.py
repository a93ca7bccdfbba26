"""GPU parity for -m address / -m rmd160 (keyhunt.cpp:2586-2937): libkhbsgs through its C ABI and
the libkhhost search driver, against the oracle restatement.  Bit-exact: every hash160, every
group point (x||y), every bloom hit (t, kind), every recovered key."""
from __future__ import annotations

import json
import os
import random

import pytest

from keyhuntm1cpu_amd import khhost

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


def _text(name: str) -> str:
    with open(os.path.join(GOLD, "address", name)) as f:
        return f.read()


@pytest.fixture(scope="module")
def keys():
    with open(os.path.join(GOLD, "puzzle_keys.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def eng():
    from keyhuntm1cpu_amd.khbsgs import Engine
    e = Engine(0, lanes=16384)
    yield e
    e.close()


def _load(eng, A: khhost.Addr):
    bf, bits, h = A.bloom()
    eng.load_addr_bloom(bf, bits, h)
    eng.load_giant_table(A.giant_table())
    offs, gpl = A.lane_offsets()
    eng.load_lane_offsets(offs, gpl)


def test_hash160_kernel_matches_oracle(eng, ora):
    A = khhost.Addr(_text("1to32.rmd"), n_seq=1 << 16)
    _load(eng, A)
    rng = random.Random(11)
    ks = [1, 2, 3, N - 1] + [rng.randrange(1, N) for _ in range(3000)]
    pts = [ora.pubkey(k) for k in ks]
    xy = b"".join(p.be64() for p in pts)
    O = ora.AddrTable(_text("1to32.rmd"))
    for kind in (0, 1, 2):
        got = eng.hash160(kind, xy)
        for i, p in enumerate(pts):
            ref = ora.x_hash160(2 + kind, p.x.value()) if kind < 2 else ora.pub_hash160(p, False)
            assert got[i][0] == ref, (kind, i)
            assert got[i][1] == (1 if O.bloom_check(ref) else 0)
    # puzzle keys 1 and 3 are members (compressed, prefix of their own y parity)
    members = [(ora.pubkey(k), k) for k in (1, 3, 7)]
    for p, k in members:
        kind = 1 if p.y.value() & 1 else 0
        assert eng.hash160(kind, p.be64())[0][1] == 1


def _oracle_groups(ora, O, gen, base: int, ngroups: int, search: int):
    hits, keys = [], []
    for g in range(ngroups):
        h, k, _ = gen.group(O, base + 1024 * g, search)
        hits += [(g, t, kind) for t, kind in h]
        keys += k
    return sorted(hits), keys


@pytest.mark.parametrize("gpl", [1, 4])
def test_addr_dump_matches_oracle(eng, ora, gpl):
    A = khhost.Addr(_text("1to32.rmd"), n_seq=1 << 16, gpl=gpl)
    _load(eng, A)
    gen = ora.AddrGen(1)
    base = 0x123456789ABCDEF0123
    centre = khhost.pubkey(base + 512)
    xy = eng.addr_dump(centre, 0, 8)
    O = ora.AddrTable(_text("1to32.rmd"))
    for g in range(8):
        _, _, ref = gen.group(O, base + 1024 * g, 2, want_xy=True)
        assert xy[g * 65536:(g + 1) * 65536] == ref, g


@pytest.mark.parametrize("search", [0, 1, 2])
def test_addr_hits_match_oracle_dense_targets(eng, ora, search):
    """A target file holding the hash160s of 3000 keys of the scanned window (compressed for even
    keys, uncompressed for odd, plus negated keys) makes thousands of true bloom hits; the GPU's hit
    set must equal the oracle's for every (group, t, kind)."""
    rng = random.Random(search)
    base, ngroups = 0x4000000000 + 1, 48
    picks = rng.sample(range(base, base + 1024 * ngroups), 3000)
    lines = []
    for i, k in enumerate(picks):
        kk = N - k if i % 7 == 0 else k
        lines.append(ora.pub_hash160(ora.pubkey(kk), i % 2 == 0).hex())
    text = "\n".join(lines) + "\n"
    A = khhost.Addr(text, n_seq=1024 * ngroups, gpl=4)
    _load(eng, A)
    O = ora.AddrTable(text)
    gen = ora.AddrGen(1)
    ref_hits, ref_keys = _oracle_groups(ora, O, gen, base, ngroups, search)
    hits, st = eng.addr_scan(khhost.pubkey(base + 512), 0, ngroups, search)
    assert st.giant_steps == 1024 * ngroups
    assert sorted((g, t, kind) for _, g, t, kind in hits) == ref_hits
    assert len(ref_hits) > 1000
    # the host search confirms exactly the oracle's keys
    found, st2 = A.search(base, base + 1024 * ngroups, search=search, lanes=16384)
    assert sorted(k for k, _, _ in found) == sorted(ref_keys)


def test_addr_search_puzzles(keys):
    """Puzzles 1..24 from tests/1to32.txt (base58 addresses) in one sequential run of [1, 2^24)."""
    A = khhost.Addr(_text("1to32.txt"), n_seq=1 << 20)
    found, st = A.search(1, 1 << 24, search=2, lanes=65536)
    got = sorted(k for k, c, _ in found)
    assert got == sorted(int(keys[str(n)]["key"], 16) for n in range(1, 25))
    assert all(c for _, c, _ in found)
    assert st["chunks"] == 16 and st["keys"] == 1 << 24


def test_addr_search_uncompressed_and_negated():
    k = 0x5A5A5A123
    xy_k = khhost.pubkey(k)
    xy_nk = khhost.pubkey(N - k)
    text = "\n".join([khhost.hash160(xy_k, False).hex(),                       # uncompressed of k
                      khhost.rmd_to_address(khhost.hash160(xy_nk, True))]) + "\n"   # compressed of n-k
    A = khhost.Addr(text, n_seq=1 << 20)
    lo, hi = k - (k % (1 << 20)), k - (k % (1 << 20)) + (1 << 20)
    f2, _ = A.search(lo, hi, search=2, lanes=16384)
    assert sorted((kk, c) for kk, c, _ in f2) == sorted([(k, False), (N - k, True)])
    f1, _ = A.search(lo, hi, search=1, lanes=16384)
    assert [(kk, c) for kk, c, _ in f1] == [(N - k, True)]
    f0, _ = A.search(lo, hi, search=0, lanes=16384)
    assert [(kk, c) for kk, c, _ in f0] == [(k, False)]


def _cli(args, cwd):
    import subprocess
    from keyhuntm1cpu_amd import BIN_DIR
    exe = os.path.join(BIN_DIR, "keyhunt_amd")
    return subprocess.run([exe] + args, cwd=cwd, capture_output=True, text=True, timeout=300)


def test_cli_address_puzzle20(tmp_path, keys):
    """keyhunt_amd -m address -f tests/1to32.txt -b 20 -n 0x100000: the reference's hit lines and
    KEYFOUNDKEYFOUND.txt entry for puzzle #20, then End (the range is scanned to its end)."""
    r = _cli(["-m", "address", "-f", os.path.join(GOLD, "address", "1to32.txt"), "-b", "20", "-n", "0x100000",
              "-q", "-s", "0"], tmp_path)
    assert r.returncode == 0, r.stderr
    k = int(keys["20"]["key"], 16)
    assert f"Hit! Private Key: {k:x}\n" in r.stdout
    assert f"pubkey: {keys['20']['pubkey']}\n" in r.stdout
    assert "Address 1HsMJxNiV7TLxmoF6uJNkydxPFDog4NQum\n" in r.stdout
    assert r.stdout.rstrip().endswith("End")
    with open(tmp_path / "KEYFOUNDKEYFOUND.txt") as f:
        assert f"Private Key: {k:x}" in f.read()


def test_cli_rmd160_compress_range(tmp_path, keys):
    """-m rmd160 with the hash160 file, -l compress, -r window around puzzle #25."""
    k = int(keys["25"]["key"], 16)
    lo = k - (k % (1 << 20))
    r = _cli(["-m", "rmd160", "-f", os.path.join(GOLD, "address", "1to32.rmd"), "-r", f"{lo:x}:{lo + (1 << 21):x}",
              "-n", "0x100000", "-l", "compress", "-q", "-s", "0"], tmp_path)
    assert r.returncode == 0, r.stderr
    assert f"Hit! Private Key: {k:x}\n" in r.stdout
    assert "[+] Search compress only" in r.stdout


def test_cli_bloom_multiplier(tmp_path, keys, ora):
    """-z 4 with more than 10,000 targets (keyhunt.cpp:766-772, 6559-6576): the CLI prints the reference's
    "[+] Bloom Size Multiplier 4" line and a target bloom of the oracle's bloom_init2(4 x items) size, and
    still finds puzzle #20 planted among 12,000 synthetic hash160 lines."""
    import random
    rng = random.Random(9)
    lines = ["%040x" % rng.getrandbits(160) for _ in range(12000)]
    with open(os.path.join(GOLD, "address", "1to32.rmd")) as f:
        p20 = f.read().split("\n")[19].strip()
    lines.insert(6000, p20)
    text = "\n".join(lines) + "\n"
    (tmp_path / "t.rmd").write_text(text)
    O = ora.AddrTable(text, bloom_multiplier=4)
    mb = O.bloom().bytes / 1048576.0
    O.close()
    r = _cli(["-m", "rmd160", "-f", "t.rmd", "-b", "20", "-n", "0x100000", "-z", "4", "-q", "-s", "0"], tmp_path)
    assert r.returncode == 0, r.stderr
    assert "[+] Bloom Size Multiplier 4\n" in r.stdout
    assert "[+] Loading data to the bloomfilter total: %.2f MB\n" % mb in r.stdout
    k = int(keys["20"]["key"], 16)
    assert f"Hit! Private Key: {k:x}\n" in r.stdout


@pytest.mark.parametrize("search", [0, 1, 2])
def test_addr_unsolvedpuzzles_bloom_matches_oracle(eng, ora, search):
    """Config E's own target file (tests/unsolvedpuzzles.rmd, sized by keyhunt.cpp:6559-6576 with its
    10,000-entry minimum): the bloom hit set of 64 groups equals the oracle's, first with the file
    alone (three windows: the puzzle-71 range start, a random 2^70 key, a key near n), then with 200
    planted hash160s of keys in a window appended to the file (keyhunt.cpp:2713-2735 checks)."""
    text = _text("unsolvedpuzzles.rmd")
    O = ora.AddrTable(text)
    A = khhost.Addr(text, n_seq=1024 * 64, gpl=4)
    assert A.table() and len(A.table()) == O.n
    _load(eng, A)
    gen = ora.AddrGen(1)
    for base in (1 << 70, 0x3A5F0C2D9E8B7164F3 + search, N - 1024 * 64 - 7):
        ref_hits, _ = _oracle_groups(ora, O, gen, base, 64, search)
        hits, st = eng.addr_scan(khhost.pubkey(base + 512), 0, 64, search)
        assert st.giant_steps == 1024 * 64
        assert sorted((g, t, kind) for _, g, t, kind in hits) == ref_hits
    rng = random.Random(100 + search)
    base = (1 << 70) + 0x5151
    picks = rng.sample(range(base, base + 1024 * 64), 200)
    extra = [ora.pub_hash160(ora.pubkey(k), i % 2 == 0).hex() for i, k in enumerate(picks)]
    text2 = text.rstrip("\n") + "\n" + "\n".join(extra) + "\n"
    O2 = ora.AddrTable(text2)
    A2 = khhost.Addr(text2, n_seq=1024 * 64, gpl=4)
    _load(eng, A2)
    ref_hits, ref_keys = _oracle_groups(ora, O2, gen, base, 64, search)
    hits, _ = eng.addr_scan(khhost.pubkey(base + 512), 0, 64, search)
    assert sorted((g, t, kind) for _, g, t, kind in hits) == ref_hits
    assert len(ref_hits) >= 90
    found, _ = A2.search(base, base + 1024 * 64, search=search, lanes=16384)
    assert sorted(k for k, _, _ in found) == sorted(ref_keys)


def test_addr_search_ragged_queue():
    """The queued device loop (two launches in flight, 8 work items per lane, a short last batch):
    75 chunks of 2^18 keys at 256 lanes and 4 groups per lane = batches of 32, 32 and 11 chunks, with
    targets planted in the first, middle and last batches (first and last key of a chunk included);
    all are found and every key is counted exactly once."""
    n_seq = 1 << 18
    lo = 0x1234567 << 18
    picks = [lo, lo + 40 * n_seq + 777, lo + 74 * n_seq + n_seq - 1, lo + 31 * n_seq + n_seq - 1]
    text = "\n".join(khhost.hash160(khhost.pubkey(k), True).hex() for k in picks) + "\n"
    A = khhost.Addr(text, n_seq=n_seq, gpl=4)
    found, st = A.search(lo, lo + 75 * n_seq, search=1, lanes=256)
    assert sorted(k for k, _, _ in found) == sorted(picks)
    assert st["chunks"] == 75 and st["keys"] == 75 * n_seq
    assert st["launches"] == 3


def test_addr_search_falls_back_to_depth_one(keys):
    """the address loop reserves both submission slots; when the second does not fit (lanes
    sized so one slot's scratch takes 60 % of HBM) it warns and runs one launch at a time, and still
    finds puzzles 1..24 over two batches (4,098 chunks of 2^12 keys, 4,096 per batch)."""
    from tests.test_gpu_depth import _one_slot_lanes
    A = khhost.Addr(_text("1to32.txt"), n_seq=1 << 12, gpl=4)
    found, st = A.search(1, (1 << 24) + (1 << 13), search=2, lanes=_one_slot_lanes())
    got = sorted(k for k, c, _ in found)
    assert got == sorted(int(keys[str(n)]["key"], 16) for n in range(1, 25))
    assert st["chunks"] == 4098 and st["launches"] == 2


def test_addr_hit_overflow_rescans_and_finds_every_key(keys):
    """Every bloom hit must reach the host check (keyhunt.cpp:2716-2937 -> searchbinary).  With a
    16-entry hit ring the 16-chunk batch overflows (24 true hits), and so does chunk 0 on its own
    (puzzles 1..20); the address loop rescans in parts -- by chunks, then chunk 0's group ranges (its
    first 16-group work item holds puzzles 1..14) -- instead of failing, and still finds puzzles 1..24,
    each once, with the chunk and key counts of one pass."""
    A = khhost.Addr(_text("1to32.txt"), n_seq=1 << 20)
    A.set_hit_capacity(16)
    found, st = A.search(1, 1 << 24, search=2, lanes=65536)
    got = sorted(k for k, c, _ in found)
    assert got == sorted(int(keys[str(n)]["key"], 16) for n in range(1, 25))
    assert st["rescans"] > 0
    assert st["chunks"] == 16 and st["keys"] == 1 << 24


def test_addr_search_two_contexts_share_the_cursor(keys):
    """-m address with two device threads (-g 0,0: two contexts on one GPU) pulling chunks from one
    shared cursor (address_host.cpp device_loop, keyhunt.cpp:2586-2937 threads): puzzles 1..24 are each
    found exactly once and the 16 chunks of [1, 2^24) are each scanned once."""
    A = khhost.Addr(_text("1to32.txt"), n_seq=1 << 20)
    found, st = A.search(1, 1 << 24, search=2, devices=(0, 0), lanes=16384)
    got = sorted(k for k, c, _ in found)
    assert got == sorted(int(keys[str(n)]["key"], 16) for n in range(1, 25))
    assert st["chunks"] == 16 and st["keys"] == 1 << 24


def test_addr_random_chunk_mode_finds_the_key(keys):
    """-m address -R: chunks of n keys start at random keys of [start, end) (keyhunt.cpp:2586-2937 with
    FLAGRANDOM); a range two chunks wide around puzzle 24's key is covered by each chunk with
    probability ~1/2, so 40 random chunks find it."""
    A = khhost.Addr(_text("1to32.txt"), n_seq=1 << 16)
    key = int(keys["24"]["key"], 16)
    found, st = A.search(key - (1 << 16) + 1, key + (1 << 16), search=2, lanes=16384, max_chunks=40,
                         random_chunks=True)
    assert key in [k for k, c, _ in found]
    assert 1 <= st["chunks"] <= 40


@pytest.mark.parametrize("search", [0, 1, 2])
def test_addr_endomorphism_hits_match_oracle(eng, ora, search):
    """-e (KHB_SEARCH_ENDOMORPHISM; keyhunt.cpp:579-585, 2646-2763, 2789-2937): 48 groups with 1,500 planted targets
    +-lambda^e * k (e = 0, 1, 2; compressed or uncompressed).  The GPU's bloom-hit set (g, t, kind = form | e << 2)
    equals the oracle's in every -l mode, and the host search recovers exactly the oracle's keys, which are the
    planted keys of that mode."""
    from tests.helpers import endo_planted_text
    rng = random.Random(60 + search)
    base, ngroups = 0x4100000000 + 1, 48
    picks = rng.sample(range(base, base + 1024 * ngroups), 1500)
    text, planted = endo_planted_text(ora, picks, 70 + search)
    A = khhost.Addr(text, n_seq=1024 * ngroups, gpl=4)
    _load(eng, A)
    O = ora.AddrTable(text)
    gen = ora.AddrGen(1)
    ref_hits, ref_keys = _oracle_groups(ora, O, gen, base, ngroups, search | ora.SEARCH_ENDO)
    hits, st = eng.addr_scan(khhost.pubkey(base + 512), 0, ngroups, search | ora.SEARCH_ENDO)
    assert st.giant_steps == 1024 * ngroups
    assert sorted((g, t, kind) for _, g, t, kind in hits) == ref_hits
    assert {kind >> 2 for _, _, kind in ref_hits} == {0, 1, 2}
    want = [K for K, c, _ in planted if search == 2 or (search == 1) == c]
    assert sorted(ref_keys) == sorted(want)
    found, st2 = A.search(base, base + 1024 * ngroups, search=search | ora.SEARCH_ENDO, lanes=16384)
    assert sorted(k for k, _, _ in found) == sorted(ref_keys)
    # without -e the same file yields only the e = 0 keys (the plain kernels are unchanged)
    hits0, _ = eng.addr_scan(khhost.pubkey(base + 512), 0, ngroups, search)
    ref0, _ = _oracle_groups(ora, O, gen, base, ngroups, search)
    assert sorted((g, t, kind) for _, g, t, kind in hits0) == ref0


def test_cli_endomorphism_lambda_multiples(tmp_path, keys, ora):
    """keyhunt_amd -m address -e -l compress: a target file holding the compressed addresses of lambda * k20 and of
    n - lambda^2 * k21 (puzzles #20 and #21 of tests/1to32.txt, keyhunt.cpp:582-585) is solved over [1, 2^33),
    each key reported once with the reference's Hit lines, and the stats line counts x6 keys (keyhunt.cpp:2175-2180)."""
    import re
    k20, k21 = int(keys["20"]["key"], 16), int(keys["21"]["key"], 16)
    lam = ora.endo_constants(0)[0]
    lam2 = ora.endo_constants(1)[0]
    K1 = lam * k20 % N
    K2 = N - lam2 * k21 % N
    text = "\n".join(khhost.rmd_to_address(khhost.hash160(khhost.pubkey(K), True)) for K in (K1, K2)) + "\n"
    (tmp_path / "endo.txt").write_text(text)
    n_seq = 1 << 28
    r = _cli(["-m", "address", "-f", "endo.txt", "-e", "-l", "compress", "-r", "1:200000000", "-n", hex(n_seq),
              "-q", "-s", "1"], tmp_path)
    assert r.returncode == 0, r.stderr
    assert "[+] Endomorphism enabled\n" in r.stdout
    for K in (K1, K2):
        assert r.stdout.count(f"Hit! Private Key: {K:x}\n") == 1, K
    totals = [int(m) for m in re.findall(r"Total (\d+) keys in", r.stdout)]
    assert totals, r.stdout[-2000:]
    assert all(t % (6 * n_seq) == 0 and t // 6 <= (1 << 33) for t in totals)


@pytest.mark.parametrize("stride,endo", [(3, False), (0x100000001, True)])
def test_addr_stride_hits_match_oracle(eng, ora, stride, endo):
    """-I stride (keyhunt.cpp:790-797, init_generator 4386-4399: Gn[i] = (i+1)*stride*G), with and without -e: the GPU's
    bloom-hit set over 16 groups equals the oracle's group loop at the same stride, and the host confirmation of every
    hit (khh_addr_confirm: key = base + (1024 g + t) * stride, then lambda^e) recovers exactly the oracle's keys, which
    are the planted ones."""
    from tests.helpers import endo_planted_text
    rng = random.Random(stride)
    base, ngroups = 0x5000000000 + 7, 16
    picks = [base + stride * t for t in rng.sample(range(1024 * ngroups), 400)]
    if endo:
        text, planted = endo_planted_text(ora, picks, 90)
    else:
        text = "\n".join(ora.pub_hash160(ora.pubkey(k), i % 2 == 0).hex() for i, k in enumerate(picks)) + "\n"
        planted = [(k, i % 2 == 0, 0) for i, k in enumerate(picks)]
    search = 2 | (ora.SEARCH_ENDO if endo else 0)
    A = khhost.Addr(text, n_seq=1024 * ngroups, stride=stride, gpl=4)
    _load(eng, A)
    O = ora.AddrTable(text)
    gen = ora.AddrGen(stride)
    hits, keys = [], []
    for g in range(ngroups):
        h, k, _ = gen.group(O, base + 1024 * stride * g, search)
        hits += [(g, t, kind) for t, kind in h]
        keys += k
    got, st = eng.addr_scan(khhost.pubkey(base + 512 * stride), 0, ngroups, search)
    assert st.giant_steps == 1024 * ngroups
    assert sorted((g, t, kind) for _, g, t, kind in got) == sorted(hits)
    assert sorted(keys) == sorted(K for K, _, _ in planted)
    conf = [A.confirm(base + stride * (1024 * g + t), kind) for _, g, t, kind in got]
    assert sorted(r[0] for r in conf if r) == sorted(keys)


def test_cli_rmd160_endomorphism_uncompressed(tmp_path, keys, ora):
    """keyhunt_amd -m rmd160 -e -l uncompress: a hash160 file holding the uncompressed hash160s of lambda^2 * k20 and of
    n - lambda * k21 (the negated point (beta*x, p - y), kind 3 | 1 << 2) is solved over [1, 2^33): each key is reported
    once with its uncompressed pubkey (keyhunt.cpp:2800-2920 -e uncompressed paths), and the totals count x6 keys."""
    import re
    k20, k21 = int(keys["20"]["key"], 16), int(keys["21"]["key"], 16)
    lam, lam2 = ora.endo_constants(0)[0], ora.endo_constants(1)[0]
    K1 = lam2 * k20 % N
    K2 = N - lam * k21 % N
    text = "\n".join(khhost.hash160(khhost.pubkey(K), False).hex() for K in (K1, K2)) + "\n"
    (tmp_path / "endo.rmd").write_text(text)
    n_seq = 1 << 28
    r = _cli(["-m", "rmd160", "-f", "endo.rmd", "-e", "-l", "uncompress", "-r", "1:200000000", "-n", hex(n_seq),
              "-q", "-s", "1"], tmp_path)
    assert r.returncode == 0, r.stderr
    assert "[+] Endomorphism enabled\n" in r.stdout
    for K in (K1, K2):
        assert r.stdout.count(f"Hit! Private Key: {K:x}\n") == 1, K
        xy = khhost.pubkey(K)
        assert f"pubkey: 04{xy.hex()}\n" in r.stdout, K
    totals = [int(m) for m in re.findall(r"Total (\d+) keys in", r.stdout)]
    assert totals and all(t % (6 * n_seq) == 0 for t in totals)
