"""The committed scan vectors (tests/golden/scan_vectors.json, written by make_golden.py from the oracle's
restatement of keyhunt.cpp:3873-3947) checked against the PRODUCT path alone: the host engine's tables
and chunk centre (libkhhost) and the HIP scan / x dump (libkhbsgs).  No oracle call: the fixture is the
only reference, so these tests hold even if the live oracle and the product drifted together.

Each vector: -n 0x100000000 (M = 65536, 64 groups per chunk), k = 1, one target, one chunk base."""
from __future__ import annotations

import hashlib
import json
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "scan_vectors.json")) as f:
    VECTORS = json.load(f)
IDS = [v["key"] for v in VECTORS]


@pytest.fixture(scope="module")
def tables():
    from keyhuntm1cpu_amd import khhost
    t = khhost.Tables(VECTORS[0]["n"], 1, threads=8, gpl=4)
    yield t
    t.close()


def test_vector_geometry(tables):
    assert all(v["n"] == VECTORS[0]["n"] and v["k"] == 1 for v in VECTORS)
    assert tables.cycles == VECTORS[0]["groups"] == 64


@pytest.mark.parametrize("v", VECTORS, ids=IDS)
def test_host_chunk_centre(tables, v):
    """keyhunt.cpp:3853-3866: startP = T + (-(base + 1025 M)) G, from the host engine."""
    from keyhuntm1cpu_amd import khhost
    assert tables.chunk_centre(int(v["base"], 16), khhost.pubkey(int(v["key"], 16))).hex() == v["centre"]


@pytest.fixture(scope="module")
def eng(tables):
    from keyhuntm1cpu_amd.khbsgs import Engine
    e = Engine(0, lanes=16384)
    bf, nb, bits, h = tables.bloom_concat(1)
    e.load_bloom(bf, nb, bits, h)
    e.load_giant_table(tables.giant_table())
    offs, gpl = tables.lane_offsets()
    e.load_lane_offsets(offs, gpl)
    yield e
    e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("v", VECTORS, ids=IDS)
def test_gpu_scan_matches_golden(eng, v):
    """Every x of the chunk (sha256 of the 64 x 1024 x-coordinates, and the first two verbatim) and the
    ungated level-1 candidate set (the reference's exact bloom_check hits) equal the committed values."""
    centre = bytes.fromhex(v["centre"])
    xs = eng.dump_x(centre, 0, v["groups"])
    assert len(xs) == v["groups"] * 1024 * 32
    assert xs[:64].hex() == v["x_first"]
    assert hashlib.sha256(xs).hexdigest() == v["xdump_sha256"]
    cands, degen, st = eng.scan(centre, 0, v["groups"])
    assert not degen
    assert st.giant_steps == v["groups"] * 1024
    assert sorted(a for _, a in cands) == sorted(v["candidates"])
    assert all(job == 0 for job, _ in cands)


# ---- second / third check vectors (tests/golden/check_vectors.json, make_golden.py check_vectors) ----
with open(os.path.join(HERE, "golden", "check_vectors.json")) as f:
    CHECK = json.load(f)
CHECK_IDS = [f"{i}-{c['kind']}" for i, c in enumerate(CHECK["cases"])]


@pytest.fixture(scope="module")
def check_tables():
    from keyhuntm1cpu_amd import khhost
    t = khhost.Tables(CHECK["n"], 1, threads=8, gpl=4)
    yield t
    t.close()


def test_check_vectors_cover_every_path():
    kinds = [c["kind"] for c in CHECK["cases"] if c["found"]]
    assert kinds.count("planted") >= 8 and kinds.count("special") >= 4
    assert all(c["found"] is None for c in CHECK["cases"] if c["kind"] == "random")


@pytest.mark.parametrize("c", CHECK["cases"], ids=CHECK_IDS)
def test_host_secondcheck_matches_golden(check_tables, c):
    """The host engine's bsgs_secondcheck (Tables::secondcheck, the CPU pool's check) vs the fixture."""
    got = check_tables.secondcheck(int(c["base"], 16), c["a"], bytes.fromhex(c["target"]))
    assert (hex(got) if got is not None else None) == c["found"]


@pytest.mark.gpu
def test_gpu_check_matches_golden(check_tables):
    """khb_check with the product's tables (libkhhost) vs the fixture, every case in one launch."""
    from keyhuntm1cpu_amd.khbsgs import Engine
    cases = CHECK["cases"]
    with Engine(0, lanes=16384) as e:
        e.load_check_tables(**check_tables.check_tables())
        got = e.check([bytes.fromhex(c["target"]) for c in cases],
                      [(int(c["base"], 16), c["a"], i) for i, c in enumerate(cases)])
    assert [hex(g["key"]) if g["found"] else None for g in got] == [c["found"] for c in cases]
