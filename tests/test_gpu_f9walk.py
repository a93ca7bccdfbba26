"""GPU parity of the alternative 9 x 29-bit walk (libkhbsgs_f9.so, KHB_F9WALK=1, device/fe29.hpp):
every x of whole groups (its own dump mode, kDumpG, through the same arithmetic as its gated scan)
equals the oracle's group loop, and its gated candidates on three full default-geometry chunks equal the
product library's (8 x 32 walk).  The product ships the 8 x 32 walk; this keeps the
measured alternative correct when it is built (`make variants`)."""
from __future__ import annotations

import os

import pytest

from keyhuntm1cpu_amd import LIB_DIR, khhost

F9_LIB = os.path.join(LIB_DIR, "libkhbsgs_f9.so")
pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not os.path.exists(F9_LIB), reason="libkhbsgs_f9.so is built by `make variants`")]


@pytest.fixture(scope="module")
def tables_k1():
    t = khhost.Tables(None, 1, threads=16)
    yield t
    t.close()


def _engine(path, t, gate=True):
    from keyhuntm1cpu_amd.khbsgs import Engine
    e = Engine(0, lib_path=path)
    bf, nb, bits, h = t.bloom_concat(1)
    e.load_bloom(bf, nb, bits, h)
    e.load_giant_table(t.giant_table())
    offs, gpl = t.lane_offsets()
    e.load_lane_offsets(offs, gpl)
    if gate:
        g, lg = t.gate()
        e.load_gate(g, lg, t.gate_probes())
    return e


def test_f9_dump_matches_oracle(ora):
    t = khhost.Tables("0x100000000", 1, threads=8)
    o = ora.Bsgs("0x100000000", 1, 8)
    e = _engine(F9_LIB, t, gate=False)
    try:
        for key, base in ((0x2000000000123457, 0x2000000000000000), (0x7FFFFFFFFFFFF123, 0x7FFFFFFE00000000)):
            tgt = ora.pubkey(key)
            centre = t.chunk_centre(base, tgt.be64())
            xs = e.dump_x(centre, 0, 16)
            start = o.chunk_start(base, tgt)
            _, ref, _ = o.scan(start, 0, 16, want_x=True)
            assert xs == ref
    finally:
        e.close()


def test_f9_gated_candidates_equal_product(tables_k1):
    key = 0x2832ED74F2B5E35EE
    tgt = khhost.pubkey(key)
    bases = [key - 123456789012, (1 << 65) + (5 << 45), (1 << 129) + (7 << 45)]
    centres = b"".join(tables_k1.chunk_centre(b, tgt) for b in bases)
    got = {}
    for name in ("product", "f9"):
        e = _engine(None if name == "product" else F9_LIB, tables_k1)
        try:
            got[name], degen, st = e.scan(centres, 0, tables_k1.cycles)
            assert not degen and st.giant_steps == 3 * tables_k1.cycles * 1024
        finally:
            e.close()
    assert sorted(got["f9"]) == sorted(got["product"])
    assert any(tables_k1.secondcheck(bases[0], a, tgt) == key for j, a in got["f9"] if j == 0)
