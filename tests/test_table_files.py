"""-S table files (keyhunt.cpp:1373-1613 read, 1881-2025 write): the reference's on-disk format.
Round trips through the product host engine, partial rebuilds, checksum checks, and a file packed
independently from the documented layout (struct bloom of bloom/bloom.h:26-45 on x86-64, with
garbage in the pointer and padding fields the reference also writes)."""
from __future__ import annotations

import hashlib
import os
import struct

import numpy as np
import pytest

from keyhuntm1cpu_amd import khhost

N_STR = "0x10000000"    # M = 16384, M2 = 512, M3 = 16


@pytest.fixture(scope="module")
def built():
    t = khhost.Tables(N_STR, 1, threads=4)
    yield t
    t.close()


def _names(t):
    return {1: f"keyhunt_bsgs_4_{t.m}.blm", 2: f"keyhunt_bsgs_6_{t.m2}.blm", 4: f"keyhunt_bsgs_2_{t.m3}.tbl",
            8: f"keyhunt_bsgs_7_{t.m3}.blm"}


def _same(a, b):
    for lvl in (1, 2, 3):
        assert a.bloom_concat(lvl) == b.bloom_concat(lvl), lvl
    assert a.bptable() == b.bptable()


def test_round_trip(built, tmp_path):
    built.save_files(str(tmp_path))
    names = _names(built)
    assert sorted(os.listdir(tmp_path)) == sorted(names.values())
    bf, nb, bits, h = built.bloom_concat(1)
    assert os.path.getsize(tmp_path / names[1]) == 256 * (80 + nb + 64)
    assert os.path.getsize(tmp_path / names[4]) == 16 * built.m3 + 32
    t2 = khhost.Tables(N_STR, 1, threads=4, files_dir=str(tmp_path))
    assert t2.have == 15
    _same(built, t2)
    t2.close()


def test_partial_rebuild_writes_missing_file_identically(built, tmp_path):
    built.save_files(str(tmp_path))
    names = _names(built)
    ref_l2 = (tmp_path / names[2]).read_bytes()
    os.remove(tmp_path / names[2])
    t3 = khhost.Tables(N_STR, 1, threads=4, files_dir=str(tmp_path), save=True)
    assert t3.have == 1 | 4 | 8
    _same(built, t3)
    assert (tmp_path / names[2]).read_bytes() == ref_l2
    t3.close()
    # with only L1 present, L2/L3/bPtable come from the m2-point rebuild
    for w in (2, 4, 8):
        os.remove(tmp_path / names[w])
    t4 = khhost.Tables(N_STR, 1, threads=4, files_dir=str(tmp_path))
    assert t4.have == 1
    _same(built, t4)
    t4.close()


def test_checksum_mismatch_is_an_error(built, tmp_path):
    built.save_files(str(tmp_path))
    p = tmp_path / _names(built)[8]
    raw = bytearray(p.read_bytes())
    raw[80 + 5] ^= 1                     # first sub-bloom's bf
    p.write_bytes(bytes(raw))
    with pytest.raises(khhost.KhhError, match="checksum"):
        khhost.Tables(N_STR, 1, threads=4, files_dir=str(tmp_path))
    t = khhost.Tables(N_STR, 1, threads=4, files_dir=str(tmp_path), skip_checksum=True)   # -6
    assert t.have == 15
    t.close()


def test_independently_packed_reference_layout(built, tmp_path):
    """Pack keyhunt_bsgs_4_<m>.blm from the documented layout with arbitrary pointer/padding bytes."""
    bf, nb, bits, h = built.bloom_concat(1)
    err = np.array([0.000001], dtype=np.longdouble).tobytes()
    assert len(err) == 16
    entries = 10000                         # items_for(m = 16384): 64 per sub-bloom, clamped to 10000
    bpe = -np.log(1e-6) / 0.480453013918201
    out = bytearray()
    for i in range(256):
        sub = bf[i * nb:(i + 1) * nb]
        hdr = struct.pack("<QQQB7s", entries, bits, nb, h, b"\xaa" * 7) + err[:10] + b"\x55" * 6
        hdr += struct.pack("<BBB5sdQ8s", 1, 2, 201, b"\x77" * 5, float(bpe), 0x00007F1234567890, b"\x33" * 8)
        assert len(hdr) == 80
        dg = hashlib.sha256(sub).digest()
        out += hdr + sub + dg + dg
    d = tmp_path / "ref"
    d.mkdir()
    (d / _names(built)[1]).write_bytes(bytes(out))
    t = khhost.Tables(N_STR, 1, threads=4, files_dir=str(d))
    assert t.have == 1
    _same(built, t)
    t.close()
