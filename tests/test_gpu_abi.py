"""GPU: the stats arrays of the host ABI.  khh_session_run / khh_addr_search write exactly the
6 entries of their original contract; the _ex entry points write min(stats_len, KHH_*_STATS) entries and
nothing past them."""
from __future__ import annotations

import ctypes as C

import pytest

from keyhuntm1cpu_amd import khhost

pytestmark = pytest.mark.gpu

CANARY = 0xC0FFEE0DDBA11


def _buf(n=16):
    b = (C.c_uint64 * n)()
    for i in range(n):
        b[i] = CANARY
    return b


def _written(b):
    return [i for i in range(len(b)) if b[i] != CANARY]


@pytest.fixture(scope="module")
def sess():
    t = khhost.Tables("0x100000000", 1, threads=8)
    s = khhost.Session(t, devices=[0])
    yield t, s
    s.close()
    t.close()


def _run(sess, fn, *extra):
    t, s = sess
    L = khhost.lib()
    tgt = khhost.pubkey(0x1234567890ABCDEF)
    start = 1 << 50
    found = (C.c_int * 1)()
    keys = C.create_string_buffer(32)
    err = C.create_string_buffer(256)
    b = _buf()
    args = [s.h, tgt, 1, start.to_bytes(32, "big"), (start + 4 * 2 * t.n_low).to_bytes(32, "big"), 4, 0, found,
            keys, b, *extra, err, 256]
    assert getattr(L, fn)(*args) == 0, err.value
    return b


def test_session_run_writes_six(sess):
    b = _run(sess, "khh_session_run")
    assert len(_written(b)) <= 6 and all(b[i] == CANARY for i in range(6, 16))
    assert b[0] == 4                                     # chunks


@pytest.mark.parametrize("n", [0, 3, 7, 9, 11, 14])
def test_session_run_ex_honours_stats_len(sess, n):
    b = _run(sess, "khh_session_run_ex", n)
    assert all(b[i] == CANARY for i in range(min(n, khhost.KHH_SESSION_STATS), 16))
    if n:
        assert b[0] == 4


def test_addr_search_stats_len():
    with open(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "address",
                                         "1to32.rmd")) as f:
        A = khhost.Addr(f.read(), n_seq=1 << 16)
    L = khhost.lib()
    keys = C.create_string_buffer(32 * 64)
    comp = C.create_string_buffer(64)
    rmd = C.create_string_buffer(20 * 64)
    nf = C.c_uint32(0)
    devs = (C.c_int * 1)(0)
    err = C.create_string_buffer(256)
    start, end = 1 << 20, (1 << 20) + 4 * (1 << 16)
    for fn, extra, limit in (("khh_addr_search", (), 6), ("khh_addr_search_ex", (5,), 5),
                             ("khh_addr_search_ex", (8,), 8), ("khh_addr_search_ex", (11,), 8)):
        b = _buf()
        rc = getattr(L, fn)(A.h, start.to_bytes(32, "big"), end.to_bytes(32, "big"), 2, 0, devs, 1, 0, 0, keys, comp,
                            rmd, 64, C.byref(nf), b, *extra, err, 256)
        assert rc == 0, err.value
        assert all(b[i] == CANARY for i in range(limit, 16)), (fn, extra)
        assert b[1] == 4 * (1 << 16)                     # keys
    A.close()
