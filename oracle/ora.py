"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/build/liboracle.so (the plain-C restatement of the reference BSGS path,
see ora.h).  Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg —
never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")


class U256(C.Structure):
    _fields_ = [("w", C.c_uint64 * 4)]

    @classmethod
    def of(cls, v: int) -> "U256":
        u = cls()
        for i in range(4):
            u.w[i] = (v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF
        return u

    def value(self) -> int:
        return sum(int(self.w[i]) << (64 * i) for i in range(4))


class Point(C.Structure):
    _fields_ = [("x", U256), ("y", U256), ("z", U256)]

    def xy(self) -> tuple[int, int]:
        return self.x.value(), self.y.value()

    def be64(self) -> bytes:
        return self.x.value().to_bytes(32, "big") + self.y.value().to_bytes(32, "big")

    @classmethod
    def of(cls, x: int, y: int) -> "Point":
        p = cls()
        p.x = U256.of(x)
        p.y = U256.of(y)
        p.z = U256.of(1)
        return p


class Bloom(C.Structure):
    _fields_ = [("entries", C.c_uint64), ("bits", C.c_uint64), ("bytes", C.c_uint64), ("hashes", C.c_uint8),
                ("error", C.c_longdouble), ("ready", C.c_uint8), ("major", C.c_uint8), ("minor", C.c_uint8),
                ("bpe", C.c_double), ("bf", C.POINTER(C.c_uint8))]


class XValue(C.Structure):
    _fields_ = [("value", C.c_uint8 * 6), ("pad", C.c_uint8 * 2), ("index", C.c_uint64)]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        L.ora_xxh64.restype = C.c_uint64
        L.ora_xxh64.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
        L.ora_bsgs_new.restype = C.c_void_p
        L.ora_bsgs_new.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_char_p, C.c_size_t]
        L.ora_bsgs_free.argtypes = [C.c_void_p]
        L.ora_bsgs_params.argtypes = [C.c_void_p, P(C.c_uint64)]
        L.ora_bsgs_bloom.restype = P(Bloom)
        L.ora_bsgs_bloom.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.ora_bsgs_bptable.restype = P(XValue)
        L.ora_bsgs_bptable.argtypes = [C.c_void_p]
        L.ora_bsgs_giant_table.argtypes = [C.c_void_p, C.c_char_p]
        L.ora_bsgs_amp_table.argtypes = [C.c_void_p, C.c_int, C.c_char_p]
        L.ora_bsgs_chunk_start.argtypes = [C.c_void_p, P(U256), P(Point), P(Point)]
        L.ora_bsgs_scan.argtypes = [C.c_void_p, P(Point), C.c_uint32, C.c_uint32, C.c_void_p, P(C.c_uint64),
                                    C.c_uint32, P(C.c_uint32), P(Point)]
        L.ora_bsgs_secondcheck.restype = C.c_int
        L.ora_bsgs_secondcheck.argtypes = [C.c_void_p, P(U256), C.c_uint32, P(Point), P(U256)]
        L.ora_bsgs_search.restype = C.c_uint64
        L.ora_bsgs_search.argtypes = [C.c_void_p, P(Point), C.c_int, P(U256), P(U256), C.c_uint64, P(C.c_int),
                                      P(U256)]
        L.ora_bsgs_bench.restype = C.c_uint64
        L.ora_bsgs_bench.argtypes = [C.c_void_p, P(Point), P(U256), C.c_int, C.c_double, P(C.c_double)]
        L.ora_compute_pubkey.argtypes = [P(Point), P(U256)]
        L.ora_add_direct.argtypes = [P(Point), P(Point), P(Point)]
        L.ora_negation.argtypes = [P(Point), P(Point)]
        L.ora_parse_pubkey_hex.restype = C.c_int
        L.ora_parse_pubkey_hex.argtypes = [C.c_char_p, P(Point), P(C.c_int)]
        L.ora_pubkey_hex.argtypes = [P(Point), C.c_int, C.c_char_p]
        L.ora_bloom_init2.restype = C.c_int
        L.ora_bloom_init2.argtypes = [P(Bloom), C.c_uint64, C.c_longdouble]
        L.ora_bloom_free.argtypes = [P(Bloom)]
        L.ora_bloom_add.restype = C.c_int
        L.ora_bloom_add.argtypes = [P(Bloom), C.c_void_p, C.c_int]
        L.ora_bloom_check.restype = C.c_int
        L.ora_bloom_check.argtypes = [P(Bloom), C.c_void_p, C.c_int]
        L.ora_sha256.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p]
        L.ora_ripemd160.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p]
        L.ora_hash160.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p]
        L.ora_pub_hash160.argtypes = [P(Point), C.c_int, C.c_char_p]
        L.ora_x_hash160.argtypes = [C.c_uint8, P(U256), C.c_char_p]
        L.ora_b58decode.restype = C.c_int
        L.ora_b58decode.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t, P(C.c_size_t)]
        L.ora_rmd_to_address.argtypes = [C.c_char_p, C.c_char_p]
        L.ora_addr_new.restype = C.c_void_p
        L.ora_addr_new.argtypes = [C.c_char_p, C.c_int]
        L.ora_addr_free.argtypes = [C.c_void_p]
        L.ora_addr_count.restype = C.c_uint64
        L.ora_addr_count.argtypes = [C.c_void_p]
        L.ora_addr_table.restype = C.c_void_p
        L.ora_addr_table.argtypes = [C.c_void_p]
        L.ora_addr_bloom.restype = P(Bloom)
        L.ora_addr_bloom.argtypes = [C.c_void_p]
        L.ora_addr_searchbinary.restype = C.c_int
        L.ora_addr_searchbinary.argtypes = [C.c_void_p, C.c_char_p]
        L.ora_addr_gen_new.restype = C.c_void_p
        L.ora_addr_gen_new.argtypes = [P(U256)]
        L.ora_addr_gen_free.argtypes = [C.c_void_p]
        L.ora_addr_gen_table.argtypes = [C.c_void_p, C.c_char_p]
        L.ora_mulmod_n.argtypes = [P(U256), P(U256), P(U256)]
        L.ora_endo_constants.argtypes = [C.c_int, P(U256), P(U256)]
        L.ora_addr_group.argtypes = [C.c_void_p, C.c_void_p, P(U256), C.c_int, C.c_void_p, P(C.c_uint32),
                                     C.c_uint32, P(C.c_uint32), P(U256), C.c_uint32, P(C.c_uint32)]
        _lib = L
    return _lib


SEARCH_ENDO = 4


def endo_constants(i: int) -> tuple[int, int]:
    """(lambda, beta) for i = 0, (lambda^2, beta^2) for i = 1 (keyhunt.cpp:582-585)."""
    lam, beta = U256(), U256()
    lib().ora_endo_constants(i, C.byref(lam), C.byref(beta))
    return lam.value(), beta.value()


def mulmod_n(a: int, b: int) -> int:
    r = U256()
    lib().ora_mulmod_n(C.byref(r), C.byref(U256.of(a)), C.byref(U256.of(b)))
    return r.value()


def xxh64(data: bytes, seed: int) -> int:
    return int(lib().ora_xxh64(data, len(data), seed))


def pubkey(k: int) -> Point:
    p = Point()
    lib().ora_compute_pubkey(C.byref(p), C.byref(U256.of(k)))
    return p


def pubkey_hex(k: int, compressed: bool = True) -> str:
    buf = C.create_string_buffer(140)
    lib().ora_pubkey_hex(C.byref(pubkey(k)), 1 if compressed else 0, buf)
    return buf.value.decode()


def parse_pubkey(s: str) -> tuple[Point, bool] | None:
    p = Point()
    comp = C.c_int(0)
    if not lib().ora_parse_pubkey_hex(s.encode(), C.byref(p), C.byref(comp)):
        return None
    return p, bool(comp.value)


def add_direct(a: Point, b: Point) -> Point:
    r = Point()
    lib().ora_add_direct(C.byref(r), C.byref(a), C.byref(b))
    return r


def negation(a: Point) -> Point:
    r = Point()
    lib().ora_negation(C.byref(r), C.byref(a))
    return r


class Bsgs:
    """The reference BSGS geometry + tables (keyhunt.cpp:1045-1880) built by the oracle."""

    def __init__(self, n: str | None = None, k: int = 1, threads: int = 8):
        err = C.create_string_buffer(256)
        self.h = lib().ora_bsgs_new(n.encode() if n else None, k, threads, err, 256)
        if not self.h:
            raise ValueError(err.value.decode())
        p = (C.c_uint64 * 10)()
        lib().ora_bsgs_params(self.h, p)
        (self.m, self.m2, self.m3, self.aux, self.cycles, self.n_low, self.l1ext, self.items1, self.items2,
         self.items3) = [int(v) for v in p]

    def close(self) -> None:
        if self.h:
            lib().ora_bsgs_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def bloom(self, level: int, idx: int) -> Bloom:
        return lib().ora_bsgs_bloom(self.h, level, idx).contents

    def bloom_concat(self, level: int = 1) -> tuple[bytes, int, int, int]:
        b0 = self.bloom(level, 0)
        parts = []
        for i in range(256):
            b = self.bloom(level, i)
            parts.append(C.string_at(b.bf, b.bytes))
        return b"".join(parts), int(b0.bytes), int(b0.bits), int(b0.hashes)

    def giant_table(self) -> bytes:
        buf = C.create_string_buffer(513 * 64)
        lib().ora_bsgs_giant_table(self.h, buf)
        return buf.raw

    def amp_table(self, level: int) -> bytes:
        buf = C.create_string_buffer(32 * 64)
        lib().ora_bsgs_amp_table(self.h, level, buf)
        return buf.raw

    def bptable(self) -> list[tuple[bytes, int]]:
        t = lib().ora_bsgs_bptable(self.h)
        return [(bytes(t[i].value), int(t[i].index)) for i in range(self.m3)]

    def chunk_start(self, base: int, target: Point) -> Point:
        r = Point()
        lib().ora_bsgs_chunk_start(self.h, C.byref(U256.of(base)), C.byref(target), C.byref(r))
        return r

    def scan(self, start: Point, j0: int, nj: int, want_x: bool = False, cap: int = 1 << 16):
        xs = C.create_string_buffer(nj * 1024 * 32) if want_x else None
        cand = (C.c_uint64 * cap)()
        n = C.c_uint32(0)
        nxt = Point()
        lib().ora_bsgs_scan(self.h, C.byref(start), j0, nj, xs, cand, cap, C.byref(n), C.byref(nxt))
        return [int(cand[i]) for i in range(min(n.value, cap))], (xs.raw if want_x else None), nxt

    def secondcheck(self, base: int, a: int, target: Point) -> int | None:
        key = U256()
        if lib().ora_bsgs_secondcheck(self.h, C.byref(U256.of(base)), a, C.byref(target), C.byref(key)):
            return key.value()
        return None

    def search(self, targets: list[Point], start: int, end: int, max_chunks: int = 0):
        n = len(targets)
        arr = (Point * n)(*targets)
        found = (C.c_int * n)()
        keys = (U256 * n)()
        chunks = lib().ora_bsgs_search(self.h, arr, n, C.byref(U256.of(start)), C.byref(U256.of(end)), max_chunks,
                                       found, keys)
        return int(chunks), [keys[i].value() if found[i] else None for i in range(n)]

    def bench(self, target: Point, base: int, threads: int, seconds: float) -> tuple[int, float]:
        el = C.c_double(0)
        steps = lib().ora_bsgs_bench(self.h, C.byref(target), C.byref(U256.of(base)), threads, seconds,
                                     C.byref(el))
        return int(steps), float(el.value)


# secp256k1 constants (SECP256K1.cpp:31-40)
P = 2**256 - 2**32 - 977
ORDER = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


# ---- -m address / -m rmd160 (ora_addr.c) ----
def sha256(data: bytes) -> bytes:
    out = C.create_string_buffer(32)
    lib().ora_sha256(data, len(data), out)
    return out.raw


def ripemd160(data: bytes) -> bytes:
    out = C.create_string_buffer(20)
    lib().ora_ripemd160(data, len(data), out)
    return out.raw


def hash160(data: bytes) -> bytes:
    out = C.create_string_buffer(20)
    lib().ora_hash160(data, len(data), out)
    return out.raw


def pub_hash160(p: Point, compressed: bool) -> bytes:
    out = C.create_string_buffer(20)
    lib().ora_pub_hash160(C.byref(p), 1 if compressed else 0, out)
    return out.raw


def x_hash160(prefix: int, x: int) -> bytes:
    out = C.create_string_buffer(20)
    lib().ora_x_hash160(prefix, C.byref(U256.of(x)), out)
    return out.raw


def b58decode(s: str, size: int = 25) -> tuple[bytes, int] | None:
    buf = C.create_string_buffer(size)
    sz = C.c_size_t(0)
    if not lib().ora_b58decode(s.encode(), buf, size, C.byref(sz)):
        return None
    return buf.raw, int(sz.value)


def rmd_to_address(rmd: bytes) -> str:
    out = C.create_string_buffer(64)
    lib().ora_rmd_to_address(rmd, out)
    return out.value.decode()


class AddrTable:
    """forceReadFileAddress + initBloomFilter + _sort over a target file's text."""

    def __init__(self, text: str, bloom_multiplier: int = 1):
        self.h = lib().ora_addr_new(text.encode(), bloom_multiplier)

    def close(self) -> None:
        if self.h:
            lib().ora_addr_free(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def n(self) -> int:
        return int(lib().ora_addr_count(self.h))

    def table(self) -> bytes:
        return C.string_at(lib().ora_addr_table(self.h), 20 * self.n)

    def bloom(self) -> Bloom:
        return lib().ora_addr_bloom(self.h).contents

    def bloom_bytes(self) -> bytes:
        b = self.bloom()
        return C.string_at(b.bf, b.bytes)

    def bloom_check(self, h20: bytes) -> bool:
        return bool(lib().ora_bloom_check(lib().ora_addr_bloom(self.h), h20, 20))

    def searchbinary(self, h20: bytes) -> bool:
        return bool(lib().ora_addr_searchbinary(self.h, h20))


class AddrGen:
    """init_generator: Gn[i] = (i+1)*stride*G, _2Gn = 1024*stride*G."""

    def __init__(self, stride: int = 1):
        self.h = lib().ora_addr_gen_new(C.byref(U256.of(stride)))
        self.stride = stride

    def close(self) -> None:
        if self.h:
            lib().ora_addr_gen_free(self.h)
            self.h = None

    def table(self) -> bytes:
        out = C.create_string_buffer(513 * 64)
        lib().ora_addr_gen_table(self.h, out)
        return out.raw

    def group(self, A: AddrTable, key: int, search: int = 2, want_xy: bool = False, cap: int = 1 << 12):
        """One thread_process group at first key `key`: (hits [(t, kind)], keys, xy bytes|None).  search | 4 = -e;
        kind = form | e << 2 (form 0/1 compressed 02/03, 2 uncompressed, 3 uncompressed of -P; e = lambda power)."""
        xy = C.create_string_buffer(1024 * 64) if want_xy else None
        hits = (C.c_uint32 * cap)()
        keys = (U256 * cap)()
        nh, nk = C.c_uint32(0), C.c_uint32(0)
        lib().ora_addr_group(A.h, self.h, C.byref(U256.of(key)), search, xy, hits, cap, C.byref(nh), keys, cap,
                             C.byref(nk))
        hl = [(int(hits[i]) >> 4, int(hits[i]) & 15) for i in range(min(nh.value, cap))]
        kl = [keys[i].value() for i in range(min(nk.value, cap))]
        return hl, kl, (xy.raw if want_xy else None)
