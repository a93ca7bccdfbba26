"""ctypes binding of libkhhost.so (include/khhost.h): the C++ host engine — BSGS geometry, tables,
chunk centres, second/third check and the multi-GPU search driver the keyhunt_amd CLI runs."""
from __future__ import annotations

import ctypes as C
import os

from . import LIB_DIR

LIB_PATH = os.path.join(LIB_DIR, "libkhhost.so")

_lib = None


KHH_ABI_VERSION = 6                 # include/khhost.h
KHH_SESSION_STATS, KHH_ADDR_STATS = 12, 8


class KhhError(RuntimeError):
    pass


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise KhhError(f"{LIB_PATH} not built: run `make`")
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        v = L.khh_abi_version() if hasattr(L, "khh_abi_version") else 0
        if v != KHH_ABI_VERSION:        # include/khhost.h KHH_ABI_VERSION
            raise KhhError(f"{LIB_PATH}: ABI {v}, this binding is written for {KHH_ABI_VERSION}: rebuild (`make`)")
        L.khh_tables_new.restype = C.c_void_p
        L.khh_tables_new.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_uint32, C.c_char_p, C.c_size_t]
        L.khh_tables_free.argtypes = [C.c_void_p]
        L.khh_tables_new_files.restype = C.c_void_p
        L.khh_tables_new_files.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_uint32, C.c_char_p, C.c_int, C.c_int,
                                           P(C.c_uint32), C.c_char_p, C.c_size_t]
        L.khh_tables_save.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_size_t]
        L.khh_tables_new_gpu.restype = C.c_void_p
        L.khh_tables_new_gpu.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_uint32, C.c_int, P(C.c_double), C.c_char_p,
                                         C.c_size_t]
        L.khh_params.argtypes = [C.c_void_p, P(C.c_uint64)]
        L.khh_bloom.restype = P(C.c_uint8)
        L.khh_bloom.argtypes = [C.c_void_p, C.c_int, C.c_int, P(C.c_uint64), P(C.c_uint64), P(C.c_uint32)]
        L.khh_giant_table.argtypes = [C.c_void_p, C.c_char_p]
        L.khh_amp_table.argtypes = [C.c_void_p, C.c_int, C.c_char_p]
        L.khh_lane_offsets.restype = C.c_uint32
        L.khh_lane_offsets.argtypes = [C.c_void_p, C.c_char_p, P(C.c_uint32)]
        L.khh_bptable.restype = P(C.c_uint8)
        L.khh_bptable.argtypes = [C.c_void_p, P(C.c_uint64)]
        L.khh_gate.restype = C.c_void_p
        L.khh_gate.argtypes = [C.c_void_p, P(C.c_uint32)]
        L.khh_gate_probes.restype = C.c_uint32
        L.khh_gate_probes.argtypes = [C.c_void_p]
        L.khh_chunk_centre.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_char_p]
        L.khh_job_centres.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_char_p, C.c_uint32, C.c_char_p, C.c_int]
        L.khh_secondcheck.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_char_p, C.c_char_p]
        L.khh_search.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.c_char_p, C.c_char_p, P(C.c_int), C.c_int,
                                 C.c_uint32, C.c_uint32, C.c_uint64, P(C.c_int), C.c_char_p, P(C.c_uint64),
                                 C.c_char_p, C.c_size_t]
        L.khh_session_open.restype = C.c_void_p
        L.khh_session_open.argtypes = [C.c_void_p, P(C.c_int), C.c_int, C.c_uint32, C.c_uint32, C.c_int, C.c_char_p,
                                       C.c_size_t]
        L.khh_session_run.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.c_char_p, C.c_char_p, C.c_uint64, C.c_int,
                                      P(C.c_int), C.c_char_p, P(C.c_uint64), C.c_char_p, C.c_size_t]
        L.khh_session_run_ex.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.c_char_p, C.c_char_p, C.c_uint64,
                                         C.c_int, P(C.c_int), C.c_char_p, P(C.c_uint64), C.c_uint32, C.c_char_p,
                                         C.c_size_t]
        L.khh_session_close.argtypes = [C.c_void_p]
        L.khh_session_set_test_hooks.argtypes = [C.c_void_p, C.c_uint32, C.c_int, C.c_int, C.c_char_p]
        L.khh_session_set_check_mode.argtypes = [C.c_void_p, C.c_int]
        L.khh_session_set_chunk_mode.argtypes = [C.c_void_p, C.c_int]
        L.khh_chunk_sequence.restype = C.c_uint64
        L.khh_chunk_sequence.argtypes = [C.c_int, C.c_char_p, C.c_char_p, C.c_char_p, C.c_uint64, C.c_char_p,
                                         C.c_uint64]
        L.khh_gtable.argtypes = [C.c_char_p]
        L.khh_session_recorded.restype = C.c_uint64
        L.khh_session_recorded.argtypes = [C.c_void_p, C.c_char_p, P(C.c_uint32), P(C.c_uint32), C.c_uint64]
        L.khh_pubkey.argtypes = [C.c_char_p, C.c_char_p]
        L.khh_parse_pubkey.argtypes = [C.c_char_p, C.c_char_p, P(C.c_int)]
        L.khh_addr_new.restype = C.c_void_p
        L.khh_addr_new.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_uint64, C.c_uint32, C.c_int, C.c_char_p,
                                   C.c_size_t]
        L.khh_addr_free.argtypes = [C.c_void_p]
        L.khh_addr_table.restype = P(C.c_uint8)
        L.khh_addr_table.argtypes = [C.c_void_p, P(C.c_uint64)]
        L.khh_addr_bloom.restype = P(C.c_uint8)
        L.khh_addr_bloom.argtypes = [C.c_void_p, P(C.c_uint64), P(C.c_uint64), P(C.c_uint32)]
        L.khh_addr_giant_table.argtypes = [C.c_void_p, C.c_char_p]
        L.khh_addr_lane_offsets.restype = C.c_uint32
        L.khh_addr_lane_offsets.argtypes = [C.c_void_p, C.c_char_p, P(C.c_uint32)]
        L.khh_addr_search.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_int, C.c_int, P(C.c_int), C.c_int,
                                      C.c_uint32, C.c_uint64, C.c_char_p, C.c_char_p, C.c_char_p, C.c_uint32,
                                      P(C.c_uint32), P(C.c_uint64), C.c_char_p, C.c_size_t]
        L.khh_addr_search_ex.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_int, C.c_int, P(C.c_int), C.c_int,
                                         C.c_uint32, C.c_uint64, C.c_char_p, C.c_char_p, C.c_char_p, C.c_uint32,
                                         P(C.c_uint32), P(C.c_uint64), C.c_uint32, C.c_char_p, C.c_size_t]
        L.khh_addr_set_hit_capacity.argtypes = [C.c_void_p, C.c_uint32]
        L.khh_addr_confirm.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_char_p, C.POINTER(C.c_int)]
        L.khh_hash160.argtypes = [C.c_char_p, C.c_int, C.c_char_p]
        L.khh_rmd_to_address.argtypes = [C.c_char_p, C.c_char_p]
        _lib = L
    return _lib


def _b32(v: int) -> bytes:
    return int(v).to_bytes(32, "big")


def pubkey(k: int) -> bytes:
    out = C.create_string_buffer(64)
    if lib().khh_pubkey(_b32(k), out):
        raise KhhError("invalid private key")
    return out.raw


def parse_pubkey(s: str) -> tuple[bytes, bool] | None:
    out = C.create_string_buffer(64)
    comp = C.c_int(0)
    if lib().khh_parse_pubkey(s.encode(), out, C.byref(comp)):
        return None
    return out.raw, bool(comp.value)


class Tables:
    """keyhunt's BSGS tables built by the product host engine."""

    def __init__(self, n: str | None = None, k: int = 1, threads: int = 0, gpl: int = 4,
                 files_dir: str | None = None, save: bool = False, skip_checksum: bool = False,
                 gpu_device: int | None = None):
        """files_dir: -S semantics — read the reference's table files from that directory, compute
        only what is missing, and with save=True write the missing files back (self.have = mask)."""
        err = C.create_string_buffer(256)
        self.have = 0
        self.build_ms = 0.0
        if gpu_device is not None:
            ms = C.c_double(0)
            self.h = lib().khh_tables_new_gpu(n.encode() if n else None, k, threads, gpl, gpu_device, C.byref(ms),
                                              err, 256)
            self.build_ms = ms.value
        elif files_dir is not None:
            have = C.c_uint32(0)
            self.h = lib().khh_tables_new_files(n.encode() if n else None, k, threads, gpl, files_dir.encode(),
                                                1 if skip_checksum else 0, 1 if save else 0, C.byref(have), err, 256)
            self.have = int(have.value)
        else:
            self.h = lib().khh_tables_new(n.encode() if n else None, k, threads, gpl, err, 256)
        if not self.h:
            raise KhhError(err.value.decode())
        p = (C.c_uint64 * 10)()
        lib().khh_params(self.h, p)
        (self.m, self.m2, self.m3, self.aux, self.cycles, self.n_low, self.l1ext, self.items1, self.items2,
         self.items3) = [int(v) for v in p]

    def close(self) -> None:
        if self.h:
            lib().khh_tables_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def save_files(self, directory: str) -> None:
        err = C.create_string_buffer(256)
        if lib().khh_tables_save(self.h, directory.encode(), err, 256):
            raise KhhError(err.value.decode())

    def bloom(self, level: int, idx: int) -> tuple[bytes, int, int]:
        nb, bits, h = C.c_uint64(), C.c_uint64(), C.c_uint32()
        p = lib().khh_bloom(self.h, level, idx, C.byref(nb), C.byref(bits), C.byref(h))
        return C.string_at(p, nb.value), int(bits.value), int(h.value)

    def bloom_concat(self, level: int = 1) -> tuple[bytes, int, int, int]:
        parts = [self.bloom(level, i)[0] for i in range(256)]
        _, bits, h = self.bloom(level, 0)
        return b"".join(parts), len(parts[0]), bits, h

    def giant_table(self) -> bytes:
        b = C.create_string_buffer(513 * 64)
        lib().khh_giant_table(self.h, b)
        return b.raw

    def amp_table(self, level: int) -> bytes:
        b = C.create_string_buffer(32 * 64)
        lib().khh_amp_table(self.h, level, b)
        return b.raw

    def lane_offsets(self) -> tuple[bytes, int]:
        g = C.c_uint32()
        n = lib().khh_lane_offsets(self.h, None, C.byref(g))
        b = C.create_string_buffer(64 * n)
        lib().khh_lane_offsets(self.h, b, C.byref(g))
        return b.raw, int(g.value)

    def gate_probes(self) -> int:
        """Bits per x of the level-0 gate (khb_load_gate's probes); 0 when there is no gate."""
        return int(lib().khh_gate_probes(self.h))

    def gate(self) -> tuple[bytes, int]:
        """The level-0 gate (khb_load_gate) and its log2 size; (b"", 0) when the tables have none."""
        lg = C.c_uint32(0)
        p = lib().khh_gate(self.h, C.byref(lg))
        return (C.string_at(p, (1 << lg.value) // 8) if lg.value else b""), int(lg.value)

    def bptable(self) -> list[tuple[bytes, int]]:
        n = C.c_uint64()
        p = lib().khh_bptable(self.h, C.byref(n))
        raw = C.string_at(p, 16 * n.value)
        return [(raw[16 * i:16 * i + 6], int.from_bytes(raw[16 * i + 8:16 * i + 16], "little")) for i in range(n.value)]

    def bptable_raw(self) -> bytes:
        """bPtable as m3 x 16-byte struct bsgs_xvalue records (khb_check_tables.bptable)."""
        n = C.c_uint64()
        p = lib().khh_bptable(self.h, C.byref(n))
        return C.string_at(p, 16 * n.value)

    def check_tables(self) -> dict:
        """Everything khb_load_check_tables takes, from these tables (Engine.load_check_tables(**...))."""
        l2, nb2, bits2, h2 = self.bloom_concat(2)
        l3, nb3, bits3, h3 = self.bloom_concat(3)
        return {"gtable": gtable(), "amp2": self.amp_table(2), "amp3": self.amp_table(3),
                "l2": (l2, nb2, bits2, h2), "l3": (l3, nb3, bits3, h3), "bptable": self.bptable_raw(), "m3": self.m3,
                "m_double": 2 * self.m, "m2_double": 2 * self.m2, "m3_value": self.m3, "m3_double": 2 * self.m3}

    def chunk_centre(self, base: int, target_xy: bytes) -> bytes:
        out = C.create_string_buffer(64)
        lib().khh_chunk_centre(self.h, _b32(base), target_xy, out)
        return out.raw

    def job_centres(self, bases: list[int], targets_xy: list[bytes], threads: int = 8) -> bytes:
        """The engine's batched centres of every (chunk, target) job, chunk-major (khh_job_centres)."""
        out = C.create_string_buffer(64 * len(bases) * len(targets_xy))
        lib().khh_job_centres(self.h, b"".join(_b32(b) for b in bases), len(bases), b"".join(targets_xy),
                              len(targets_xy), out, threads)
        return out.raw

    def secondcheck(self, base: int, a: int, target_xy: bytes) -> int | None:
        key = C.create_string_buffer(32)
        if lib().khh_secondcheck(self.h, _b32(base), a, target_xy, key):
            return int.from_bytes(key.raw, "big")
        return None

    def search(self, targets_xy: list[bytes], start: int, end: int, devices=(0,), lanes: int = 0,
               chunks_per_batch: int = 0, max_chunks: int = 0):
        n = len(targets_xy)
        found = (C.c_int * n)()
        keys = C.create_string_buffer(32 * n)
        stats = (C.c_uint64 * 6)()
        devs = (C.c_int * len(devices))(*devices)
        err = C.create_string_buffer(256)
        rc = lib().khh_search(self.h, b"".join(targets_xy), n, _b32(start), _b32(end), devs, len(devices), lanes,
                              chunks_per_batch, max_chunks, found, keys, stats, err, 256)
        if rc:
            raise KhhError(f"search failed ({rc}): {err.value.decode()}")
        res = [int.from_bytes(keys.raw[32 * i:32 * i + 32], "big") if found[i] else None for i in range(n)]
        return res, {"chunks": stats[0], "giant_steps": stats[1], "candidates": stats[2], "degenerate": stats[3],
                     "kernel_s": stats[4] / 1e6, "launches": stats[5]}


_STAT_KEYS = ("chunks", "giant_steps", "candidates", "degenerate", "kernel_s", "launches", "rescans", "busy_s",
              "shader_mhz", "device_checked", "device_check_s", "event_s")
CHECK_HOST, CHECK_DEVICE, CHECK_AUTO = 0, 1, 2      # include/khhost.h KHH_CHECK_*
BSGS_MODES = ("sequential", "backward", "both", "random", "dance")     # keyhunt.cpp:227, -B


def chunk_sequence(mode: int, start: int, end: int, two_n: int, seed: int = 1, cap: int = 1 << 16) -> list[int]:
    """The chunk bases -B mode `mode` claims from [start, end) (khh_chunk_sequence; the engine's order)."""
    out = C.create_string_buffer(32 * cap)
    n = lib().khh_chunk_sequence(mode, _b32(start), _b32(end), _b32(two_n), seed, out, cap)
    return [int.from_bytes(out.raw[32 * i:32 * i + 32], "big") for i in range(n)]


def gtable() -> bytes:
    """Secp256K1::Init's GTable as 32*256 points x||y BE (khh_gtable; khb_check_tables.gtable)."""
    b = C.create_string_buffer(32 * 256 * 64)
    lib().khh_gtable(b)
    return b.raw


class Session:
    """Opened devices with the tables resident in HBM (khh_session_*)."""

    def __init__(self, tables: Tables, devices=(0,), lanes: int = 0, chunks_per_batch: int = 0,
                 check_threads: int = 0):
        self.tables = tables
        devs = (C.c_int * len(devices))(*devices)
        err = C.create_string_buffer(256)
        self.h = lib().khh_session_open(tables.h, devs, len(devices), lanes, chunks_per_batch, check_threads, err, 256)
        if not self.h:
            raise KhhError(err.value.decode())

    def close(self) -> None:
        if self.h:
            lib().khh_session_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def run(self, targets_xy: list[bytes], start: int, end: int, max_chunks: int = 0, random_chunks: bool = False):
        n = len(targets_xy)
        found = (C.c_int * n)()
        keys = C.create_string_buffer(32 * n)
        stats = (C.c_uint64 * KHH_SESSION_STATS)()
        err = C.create_string_buffer(256)
        rc = lib().khh_session_run_ex(self.h, b"".join(targets_xy), n, _b32(start), _b32(end), max_chunks,
                                      1 if random_chunks else 0, found, keys, stats, KHH_SESSION_STATS, err, 256)
        if rc:
            raise KhhError(f"search failed ({rc}): {err.value.decode()}")
        res = [int.from_bytes(keys.raw[32 * i:32 * i + 32], "big") if found[i] else None for i in range(n)]
        st = {k: int(stats[i]) for i, k in enumerate(_STAT_KEYS)}
        st["kernel_s"] = stats[4] / 1e6
        st["busy_s"] = stats[7] / 1e6
        st["shader_mhz"] = stats[8] / 1e3
        st["device_check_s"] = stats[10] / 1e6
        st["event_s"] = stats[11] / 1e6
        return res, st

    def set_chunk_mode(self, mode: int) -> None:
        """keyhunt's -B mode for later runs: BSGS_MODES.index(name) (0 sequential ... 4 dance)."""
        rc = lib().khh_session_set_chunk_mode(self.h, mode)
        if rc:
            raise KhhError(f"set_chunk_mode failed ({rc})")

    def set_check_mode(self, mode: int) -> None:
        """Where later runs confirm candidates: CHECK_HOST (CPU pool), CHECK_DEVICE (khb_check), CHECK_AUTO."""
        rc = lib().khh_session_set_check_mode(self.h, mode)
        if rc:
            raise KhhError(f"set_check_mode failed ({rc})")

    def set_test_hooks(self, cand_cap: int = 0, use_gate: bool = True, record: bool = False,
                       l1_concat: bytes | None = None) -> None:
        """Tests: candidate ring capacity (0 = default), gate on/off, candidate recording, replacement L1."""
        rc = lib().khh_session_set_test_hooks(self.h, cand_cap, 1 if use_gate else 0, 1 if record else 0, l1_concat)
        if rc:
            raise KhhError(f"set_test_hooks failed ({rc})")

    def recorded(self) -> list[tuple[int, int, int]]:
        """Level-1 candidates of the last run: (chunk base, target index, a)."""
        n = lib().khh_session_recorded(self.h, None, None, None, 0)
        bases = C.create_string_buffer(32 * max(1, n))
        tg = (C.c_uint32 * max(1, n))()
        a = (C.c_uint32 * max(1, n))()
        lib().khh_session_recorded(self.h, bases, tg, a, n)
        return [(int.from_bytes(bases.raw[32 * i:32 * i + 32], "big"), int(tg[i]), int(a[i])) for i in range(n)]


# ---- -m address / -m rmd160 ----
def hash160(xy: bytes, compressed: bool) -> bytes:
    out = C.create_string_buffer(20)
    lib().khh_hash160(xy, 1 if compressed else 0, out)
    return out.raw


def rmd_to_address(rmd: bytes) -> str:
    out = C.create_string_buffer(64)
    lib().khh_rmd_to_address(rmd, out)
    return out.value.decode()


class Addr:
    """-m address targets (a target file's text) + generator for chunks of n_seq keys."""

    def __init__(self, text: str, n_seq: int = 1 << 32, stride: int = 1, gpl: int = 16, bloom_multiplier: int = 1,
                 threads: int = 0):
        err = C.create_string_buffer(256)
        self.h = lib().khh_addr_new(text.encode(), bloom_multiplier, _b32(stride), n_seq, gpl, threads, err, 256)
        if not self.h:
            raise KhhError(err.value.decode())
        self.n_seq, self.stride = n_seq, stride

    def close(self) -> None:
        if self.h:
            lib().khh_addr_free(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def table(self) -> list[bytes]:
        n = C.c_uint64(0)
        p = lib().khh_addr_table(self.h, C.byref(n))
        raw = C.string_at(p, 20 * n.value) if n.value else b""
        return [raw[20 * i:20 * i + 20] for i in range(n.value)]

    def bloom(self) -> tuple[bytes, int, int]:
        nb, bits, h = C.c_uint64(0), C.c_uint64(0), C.c_uint32(0)
        p = lib().khh_addr_bloom(self.h, C.byref(nb), C.byref(bits), C.byref(h))
        return C.string_at(p, nb.value), int(bits.value), int(h.value)

    def giant_table(self) -> bytes:
        out = C.create_string_buffer(513 * 64)
        lib().khh_addr_giant_table(self.h, out)
        return out.raw

    def lane_offsets(self) -> tuple[bytes, int]:
        g = C.c_uint32(0)
        n = lib().khh_addr_lane_offsets(self.h, None, C.byref(g))
        out = C.create_string_buffer(64 * n)
        lib().khh_addr_lane_offsets(self.h, out, C.byref(g))
        return out.raw, int(g.value)

    def set_hit_capacity(self, cap: int) -> None:
        """Tests: the launches' bloom-hit ring capacity (0 = default 2^18); overflow -> rescan in parts."""
        if lib().khh_addr_set_hit_capacity(self.h, cap):
            raise KhhError("khh_addr_set_hit_capacity")

    def confirm(self, key: int, kind: int):
        """khh_addr_confirm: (key, compressed) recovered from a bloom hit of kind `kind` on the point of `key`, or
        None when its hash is not a target."""
        out = C.create_string_buffer(32)
        comp = C.c_int(0)
        r = lib().khh_addr_confirm(self.h, _b32(key), kind, out, C.byref(comp))
        if r < 0:
            raise KhhError(f"khh_addr_confirm [{r}]")
        return (int.from_bytes(out.raw, "big"), bool(comp.value)) if r == 1 else None

    def search(self, start: int, end: int, search: int = 2, devices=(0,), lanes: int = 0, max_chunks: int = 0,
               random_chunks: bool = False, cap: int = 4096):
        """Found [(key, compressed, rmd160)] in discovery order, plus stats.  search | 4 (KHB_SEARCH_ENDOMORPHISM)
        is -e."""
        keys = C.create_string_buffer(32 * cap)
        comp = C.create_string_buffer(cap)
        rmd = C.create_string_buffer(20 * cap)
        nf = C.c_uint32(0)
        st = (C.c_uint64 * KHH_ADDR_STATS)()
        devs = (C.c_int * len(devices))(*devices)
        err = C.create_string_buffer(256)
        rc = lib().khh_addr_search_ex(self.h, _b32(start), _b32(end), search, 1 if random_chunks else 0, devs,
                                      len(devices), lanes, max_chunks, keys, comp, rmd, cap, C.byref(nf), st,
                                      KHH_ADDR_STATS, err, 256)
        if rc:
            raise KhhError(f"khh_addr_search: {err.value.decode()} [{rc}]")
        n = min(nf.value, cap)
        found = [(int.from_bytes(keys.raw[32 * i:32 * i + 32], "big"), bool(comp.raw[i]), rmd.raw[20 * i:20 * i + 20])
                 for i in range(n)]
        return found, {"chunks": st[0], "keys": st[1], "hits": st[2], "degenerate": st[3], "kernel_s": st[4] / 1e6,
                       "launches": st[5], "shader_mhz": st[6] / 1e3, "rescans": st[7]}
