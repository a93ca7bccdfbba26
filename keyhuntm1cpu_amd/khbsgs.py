"""ctypes binding of libkhbsgs.so (include/khbsgs.h): the MI355X giant-step scan.

Replaces the CPU group loop of keyhunt.cpp:3867-4004 (thread_process_bsgs).  No fallback: if the
library or a gfx950 device is missing, KhbError is raised.
"""
from __future__ import annotations

import ctypes as C
import os

from . import LIB_DIR

LIB_PATH = os.path.join(LIB_DIR, "libkhbsgs.so")

KHB_GROUP = 1024


class KhbError(RuntimeError):
    pass


class Cand(C.Structure):
    _fields_ = [("job", C.c_uint32), ("a", C.c_uint32)]


class Degenerate(C.Structure):
    _fields_ = [("job", C.c_uint32), ("group", C.c_uint32)]


class AddrHit(C.Structure):
    _fields_ = [("job", C.c_uint32), ("group", C.c_uint32), ("t", C.c_uint32), ("kind", C.c_uint32)]


class CheckTables(C.Structure):     # khb_check_tables
    _fields_ = [("gtable", C.c_char_p), ("amp2", C.c_char_p), ("amp3", C.c_char_p),
                ("l2", C.c_char_p), ("l2_bytes_per_sub", C.c_uint64), ("l2_bits_per_sub", C.c_uint64),
                ("l2_hashes", C.c_uint32),
                ("l3", C.c_char_p), ("l3_bytes_per_sub", C.c_uint64), ("l3_bits_per_sub", C.c_uint64),
                ("l3_hashes", C.c_uint32),
                ("bptable", C.c_char_p), ("m3", C.c_uint64),
                ("m_double_be", C.c_uint8 * 32), ("m2_double_be", C.c_uint8 * 32), ("m3_be", C.c_uint8 * 32),
                ("m3_double_be", C.c_uint8 * 32)]


class CheckIn(C.Structure):        # khb_check_in
    _fields_ = [("start_be", C.c_uint8 * 32), ("a", C.c_uint32), ("target", C.c_uint32)]


class CheckOut(C.Structure):       # khb_check_out
    _fields_ = [("key_be", C.c_uint8 * 32), ("found", C.c_uint32), ("l2_hits", C.c_uint32),
                ("l3_hits", C.c_uint32), ("bp_hits", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("n_cand", C.c_uint32), ("n_degenerate", C.c_uint32), ("giant_steps", C.c_uint64),
                ("kernel_ms", C.c_float), ("launch_begin_ms", C.c_double), ("launch_end_ms", C.c_double),
                ("shader_mhz", C.c_float), ("event_ms", C.c_float)]


_libs: dict[str, C.CDLL] = {}
KHB_ABI_VERSION = 7


def lib(path: str | None = None) -> C.CDLL:
    """The bound library; `path` selects an alternative build (kernel variants in tools/)."""
    path = path or LIB_PATH
    if path not in _libs:
        if not os.path.exists(path):
            raise KhbError(f"{path} not built: run `make` (or __graft_entry__.build())")
        L = C.CDLL(path)
        P = C.POINTER
        # include/khbsgs.h KHB_ABI_VERSION: the structs and signatures below are written for it (older
        # timing-only variant builds without the symbol are accepted for tools/perf_variants.py)
        if hasattr(L, "khb_abi_version"):
            v = L.khb_abi_version()
            if v != KHB_ABI_VERSION:
                raise KhbError(f"{path}: ABI {v}, this binding is written for {KHB_ABI_VERSION}: rebuild (`make`)")
        elif path == LIB_PATH:
            raise KhbError(f"{path} predates khb_abi_version: rebuild (`make`)")
        L.khb_device_count.argtypes = [P(C.c_int)]
        L.khb_open.argtypes = [C.c_int, C.c_uint32, P(C.c_void_p)]
        L.khb_close.argtypes = [C.c_void_p]
        L.khb_strerror.restype = C.c_char_p
        L.khb_strerror.argtypes = [C.c_int]
        L.khb_last_hip_error.argtypes = [C.c_void_p]
        L.khb_stream.restype = C.c_void_p
        L.khb_stream.argtypes = [C.c_void_p]
        L.khb_lanes.restype = C.c_uint32
        L.khb_lanes.argtypes = [C.c_void_p]
        L.khb_default_lanes.restype = C.c_uint32
        L.khb_default_lanes.argtypes = [C.c_int]
        L.khb_groups_per_item.restype = C.c_uint32
        L.khb_groups_per_item.argtypes = []
        for name in ("khb_reserve_slots", "khb_set_candidate_capacity"):
            if hasattr(L, name):                 # absent only in older timing builds
                getattr(L, name).argtypes = [C.c_void_p, C.c_uint32 if "capacity" in name else C.c_int]
        if hasattr(L, "khb_candidate_capacity"):
            L.khb_candidate_capacity.restype = C.c_uint32
            L.khb_candidate_capacity.argtypes = [C.c_void_p]
            L.khb_reset_epoch.argtypes = [C.c_void_p]
        L.khb_load_bloom.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64, C.c_uint64, C.c_uint32]
        L.khb_load_giant_table.argtypes = [C.c_void_p, C.c_char_p]
        L.khb_load_gate.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint32]
        if hasattr(L, "khb_set_gate_stage1"):    # absent only in older timing builds (tools/perf_variants.py)
            L.khb_set_gate_stage1.argtypes = [C.c_void_p, C.c_uint32]
        if hasattr(L, "khb_build_info"):         # ABI 7
            L.khb_build_info.restype = C.c_char_p
            L.khb_build_info.argtypes = []
            L.khb_set_gate_stage0.argtypes = [C.c_void_p, C.c_uint32]
            L.khb_gate_stages.argtypes = [C.c_void_p]
            L.khb_last_handoff.argtypes = [C.c_void_p, P(C.c_uint32), P(C.c_uint32)]
        L.khb_load_lane_offsets.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint32]
        L.khb_submit.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32]
        L.khb_collect.argtypes = [C.c_void_p, P(Cand), C.c_uint32, P(Degenerate), C.c_uint32, P(Stats)]
        L.khb_scan.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32, P(Cand), C.c_uint32,
                               P(Stats)]
        L.khb_dump_x.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint32, C.c_char_p]
        L.khb_field_op.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_char_p, C.c_char_p, C.c_uint32]
        L.khb_probe.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_uint32]
        L.khb_load_addr_bloom.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64, C.c_uint64, C.c_uint32]
        L.khb_addr_submit.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int]
        L.khb_addr_collect.argtypes = [C.c_void_p, P(AddrHit), C.c_uint32, P(Stats)]
        L.khb_addr_scan.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                    P(AddrHit), C.c_uint32, P(Stats)]
        L.khb_addr_dump.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint32, C.c_char_p]
        L.khb_hash160.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_char_p, C.c_uint32]
        if hasattr(L, "khb_check"):              # ABI 5
            L.khb_load_check_tables.argtypes = [C.c_void_p, P(CheckTables)]
            L.khb_check.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, P(CheckIn), C.c_uint32, P(CheckOut)]
        _libs[path] = L
    return _libs[path]


KHB_EHANDOFF = -8


def _check(rc: int, ctx=None, L: C.CDLL | None = None) -> None:
    if rc != 0:
        L = L or lib()
        msg = L.khb_strerror(rc).decode()
        if ctx and rc == KHB_EHANDOFF and hasattr(L, "khb_last_handoff"):
            seen, total = C.c_uint32(0), C.c_uint32(0)
            L.khb_last_handoff(ctx, C.byref(seen), C.byref(total))
            msg += f" ({seen.value} of {total.value} waves)"
        elif ctx:
            msg += f" (hipError {L.khb_last_hip_error(ctx)})"
        raise KhbError(f"khbsgs: {msg} [{rc}]")


def build_info(path: str | None = None) -> dict:
    """khb_build_info of the library at `path` (the in-tree build by default) as a dict, plus its path and the
    first 16 hex digits of its sha256: what a bench line records so that its number names the kernel."""
    import hashlib
    path = os.path.realpath(path or LIB_PATH)
    L = lib(path)
    info = {}
    if hasattr(L, "khb_build_info"):
        for w in L.khb_build_info().decode().split(" compiler=")[0].split():
            k, _, v = w.partition("=")
            info[k] = v
        info["compiler"] = L.khb_build_info().decode().split(" compiler=", 1)[-1]
    with open(path, "rb") as f:
        info["sha16"] = hashlib.sha256(f.read()).hexdigest()[:16]
    info["path"] = path
    return info


def groups_per_item() -> int:
    """Groups per work item of the -m bsgs scan kernel (khb_groups_per_item)."""
    return int(lib().khb_groups_per_item())


def default_lanes(device: int = 0) -> int:
    """Work lanes of one full residency on `device` (khb_default_lanes; 0 = unusable)."""
    return int(lib().khb_default_lanes(device))


def device_count() -> int:
    n = C.c_int(0)
    _check(lib().khb_device_count(C.byref(n)))
    return n.value


class Engine:
    """One libkhbsgs context (one device)."""

    def __init__(self, device: int = 0, lanes: int = 0, lib_path: str | None = None):
        self.L = lib(lib_path)
        self.h = C.c_void_p()
        _check(self.L.khb_open(device, lanes, C.byref(self.h)), None, self.L)
        self.gpl = 0

    def close(self) -> None:
        if self.h:
            self.L.khb_close(self.h)
            self.h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def lanes(self) -> int:
        return int(self.L.khb_lanes(self.h))

    def stream(self) -> int:
        return int(self.L.khb_stream(self.h) or 0)

    def reserve_slots(self, depth: int) -> None:
        _check(self.L.khb_reserve_slots(self.h, depth), self.h, self.L)

    def set_candidate_capacity(self, cap: int) -> None:
        _check(self.L.khb_set_candidate_capacity(self.h, cap), self.h, self.L)

    def candidate_capacity(self) -> int:
        return int(self.L.khb_candidate_capacity(self.h))

    def reset_epoch(self) -> None:
        _check(self.L.khb_reset_epoch(self.h), self.h, self.L)

    def load_bloom(self, bf: bytes, bytes_per_sub: int, bits: int, hashes: int) -> None:
        assert len(bf) == 256 * bytes_per_sub
        _check(self.L.khb_load_bloom(self.h, bf, bytes_per_sub, bits, hashes), self.h, self.L)

    def load_gate(self, gate: bytes | None, log2_bits: int = 0, probes: int = 1) -> None:
        """Level-0 gate in front of the L1 probe (None removes it); probes = bits per x."""
        if gate is not None:
            assert len(gate) == (1 << log2_bits) // 8
        _check(self.L.khb_load_gate(self.h, gate, log2_bits if gate is not None else 0, probes), self.h, self.L)

    def set_gate_stage0(self, log2_bytes: int) -> None:
        """Stage-0 filter size for gates loaded later (0 none, 1 = KHB_GATE_STAGE0_AUTO, else log2 bytes)."""
        _check(self.L.khb_set_gate_stage0(self.h, log2_bytes), self.h, self.L)

    def gate_stages(self) -> int:
        """khb_gate_stages: bit 2 gate, bit 1 stage-1 fold, bit 0 stage-0 filter."""
        return int(self.L.khb_gate_stages(self.h))

    def set_gate_stage1(self, log2_bytes: int) -> None:
        """Stage-1 fold size (2^log2_bytes bytes) for gates loaded afterwards; 0 = none."""
        _check(self.L.khb_set_gate_stage1(self.h, log2_bytes), self.h, self.L)

    def load_giant_table(self, gsn: bytes) -> None:
        assert len(gsn) == 513 * 64
        _check(self.L.khb_load_giant_table(self.h, gsn), self.h, self.L)

    def load_lane_offsets(self, offs: bytes, gpl: int) -> None:
        assert len(offs) % 64 == 0
        _check(self.L.khb_load_lane_offsets(self.h, offs, len(offs) // 64, gpl), self.h, self.L)
        self.gpl = gpl

    def submit(self, centres: bytes, group_begin: int, group_count: int) -> None:
        _check(self.L.khb_submit(self.h, centres, len(centres) // 64, group_begin, group_count), self.h, self.L)

    def collect(self, cap: int = 1 << 20):
        cand = (Cand * cap)()
        deg = (Degenerate * 4096)()
        st = Stats()
        _check(self.L.khb_collect(self.h, cand, cap, deg, 4096, C.byref(st)), self.h, self.L)
        n = min(st.n_cand, cap)
        return ([(int(cand[i].job), int(cand[i].a)) for i in range(n)],
                [(int(deg[i].job), int(deg[i].group)) for i in range(min(st.n_degenerate, 4096))], st)

    def scan(self, centres: bytes, group_begin: int, group_count: int, cap: int = 1 << 20):
        self.submit(centres, group_begin, group_count)
        return self.collect(cap)

    def dump_x(self, centre: bytes, group_begin: int, group_count: int) -> bytes:
        out = C.create_string_buffer(group_count * KHB_GROUP * 32)
        _check(self.L.khb_dump_x(self.h, centre, group_begin, group_count, out), self.h, self.L)
        return out.raw

    def field_op(self, op: int, a: bytes, b: bytes | None) -> bytes:
        n = len(a) // 32
        out = C.create_string_buffer(n * 32)
        _check(self.L.khb_field_op(self.h, op, a, b, out, n), self.h, self.L)
        return out.raw

    def probe(self, xs: bytes) -> bytes:
        n = len(xs) // 32
        out = C.create_string_buffer(n)
        _check(self.L.khb_probe(self.h, xs, out, n), self.h, self.L)
        return out.raw

    # ---- -m address ----
    def load_addr_bloom(self, bf: bytes, bits: int, hashes: int) -> None:
        _check(self.L.khb_load_addr_bloom(self.h, bf, len(bf), bits, hashes), self.h, self.L)

    def addr_scan(self, centres: bytes, group_begin: int, group_count: int, search: int = 2, cap: int = 1 << 18):
        """Bloom hits [(job, group, t, kind)] of -m address over group_count groups of each job."""
        hits = (AddrHit * cap)()
        st = Stats()
        _check(self.L.khb_addr_scan(self.h, centres, len(centres) // 64, group_begin, group_count, search, hits, cap,
                                    C.byref(st)), self.h, self.L)
        n = min(st.n_cand, cap)
        return [(int(hits[i].job), int(hits[i].group), int(hits[i].t), int(hits[i].kind)) for i in range(n)], st

    def addr_dump(self, centre: bytes, group_begin: int, group_count: int) -> bytes:
        out = C.create_string_buffer(group_count * KHB_GROUP * 64)
        _check(self.L.khb_addr_dump(self.h, centre, group_begin, group_count, out), self.h, self.L)
        return out.raw

    def hash160(self, kind: int, xy: bytes) -> list[tuple[bytes, int]]:
        """[(hash160, bloom bit)] of each x||y point for kind 0/1 (compressed 02/03) or 2."""
        n = len(xy) // 64
        out = C.create_string_buffer(21 * n)
        _check(self.L.khb_hash160(self.h, kind, xy, out, n), self.h, self.L)
        r = out.raw
        return [(r[21 * i:21 * i + 20], r[21 * i + 20]) for i in range(n)]

    # ---- second / third check (khb_load_check_tables, khb_check) ----
    def load_check_tables(self, gtable: bytes, amp2: bytes, amp3: bytes, l2: tuple, l3: tuple, bptable: bytes,
                          m3: int, m_double: int, m2_double: int, m3_value: int, m3_double: int) -> None:
        """l2 / l3: (256 sub-blooms concatenated, bytes per sub-bloom, bits, hashes) as bloom_concat gives them.
        The library copies every table to the device before it returns."""
        assert len(gtable) == 32 * 256 * 64 and len(amp2) == len(amp3) == 32 * 64 and len(bptable) == 16 * m3
        t = CheckTables()
        t.gtable, t.amp2, t.amp3 = gtable, amp2, amp3
        t.l2, t.l2_bytes_per_sub, t.l2_bits_per_sub, t.l2_hashes = l2
        t.l3, t.l3_bytes_per_sub, t.l3_bits_per_sub, t.l3_hashes = l3
        t.bptable, t.m3 = bptable, m3
        for name, v in (("m_double_be", m_double), ("m2_double_be", m2_double), ("m3_be", m3_value),
                        ("m3_double_be", m3_double)):
            getattr(t, name)[:] = list(v.to_bytes(32, "big"))
        _check(self.L.khb_load_check_tables(self.h, C.byref(t)), self.h, self.L)

    def check(self, targets_xy: list[bytes], cands: list[tuple[int, int, int]]) -> list[dict]:
        """bsgs_secondcheck on the device for [(chunk base, giant step a, target index)]: per candidate
        {"found", "key" (int or None), "l2_hits", "l3_hits", "bp_hits"}."""
        n = len(cands)
        ins = (CheckIn * max(1, n))()
        for i, (base, a, k) in enumerate(cands):
            ins[i].start_be[:] = list(base.to_bytes(32, "big"))
            ins[i].a = a
            ins[i].target = k
        outs = (CheckOut * max(1, n))()
        _check(self.L.khb_check(self.h, b"".join(targets_xy), len(targets_xy), ins, n, outs), self.h, self.L)
        return [{"found": int(o.found), "key": int.from_bytes(bytes(o.key_be), "big") if o.found else None,
                 "l2_hits": int(o.l2_hits), "l3_hits": int(o.l3_hits), "bp_hits": int(o.bp_hits)}
                for o in outs[:n]]
