"""CPU-only checks of the native boundary: every symbol include/*.h declares is exported by the
built libraries, and the libraries load without a GPU (no compute calls)."""
from __future__ import annotations

import ctypes as C
import os
import re

from keyhuntm1cpu_amd import LIB_DIR, REPO_DIR


def declared(header: str) -> list[str]:
    src = open(os.path.join(REPO_DIR, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kh[bh]_[a-z0-9_]+)\s*\(", src)))


def test_khbsgs_exports_every_declared_symbol():
    lib = C.CDLL(os.path.join(LIB_DIR, "libkhbsgs.so"))
    names = declared("khbsgs.h")
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n


def test_khhost_exports_every_declared_symbol():
    lib = C.CDLL(os.path.join(LIB_DIR, "libkhhost.so"))
    names = declared("khhost.h")
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n


def test_no_gpu_fails_loudly():
    """Without a gfx950 device the library refuses to open (no CPU fallback)."""
    from keyhuntm1cpu_amd import khbsgs
    if khbsgs.device_count() > 0:
        return
    try:
        khbsgs.Engine(0)
    except khbsgs.KhbError as e:
        assert "gfx950" in str(e) or "device" in str(e)
    else:
        raise AssertionError("Engine opened without a GPU")


def test_strerror():
    lib = C.CDLL(os.path.join(LIB_DIR, "libkhbsgs.so"))
    lib.khb_strerror.restype = C.c_char_p
    assert lib.khb_strerror(0) == b"ok"
    assert b"gfx950" in lib.khb_strerror(-2)


def test_null_context_is_einval():
    """Entry points that take a context reject a null one with KHB_EINVAL (-1) before any HIP call."""
    lib = C.CDLL(os.path.join(LIB_DIR, "libkhbsgs.so"))
    lib.khb_set_gate_stage1.argtypes = [C.c_void_p, C.c_uint32]
    lib.khb_load_gate.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint32]
    assert lib.khb_set_gate_stage1(None, 25) == -1
    assert lib.khb_load_gate(None, None, 0, 1) == -1


def _header_define(header: str, name: str) -> int:
    src = open(os.path.join(REPO_DIR, "include", header)).read()
    return int(re.search(r"#define\s+" + name + r"\s+(\d+)", src).group(1))


def test_abi_versions_match_headers_and_bindings():
    """The libraries report the ABI version their headers declare, and the Python bindings are written
    for that version (they refuse a library of another one)."""
    from keyhuntm1cpu_amd import khbsgs, khhost
    b = C.CDLL(os.path.join(LIB_DIR, "libkhbsgs.so"))
    h = C.CDLL(os.path.join(LIB_DIR, "libkhhost.so"))
    assert b.khb_abi_version() == _header_define("khbsgs.h", "KHB_ABI_VERSION") == khbsgs.KHB_ABI_VERSION
    assert h.khh_abi_version() == _header_define("khhost.h", "KHH_ABI_VERSION") == khhost.KHH_ABI_VERSION
    assert _header_define("khhost.h", "KHH_SESSION_STATS") == khhost.KHH_SESSION_STATS
    assert _header_define("khhost.h", "KHH_ADDR_STATS") == khhost.KHH_ADDR_STATS
    khbsgs.lib()
    khhost.lib()


def test_khb_stats_layout():
    """khb_stats as the binding reads it (include/khbsgs.h, ABI 6: event_ms fills shader_mhz's padding)."""
    from keyhuntm1cpu_amd.khbsgs import Stats
    assert [f for f, _ in Stats._fields_] == ["n_cand", "n_degenerate", "giant_steps", "kernel_ms", "launch_begin_ms",
                                             "launch_end_ms", "shader_mhz", "event_ms"]
    assert C.sizeof(Stats) == 48
