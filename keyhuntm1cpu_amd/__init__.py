"""keyhuntm1cpu_amd — MI355X-native BSGS giant-step engine for keyhunt's `-m bsgs` path.

Native parts (built in-tree by `make`, see __graft_entry__.build):
  lib/libkhbsgs.so   HIP/gfx950 giant-step library behind include/khbsgs.h (the drop-in boundary)
  lib/libkhhost.so   C++ host engine (geometry, tables, chunk scheduling, second/third check)
  bin/keyhunt_amd    keyhunt-compatible CLI (-m bsgs ...) driving both

The Python modules are thin ctypes bindings used by tests and bench.py; there is no Python or CPU
fallback for the giant-step scan: loading fails loudly when the native library is missing.
"""
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# KHB_LIB_DIR: another directory holding a libkhbsgs.so + libkhhost.so pair (whole-bench A/B of a kernel build,
# tools/gpu/bench_ab.sh); the in-tree lib/ otherwise
LIB_DIR = os.environ.get("KHB_LIB_DIR") or os.path.join(PKG_DIR, "lib")
BIN_DIR = os.path.join(PKG_DIR, "bin")
REPO_DIR = os.path.dirname(PKG_DIR)

__all__ = ["PKG_DIR", "LIB_DIR", "BIN_DIR", "REPO_DIR"]
