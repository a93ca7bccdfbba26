"""Host-compiled checks of the device headers (fe.hpp, bloom_probe.hpp, hash160.hpp) against the
oracle: the arithmetic and hashing the kernels run, executed on the CPU (no GPU needed)."""
from __future__ import annotations

import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
ORACLE = os.path.join(REPO, "oracle")


def _build_and_run(src: str, tmp_path) -> str:
    subprocess.run(["make", "-s", "-C", ORACLE], check=True)
    exe = str(tmp_path / os.path.splitext(os.path.basename(src))[0])
    srcs = [os.path.join(ORACLE, f) for f in ("ora_field.c", "ora_secp.c", "ora_hash.c", "ora_bsgs.c", "ora_addr.c")]
    objs = []
    for s in srcs:
        o = str(tmp_path / (os.path.basename(s) + ".o"))
        subprocess.run(["gcc", "-O2", "-std=gnu11", "-c", s, "-o", o], check=True)
        objs.append(o)
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(HERE, "native", src), *objs, "-o", exe, "-lm",
                    "-lpthread"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_device_math_headers_on_host(tmp_path):
    out = _build_and_run("test_device_math_host.cpp", tmp_path)
    assert "FAIL" not in out


def test_hash160_header_on_host(tmp_path):
    out = _build_and_run("test_hash160_host.cpp", tmp_path)
    assert "ok" in out


def test_confirm_header_on_host(tmp_path):
    """device/confirm.hpp (khb_check's second/third check) vs the oracle's bsgs_secondcheck: planted keys,
    the AddDirect(P, -P) special case, random candidates, and every level-2/3 bloom bit set."""
    out = _build_and_run("test_confirm_host.cpp", tmp_path)
    assert out.strip().endswith("ok"), out
