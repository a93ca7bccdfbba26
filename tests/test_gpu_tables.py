"""GPU baby-step table build (khb_build_baby; thread_bPload keyhunt.cpp:4404-4592): the three
bloom levels, the bPtable and the level-0 gate built on the GPU equal the host build byte for byte."""
from __future__ import annotations

import pytest

from keyhuntm1cpu_amd import khhost

pytestmark = pytest.mark.gpu


def _same(a, b):
    for lvl in (1, 2, 3):
        assert a.bloom_concat(lvl) == b.bloom_concat(lvl), lvl
    assert a.bptable() == b.bptable()
    assert a.giant_table() == b.giant_table()
    assert a.lane_offsets() == b.lane_offsets()
    assert a.gate() == b.gate() and a.gate()[1] >= 13 and a.gate_probes() == b.gate_probes() == 3


@pytest.mark.parametrize("n,k", [("0x40000000", 33),      # M = 33*2^15: L1 extent overshoot (quirk vi)
                                 (None, 1),                # default 2^44, k=1: 2^22 baby steps
                                 (None, 4)])               # config C: 2^24 baby steps
def test_gpu_build_equals_host_build(n, k):
    cpu = khhost.Tables(n, k, threads=16)
    gpu = khhost.Tables(n, k, threads=16, gpu_device=0)
    if n == "0x40000000":
        assert cpu.l1ext > cpu.m      # the overshoot is exercised
    _same(cpu, gpu)
    assert gpu.build_ms > 0
    cpu.close()
    gpu.close()
