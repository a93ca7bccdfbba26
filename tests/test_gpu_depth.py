"""GPU completeness at the product batch depth (keyhunt.cpp:3867-4004 run over a whole CLI batch).

The product launches the CLI's auto batch: about eight work items per lane of a full residency,
handed out dynamically per wave from a launch-wide counter (KHB_DYN).  The oracle-parity tests run
fewer jobs than lanes, so they never see a wave come back for its second item.  Here one batch of
that depth is searched through the product session with keys planted in the first job, a middle job
and the ragged last group of the last job, on a geometry whose groups per chunk (342) is not a
multiple of the 8 groups per item and whose item count is not a multiple of 64.  Every key must be
found, and the giant steps the device counted (count_walked) must equal jobs x cycles x 1024.
"""
from __future__ import annotations

import pytest

from keyhuntm1cpu_amd import khbsgs, khhost

pytestmark = pytest.mark.gpu

N_STR, KF = "0x10000000000", 3          # M = 3 * 2^20, aux = 349525, cycles = 342 (keyhunt.cpp:3810-3813)


def _auto_chunks(cycles: int, lanes: int, ntargets: int) -> int:
    """engine.cpp batch_chunks: ceil(8 * lanes / items per job) jobs, split over the targets."""
    per_job = -(-cycles // khbsgs.groups_per_item())
    jobs = -(-8 * lanes // per_job)
    return max(1, min(jobs // ntargets, 65536))


def _planted(base: int, m: int, a: int) -> int:
    """A key whose first giant-step hit in the chunk at `base` is step a: the key sits in the window
    [base + 2M a, base + 2M (a + 1)) that secondcheck rebuilds (keyhunt.cpp:4271-4296)."""
    return base + 2 * m * a + m // 2 + 17


def test_batch_depth_completeness():
    t = khhost.Tables(N_STR, KF, threads=16)
    assert t.cycles == 342 and t.m == 3 << 20
    lanes = khbsgs.default_lanes(0)
    assert lanes > 0
    nt = 3
    chunks = _auto_chunks(t.cycles, lanes, nt)
    per_job = -(-t.cycles // khbsgs.groups_per_item())
    n_items = chunks * nt * per_job
    assert n_items >= 8 * lanes - 64 * per_job * nt      # at least ~8 items per lane
    assert n_items % 64 != 0                             # the last wave's item block is ragged
    two_n = 2 * t.n_low
    start = 1 << 52
    bases = [start + c * two_n for c in range(chunks)]
    mid = chunks // 2
    last_a = t.cycles * 1024 - 1                         # last step of the ragged last group
    keys = [
        _planted(bases[0], t.m, 0),                      # first job, first giant step
        _planted(bases[mid], t.m, 1024 * 171 + 500),     # a middle job, a middle work item
        _planted(bases[-1], t.m, last_a),                # last job, ragged last item, last step
    ]
    # the last key lies beyond the last chunk's 2N keys (cycles * 1024 > aux), i.e. inside the next
    # chunk's range, which this batch does not claim: only the last group of the last job reaches it
    assert keys[2] >= bases[-1] + two_n
    targets = [khhost.pubkey(k) for k in keys]
    with khhost.Session(t, devices=[0]) as s:
        res, st = s.run(targets, start, start + (chunks + 8) * two_n, max_chunks=chunks)
    assert st["launches"] == 1 and st["chunks"] == chunks
    assert st["giant_steps"] == chunks * nt * t.cycles * 1024     # counted on the device
    assert res == keys
    t.close()


def test_device_step_count_matches_submission():
    """khb_collect reports the device-counted giant steps for ragged shapes (one job; a job count
    that leaves most lanes idle; a group range starting past group 0)."""
    from keyhuntm1cpu_amd.khbsgs import Engine
    t = khhost.Tables(N_STR, KF, threads=8)
    tgt = khhost.pubkey(0x1234567890ABCDEF)
    with Engine(0) as e:
        bf, nb, bits, h = t.bloom_concat(1)
        e.load_bloom(bf, nb, bits, h)
        e.load_giant_table(t.giant_table())
        offs, gpl = t.lane_offsets()
        e.load_lane_offsets(offs, gpl)
        for n_jobs, g0, gc in ((1, 0, 342), (37, 0, 342), (5, 8, 14), (3, 336, 6)):
            centres = b"".join(t.chunk_centre((1 << 50) + i * 2 * t.n_low, tgt) for i in range(n_jobs))
            _, _, st = e.scan(centres, g0, gc)
            assert st.giant_steps == n_jobs * gc * 1024
    t.close()


def test_two_queued_submissions_fifo(ora):
    """khb_submit twice before collecting (the context's two slots, one stream each): each collect
    returns its own submission's candidates in submission order, a third submission is refused with
    KHB_EBUSY while both are in flight, and the candidates equal the oracle's."""
    from keyhuntm1cpu_amd.khbsgs import Engine, KhbError
    t = khhost.Tables("0x100000000", 1, threads=8)
    o = ora.Bsgs("0x100000000", 1, 8)
    key = 0x2000000000123457
    tgt = ora.pubkey(key)
    batches = [[0x2000000000000000 + (3 * b + c) * (1 << 33) for c in range(3)] for b in range(3)]
    with Engine(0, lanes=16384) as e:
        bf, nb, bits, h = t.bloom_concat(1)
        e.load_bloom(bf, nb, bits, h)
        e.load_giant_table(t.giant_table())
        offs, gpl = t.lane_offsets()
        e.load_lane_offsets(offs, gpl)
        cent = [b"".join(t.chunk_centre(b, tgt.be64()) for b in bs) for bs in batches]
        e.submit(cent[0], 0, t.cycles)
        e.submit(cent[1], 0, t.cycles)
        with pytest.raises(KhbError, match="in flight"):
            e.submit(cent[2], 0, t.cycles)
        got = [e.collect()]
        e.submit(cent[2], 0, t.cycles)
        got += [e.collect(), e.collect()]
        with pytest.raises(KhbError, match="call order"):
            e.collect()
    for bs, (cands, degen, st) in zip(batches, got):
        assert st.giant_steps == 3 * t.cycles * 1024 and not degen
        for j, b in enumerate(bs):
            ref, _, _ = o.scan(o.chunk_start(b, tgt), 0, o.cycles)
            assert sorted(a for jj, a in cands if jj == j) == sorted(ref)
    assert [a for jj, a in got[0][0] if jj == 0]         # the key's chunk (batch 0, chunk 0) has a hit
    t.close()


def test_scan_refused_while_submission_pending():
    """khb_scan (submit + collect) with a submission in flight returns KHB_EBUSY instead of collecting
    the older submission's results as its own (the FIFO collect); after the pending one is collected it
    runs.  The launch intervals of khb_stats lie on the context's clock (khb_reset_epoch) in order."""
    from keyhuntm1cpu_amd.khbsgs import Engine, KhbError
    t = khhost.Tables("0x100000000", 1, threads=8)
    tgt = khhost.pubkey(0x2000000000123457)
    with Engine(0, lanes=16384) as e:
        bf, nb, bits, h = t.bloom_concat(1)
        e.load_bloom(bf, nb, bits, h)
        e.load_giant_table(t.giant_table())
        offs, gpl = t.lane_offsets()
        e.load_lane_offsets(offs, gpl)
        e.reserve_slots(2)
        e.reset_epoch()
        c0 = t.chunk_centre(0x2000000000000000, tgt)
        c1 = t.chunk_centre(0x2000000200000000, tgt)
        import ctypes as C
        from keyhuntm1cpu_amd.khbsgs import Cand, Stats
        buf, st = (Cand * 4096)(), Stats()
        e.submit(c0, 0, t.cycles)
        assert e.L.khb_scan(e.h, c1, 1, 0, t.cycles, buf, 4096, C.byref(st)) == -6      # KHB_EBUSY
        with pytest.raises(KhbError, match="in flight"):
            e.reset_epoch()
        cands0, _, st0 = e.collect()
        assert [a for _, a in cands0]                      # the key's chunk: its true hit
        assert e.L.khb_scan(e.h, c1, 1, 0, t.cycles, buf, 4096, C.byref(st)) == 0
        st1 = st
        assert st0.giant_steps == st1.giant_steps == t.cycles * 1024
        assert 0 <= st0.launch_begin_ms < st0.launch_end_ms <= st1.launch_begin_ms < st1.launch_end_ms
        assert abs((st0.launch_end_ms - st0.launch_begin_ms) - st0.kernel_ms) < 0.05
    t.close()


def _one_slot_lanes() -> int:
    """Lanes whose scratch (kBatch x 515 entries of 32 B per lane) takes 60 % of the device's HBM: one
    submission slot fits, a second cannot."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")                      # already loaded by libkhbsgs
    free, total = C.c_size_t(), C.c_size_t()
    assert hip.hipSetDevice(0) == 0 and hip.hipMemGetInfo(C.byref(free), C.byref(total)) == 0
    total = total.value
    per_lane = 32 * khbsgs.groups_per_item() * 515
    return int(0.6 * total / per_lane) // 256 * 256


def test_second_slot_enomem_leaves_one_slot_usable():
    """khb_reserve_slots on a context whose second slot does not fit returns KHB_ENOMEM and
    frees the partial slot; the context still scans with one submission in flight (the key's chunk
    gives its true hit)."""
    from keyhuntm1cpu_amd.khbsgs import Engine, KhbError
    t = khhost.Tables("0x100000000", 1, threads=8)
    tgt = khhost.pubkey(0x2000000000123457)
    try:
        with Engine(0, lanes=_one_slot_lanes()) as e:
            bf, nb, bits, h = t.bloom_concat(1)
            e.load_bloom(bf, nb, bits, h)
            e.load_giant_table(t.giant_table())
            offs, gpl = t.lane_offsets()
            e.load_lane_offsets(offs, gpl)
            with pytest.raises(KhbError, match="out of memory"):
                e.reserve_slots(2)
            e.reserve_slots(1)                      # slot 0 is intact
            cands, _, st = e.scan(t.chunk_centre(0x2000000000000000, tgt), 0, t.cycles)
            assert [a for _, a in cands] and st.giant_steps == t.cycles * 1024
    finally:
        t.close()


def test_engine_falls_back_to_depth_one():
    """the search engine asks for two slots; when the second does not fit it warns and runs
    one batch at a time instead of failing, and still finds every key."""
    import json
    import os
    gold = os.path.join(os.path.dirname(__file__), "golden", "puzzle_keys.json")
    with open(gold) as f:
        keys = json.load(f)
    ns = [26, 27, 28]
    t = khhost.Tables(hex(1 << 24), 1, threads=8)
    try:
        targets = [khhost.parse_pubkey(keys[str(n)]["pubkey"])[0] for n in ns]
        with khhost.Session(t, lanes=_one_slot_lanes(), chunks_per_batch=2) as s:
            res, st = s.run(targets, 1 << (ns[0] - 1), 1 << ns[-1])
        assert res == [int(keys[str(n)]["key"], 16) for n in ns]
        assert st["launches"] >= 3                   # [2^25, 2^28) is 7 chunks of 2N = 2^25: 4 batches
    finally:
        t.close()


def test_lazy_second_slot_under_a_full_residency_launch():
    """Round 5's host hand-over (launch epilogue, counters zeroed by the kernel): a small warm-up launch, then a
    full-residency launch on slot 0 with the second slot allocated while it runs.  The second slot's counters are
    zeroed on its own stream (a null-stream hipMemset queued behind the running launch zeroed them mid-launch
    and re-walked 6,144 groups: tools/debug/epilogue_diag.py).  Every collect has the submitted walked count, and
    the execution span (khb_stats.kernel_ms) is positive and no longer than the launch's events (event_ms)."""
    import ctypes as C
    from keyhuntm1cpu_amd.khbsgs import Engine, Cand, Degenerate, Stats
    t = khhost.Tables(None, 1, threads=16)
    tgt = khhost.pubkey(0x2832ED74F2B5E35EE)
    jobs = 512
    centres = b"".join(t.chunk_centre((1 << 65) + c * (1 << 45), tgt) for c in range(jobs))
    with Engine(0) as e:
        bf, nb, bits, h = t.bloom_concat(1)
        e.load_bloom(bf, nb, bits, h)
        gate, lg = t.gate()
        e.load_gate(gate, lg, t.gate_probes())
        e.load_giant_table(t.giant_table())
        offs, gpl = t.lane_offsets()
        e.load_lane_offsets(offs, gpl)
        e.scan(centres[:64 * 8], 0, 64)                 # warm-up: small, slot 0
        e.submit(centres, 0, t.cycles)                   # slot 0, full residency
        e.submit(centres, 0, t.cycles)                   # slot 1 allocated now, while slot 0 runs
        for _ in range(2):
            cand, deg, st = (Cand * 4096)(), (Degenerate * 4096)(), Stats()
            rc = e.L.khb_collect(e.h, cand, 4096, deg, 4096, C.byref(st))
            assert rc == 0 and st.giant_steps == jobs * t.cycles * 1024, (rc, st.giant_steps)
            assert 0 < st.kernel_ms and st.launch_end_ms - st.launch_begin_ms == pytest.approx(st.kernel_ms, abs=1e-3)
            assert 1000 < st.shader_mhz < 3000
            assert st.event_ms >= st.kernel_ms - 1e-3, (st.event_ms, st.kernel_ms)
    t.close()
