#!/usr/bin/env python3
"""bench.py — BSGS giant-step throughput (BASELINE.json metric) on puzzle #66 or puzzle #130.

--workload p66 (default; BASELINE.json configs[1], -b 66, k=1; --k 4 = configs[2]):
  one step = one GPU scan batch of the product search (libkhhost -> libkhbsgs): host centres for
  4096 chunks, the HIP giant-step kernel over all 4096 groups of each chunk (2^34 giant steps:
  eight 8-group work items per lane of a full residency of 262,144 lanes at 4 waves/SIMD, as the CLI's
  auto batch), and the CPU confirmation
  of every candidate, pipelined exactly as the keyhunt_amd CLI runs it.  The -b 66 range [2^65, 2^66)
  is partitioned statically into one contiguous chunk block per rank (partition.key_block, north_star);
  the block holding puzzle #66's (public) key starts at the chunk after the key's, so the search never
  stops early and every rank times exactly K steps of sequential 2N-key chunks.  A rank whose W + K
  steps would run past its block (so past 2^66 for the last rank) is an error: the script exits non-zero
  before timing (at k=1 and the auto batch each rank's block holds 32 steps at N = 8, 64 at N = 4).
--workload p130 (BASELINE.json configs[3], -f tests/130.txt -b 130, k=1): the real #130 pubkey; the
  whole -b 130 range [2^129, 2^130) is partitioned statically into one contiguous chunk block per
  rank (partition.rank_range, north_star), and every rank scans (W + K) batches from its block start.
--workload address (BASELINE.json configs[4], -m address -f tests/unsolvedpuzzles.rmd, -l both): one step =
  8 chunks of 2^32 keys (one queued launch of ~8 work items per lane) through the product address search
  (SHA-256 + RIPEMD-160 kernels, bloom hits confirmed on the host); -b 71's range [2^70, 2^71) split
  into static rank blocks.  The line's metric is keys hashed and probed per second; use a small --steps
  (a step is ~8 s at -l both).

Tables are built and resident in HBM before the timed region.  Multi-GPU: one process per GPU
(torch.distributed.run); no data-path collective (gloo only times it).

Prints ONE JSON line (rank 0).  See DESIGN.md §5-§6 for the roofline definitions.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# Algorithmic work per giant step, counted in 32-bit multiply-class
# lane ops of the reference algorithm: per 1024-step group 2561 field mul (64 products + 8 fold) +
# 1023 field sqr (36 + 8) + one inversion (255 sqr + 15 mul), plus two XXH64 of 32 bytes (22 64-bit
# multiplies = 66 32-bit) and two 64-bit "% bits" (4 each).
MUL_OPS, SQR_OPS = 72, 44
INV_OPS = 255 * SQR_OPS + 15 * MUL_OPS
OPS_PER_STEP = (2561 * MUL_OPS + 1023 * SQR_OPS + INV_OPS) / 1024.0 + 2 * 66 + 2 * 4
# The multiply-class work this kernel executes per giant step: per group 511 forward
# prefix products + the walk's 2045 products and 1023 squarings (walk_group_g) + 9 products and one
# squaring of the work item's centre and chained-product bookkeeping (scan_batch), and two inversions
# per 8-group work item; no XXH64 / "% bits" for the 99.96 % of x the level-0 gate stops.  The half prefix
# stream (KHB_HALF_STREAM, the product since round 6) rebuilds every even prefix in the walk: 255 more
# products per group (walk_group_g_half: one per pair of walk steps but the last, plus the peeled step 511).
HALF_STREAM_MULS = 255
EXEC_OPS_PER_STEP_FULL = ((2556 + 9) * MUL_OPS + (1023 + 1) * SQR_OPS) / 1024.0 + 2 * INV_OPS / (8 * 1024.0)
EXEC_OPS_PER_STEP = EXEC_OPS_PER_STEP_FULL + HALF_STREAM_MULS * MUL_OPS / 1024.0


def exec_ops_per_step(build: dict) -> float:
    """Executed multiply-class ops per giant step of the loaded build (khb_build_info's half_stream)."""
    return EXEC_OPS_PER_STEP if build.get("half_stream", "1") == "1" else EXEC_OPS_PER_STEP_FULL
# Peak of the binding unit: v_mad_u64_u32 issue rate measured on MI355X by tools/microbench/intops2.hip
# at full occupancy, 57.8 lane-ops/clk/CU at the 2.16 GHz the microbenchmark ran at
# (profiles/r01_intops2.txt); the same rate at the 2.4 GHz peak engine clock is 35.5 T.
# The headline peak uses the guide's 2.4 GHz peak engine clock (MI355X_MICROARCH.md): 35.51 T; the same
# rate at the microbenchmark's 2.16 GHz (32.04 T) and at the launches' own measured shader clock are
# reported beside it.
PEAK_LANES_PER_CLK_CU, CUS = 57.8, 256
PEAK_CLK_GHZ, MICROBENCH_CLK_GHZ = 2.4, 2.16


def pmc_traffic(pmc: dict, chunks: int, launch_steps: int) -> dict:
    """roofline.traffic for one launch of `chunks` chunks from profiles/pmc_latest.json: its measured bytes
    when the PMC launch had the same size, else its bytes per giant step scaled to this launch (noted)."""
    if pmc.get("chunks_per_launch") == chunks:
        return {"traffic": pmc.get("hbm_bytes_per_launch")}
    return {"traffic": int(round(pmc["bytes_per_giant_step"] * launch_steps)),
            "traffic_note": "PMC bytes per giant step measured at %d chunks per launch, scaled to %d"
                            % (pmc["chunks_per_launch"], chunks)}


def pmc_mismatch(pmc: dict, run_cfg: dict) -> str | None:
    """None when profiles/pmc_latest.json was measured on this run's kernel configuration (k, level-0 gate, lanes,
    waves per SIMD; a key the record lacks counts as a mismatch), else the note the line carries instead of the
    traffic and VALU figures (a --no-gate or other-build run must not borrow them)."""
    mism = {key: (pmc.get(key), v) for key, v in run_cfg.items() if pmc.get(key) != v}
    if not mism:
        return None
    return ("profiles/pmc_latest.json was measured for another configuration (%s); traffic not measured for this run"
            % ", ".join("%s %s vs %s" % (k, a, b) for k, (a, b) in mism.items()))


def mulops_peak_t(ghz: float) -> float:
    return round(PEAK_LANES_PER_CLK_CU * CUS * ghz * 1e9 / 1e12, 2)


PEAK_MULOPS_T = mulops_peak_t(PEAK_CLK_GHZ)                   # 35.51
PEAK_MULOPS_T_2P16 = mulops_peak_t(MICROBENCH_CLK_GHZ)        # 32.04
HBM_PEAK_GBS = 8000.0
BSGSD_CPU_MKEYS = 16.9     # the reference's own published BSGS rate (BSGSD.md:52-58, 8 threads)

PUZZLE66_KEY = 0x2832ED74F2B5E35EE            # public solution; pinned to tests/66.rmd below
PUZZLE66_HASH160 = "20d45a6a762535700ce9e0b216e31994335db8a5"   # tests/66.rmd


def puzzle66_target():
    from keyhuntm1cpu_amd import khhost
    from keyhuntm1cpu_amd.hash160 import compressed_pubkey, hash160
    xy = khhost.pubkey(PUZZLE66_KEY)
    if hash160(compressed_pubkey(xy)).hex() != PUZZLE66_HASH160:
        raise SystemExit("puzzle #66 key does not match tests/66.rmd")
    return xy


def puzzle130_target():
    """tests/130.txt of the reference (the committed fixture tests/golden/puzzle_targets.json)."""
    from keyhuntm1cpu_amd import khhost
    with open(os.path.join(REPO, "tests", "golden", "puzzle_targets.json")) as f:
        line = json.load(f)["130.txt"][0]
    xy, _ = khhost.parse_pubkey(line)
    return xy, line


def host_cores():
    """Cores this job may use: the affinity set, capped by a cgroup v2 CPU quota and by the job's CPU
    share when the environment states one (OMP_NUM_THREADS: a one-GPU box gives each job 16 of its
    host's cores, while nproc shows the whole machine); plus nproc and the CPU model for the report."""
    n = len(os.sched_getaffinity(0))
    caps = {"affinity": n, "nproc": os.cpu_count()}
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        if q != "max":
            caps["cgroup_quota"] = max(1, int(q) // int(per))
    except (OSError, ValueError):
        pass
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        caps["job_share"] = int(os.environ["OMP_NUM_THREADS"])
    cores = min(v for k, v in caps.items() if k != "nproc" and v)
    try:
        with open("/proc/cpuinfo") as f:
            caps["cpu_model"] = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), None)
    except OSError:
        pass
    return cores, caps


def cpu_baseline(seconds: float, threads: int, target, base: int):
    """Oracle (plain-C restatement of thread_process_bsgs) on the host cores, same workload."""
    from oracle import ora
    bs = ora.Bsgs(None, 1, threads)
    steps, el = bs.bench(target, base, threads, seconds)
    bs.close()
    return steps / el


def power_sampler(torch, local: int, args):
    """Board power / clock sampler over the timed region (keyhuntm1cpu_amd/power.py; amdsmi, not HIP)."""
    from keyhuntm1cpu_amd.power import PowerSampler
    if args.no_power:
        return PowerSampler.disabled("--no-power")
    bdf = physical_gpu(torch, local)                   # "dddd:bb:dd" (full domain:bus:device)
    return PowerSampler(None if bdf.startswith("device") else bdf)


def physical_gpu(torch, local: int) -> str:
    """The PCI address of this rank's GPU (ranks on the same physical GPU report the same string)."""
    try:
        p = torch.cuda.get_device_properties(local)
        return "%04x:%02x:%02x" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
    except Exception:                                  # noqa: BLE001
        return "device%d" % local


PRODUCT_LIB_DIR = os.path.join(REPO, "keyhuntm1cpu_amd", "lib")


def check_lib_dir(args):
    """A line must name the kernel that produced it: KHB_LIB_DIR redirects the libraries to
    another build (tools/gpu/bench_ab.sh), which is refused unless --variant names it.  Checked before any rank is
    started or the GPU is touched."""
    d = os.environ.get("KHB_LIB_DIR")
    if d and os.path.realpath(d) != os.path.realpath(PRODUCT_LIB_DIR) and not args.variant:
        raise SystemExit(f"[bench] KHB_LIB_DIR={d} loads a library other than the in-tree product build; pass "
                         f"--variant NAME for an A/B run of a timing build (the line is then marked with it)")


def lib_record(args) -> dict:
    """config.lib: the loaded libkhbsgs.so (path, sha256 prefix, khb_build_info's words) and libkhhost.so.  A build
    whose khb_build_info says it is not the product is refused without --variant; with --variant the names must
    agree."""
    import hashlib
    from keyhuntm1cpu_amd import khbsgs, khhost
    info = khbsgs.build_info()
    built_as = info.get("variant", "unknown")
    if args.variant is None and built_as != "product":
        raise SystemExit(f"[bench] {info['path']} was built as variant {built_as!r}, not the product: pass --variant")
    if args.variant is not None and built_as not in (args.variant, "unknown"):
        raise SystemExit(f"[bench] --variant {args.variant} but {info['path']} was built as {built_as!r}")
    host_path = os.path.realpath(khhost.LIB_PATH)
    with open(host_path, "rb") as f:
        host_sha = hashlib.sha256(f.read()).hexdigest()[:16]
    rel = lambda p: os.path.relpath(p, REPO) if p.startswith(REPO + os.sep) else p   # noqa: E731
    return {"lib_sha16": info["sha16"], "lib_path": rel(info["path"]), "host_lib_sha16": host_sha,
            "host_lib_path": rel(host_path), "build": {k: v for k, v in info.items() if k not in ("sha16", "path")}}


def init_gloo(dist, rank: int, world: int):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    # gloo's C++ connect messages go to fd 1; keep stdout for the one JSON line (rank 0)
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dist.barrier()
    finally:
        os.dup2(saved, 1)
        os.close(saved)


def launch_check(args, world: int, rank: int, local: int):
    """--launch-check: the rank layout only (no GPU).  Rank 0 prints every rank's (rank, local, pid)."""
    if args.launch_check_fail == rank:
        raise SystemExit(3)
    import torch.distributed as dist
    view = {"rank": rank, "local_rank": local, "world": world, "pid": os.getpid()}
    views = [view]
    if world > 1:
        init_gloo(dist, rank, world)
        views = [None] * world
        dist.all_gather_object(views, view)
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "ranks": views}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", choices=("p66", "p130", "address"), default="p66",
                    help="p66: BASELINE configs[1] (-b 66; --k 4 = configs[2]); p130: configs[3] (-b 130); "
                         "address: configs[4] (-m address unsolvedpuzzles.rmd, -l both)")
    ap.add_argument("--search", type=int, default=2, help="--workload address: -l 0 uncompress, 1 compress, 2 both")
    ap.add_argument("--endo", action="store_true",
                    help="--workload address: -e (endomorphism: beta*x, beta^2*x and negated points, keyhunt.cpp:2646-2763)")
    # default: >= 30 s of steady state — 100 steps x 2^34 giant steps at ~360 ms
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--chunks", type=int, default=0,
                    help="chunks (2N keys each) per step; default: the chunks that give every lane of the device "
                         "eight work items (4096 at k=1, 16384 at k=4), as the CLI's auto batch does "
                         "(engine.cpp batch_chunks)")
    ap.add_argument("--k", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=20.0,
                    help="CPU-baseline window after the table build (default 3 windows of 20 s: SURVEY.md section 8d's "
                         "60 s, with the spread between windows)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-windows", type=int, default=3,
                    help="repeat the CPU-baseline window this many times and report the mean and spread")
    ap.add_argument("--no-power", action="store_true", help="do not sample board power during the timed region")
    ap.add_argument("--share-gpus", action="store_true",
                    help="allow more ranks than visible GPUs (a multi-rank rehearsal: ranks share GPUs round-robin "
                         "and the line says so in config.physical_gpus / gpus_shared); refused otherwise")
    ap.add_argument("--no-gate", action="store_true",
                    help="no level-0 gate: every giant step probes the level-1 bloom (the reference's exact candidate "
                         "stream, ~1e-6 false positives per step); not the headline configuration")
    ap.add_argument("--check", choices=("host", "gpu", "auto"), default="host",
                    help="where candidates are confirmed (bsgs_secondcheck): the host pool (default), the GPU "
                         "(khb_check) or auto (the GPU for batches of more than 4096 candidates)")
    # launcher self-test (tests/test_launch.py): every rank joins the gloo world and rank 0 prints the
    # ranks' view; no GPU is touched.  --launch-check-fail R makes rank R exit with status 3.
    ap.add_argument("--variant", default=None,
                    help="an A/B run of the timing build named NAME in KHB_LIB_DIR: required whenever KHB_LIB_DIR points "
                         "away from the in-tree keyhuntm1cpu_amd/lib, and the line is then marked \"variant\": NAME")
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--launch-check-fail", type=int, default=-1, help=argparse.SUPPRESS)
    args = ap.parse_args()
    check_lib_dir(args)
    if args.workload == "p130" and args.k != 1:
        raise SystemExit("--workload p130 is BASELINE configs[3]: k = 1")

    # --gpus N: one process per GPU.  Under a launcher (WORLD_SIZE set) this process is one rank and
    # WORLD_SIZE must equal N; run bare with N > 1, the ranks are started here as child processes before
    # anything touches the GPU (keyhuntm1cpu_amd/launch.py), and this process only forwards rank 0's line.
    from keyhuntm1cpu_amd import launch
    # rank 0 runs the CPU baseline alone after the other ranks return (only at N = 1, but the budget is passed anyway)
    cpu_budget = 0.0 if args.no_cpu_baseline else args.cpu_seconds * max(1, args.cpu_windows) + 120.0
    launch.main_or_spawn(args.gpus, sys.argv[1:], os.path.abspath(__file__), rank0_extra_s=cpu_budget)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_check:
        return launch_check(args, world, rank, local)
    import torch                                   # first: share torch's HIP runtime with our libraries
    import torch.distributed as dist
    ndev = torch.cuda.device_count()
    if ndev and local >= ndev:
        # fewer visible GPUs than this LOCAL_RANK: either a launcher that shows each rank its own GPU only
        # (then device 0 is this rank's), or more ranks than GPUs (a rehearsal) -- told apart below
        local = local % ndev
    torch.cuda.set_device(local)
    gpu_id = physical_gpu(torch, local)
    ids = [gpu_id]
    if world > 1:
        init_gloo(dist, rank, world)
        ids = [None] * world
        dist.all_gather_object(ids, gpu_id)
    physical = len(set(ids))
    gpu_info = {"physical_gpus": physical, "gpus_shared": physical < world}
    if physical < world:
        # a line from ranks sharing GPUs would read as an N-GPU measurement: refuse unless asked
        msg = (f"[bench] {world} ranks on {physical} physical GPU(s) (PCI {sorted(set(ids))})")
        if not args.share_gpus:
            if world > 1:
                dist.destroy_process_group()
            raise SystemExit(msg + "; pass --share-gpus for a multi-rank rehearsal on fewer GPUs")
        print(msg + ": a rehearsal (--share-gpus); the line says gpus_shared", file=sys.stderr, flush=True)

    from keyhuntm1cpu_amd import khhost
    from keyhuntm1cpu_amd.partition import blocks_fit, fit_batch, rank_range
    host_threads = min(16, os.cpu_count() or 1)
    lib_rec = lib_record(args)
    if args.workload == "address":
        return bench_address(args, world, rank, dist, torch, lib_rec)
    t0 = time.time()
    tables = khhost.Tables(None, args.k, threads=host_threads, gpl=4)
    t_build = time.time() - t0
    auto_chunks = not args.chunks
    from keyhuntm1cpu_amd import khbsgs
    # chunks that give every lane of the device one work item
    fill = -(-khbsgs.default_lanes(local) * khbsgs.groups_per_item() // tables.cycles)
    if auto_chunks:
        # eight work items per lane, as the CLI's auto batch (engine.cpp batch_chunks): waves take
        # items dynamically (KHB_DYN), so a deeper queue keeps every SIMD 4 waves deep until the
        # launch's last items (profiles/r01c_dyn_probe.txt)
        args.chunks = max(1, (1 << 30) // (tables.cycles * 1024), 8 * fill)
    two_n = 2 * (tables.n_low)                     # 2N keys per chunk
    per_rank = (args.warmup + args.steps) * args.chunks
    chunks_note = None
    if args.workload == "p66":
        target = puzzle66_target()
        lo, hi = 1 << 65, 1 << 66
        blocks = blocks_fit(lo, hi, two_n, world, per_rank, PUZZLE66_KEY)
        bad = [r for r, (_, _, ok) in enumerate(blocks) if not ok]
        if bad and auto_chunks:
            # -b 66 holds 2^20 chunks of 2^45 keys: split N ways, a long run (many --steps) at the auto
            # batch would leave some rank's block.  Shrink the batch to whole work items per lane so that
            # every rank's W + K steps stay inside its block (at least one item per lane), else refuse.
            shrunk = fit_batch(lo, hi, two_n, world, args.warmup + args.steps, args.chunks, fill, PUZZLE66_KEY)
            if shrunk:
                chunks_note = ("auto batch %d chunks per step shrunk to %d (%d work items per lane) so that %d "
                               "steps fit every rank's -b 66 block" % (args.chunks, shrunk, shrunk // fill,
                                                                      args.warmup + args.steps))
                print("[bench] " + chunks_note, file=sys.stderr, flush=True)
                args.chunks = shrunk
                per_rank = (args.warmup + args.steps) * args.chunks
                blocks = blocks_fit(lo, hi, two_n, world, per_rank, PUZZLE66_KEY)
                bad = [r for r, (_, _, ok) in enumerate(blocks) if not ok]
        if bad:
            s0, e0, _ = blocks[bad[0]]
            raise SystemExit("[bench] -b 66 split %d ways: rank %d's block holds %d steps of %d chunks, %d requested "
                             "(warmup + steps); lower --steps/--warmup/--chunks" %
                             (world, bad[0], (e0 - s0) // (args.chunks * two_n), args.chunks, args.warmup + args.steps))
        start, end, _ = blocks[rank]
        cfg_idx = {1: "1", 4: "2"}.get(args.k, "1, k varied")
        workload = "puzzle66 -m bsgs -b 66 -k %d (BASELINE configs[%s])" % (args.k, cfg_idx)
        data = ("real puzzle #66 pubkey (solved key, hash160 == tests/66.rmd), -b 66 range [2^65, 2^66) split into %d "
                "static contiguous chunk blocks, one per rank; each rank scans sequential chunks from its block start "
                "(the key's block from the chunk after the key's); every rank's chunks inside -b 66" % world)
        cpu_base = 1 << 65
    else:
        target, line = puzzle130_target()
        lo, hi = 1 << 129, 1 << 130
        start, end = rank_range(lo, hi, two_n, rank, world)      # the rank's static block of -b 130
        if end - start < per_rank * two_n:
            raise SystemExit("-b 130 block too small for the requested steps")
        workload = "puzzle130 -m bsgs -f tests/130.txt -b 130 -k 1 (BASELINE configs[3])"
        data = ("real puzzle #130 pubkey (tests/130.txt: %s...), -b 130 range [2^129, 2^130) split into %d static "
                "contiguous chunk blocks, one per rank; each rank scans sequential chunks from its block start"
                % (line[:16], world))
        cpu_base = lo
    sess = khhost.Session(tables, devices=[local], chunks_per_batch=args.chunks, check_threads=host_threads)
    if args.no_gate:
        sess.set_test_hooks(use_gate=False)
    sess.set_check_mode({"host": khhost.CHECK_HOST, "gpu": khhost.CHECK_DEVICE, "auto": khhost.CHECK_AUTO}[args.check])

    def sync():
        torch.cuda.synchronize()

    # warmup (untimed)
    if args.warmup:
        sess.run([target], start, end, max_chunks=args.warmup * args.chunks)
    tstart = start + args.warmup * args.chunks * two_n
    sampler = power_sampler(torch, local, args)
    if world > 1:
        dist.barrier()
    sync()
    with sampler:
        t0 = time.perf_counter()
        res, st = sess.run([target], tstart, end, max_chunks=args.steps * args.chunks)
        sync()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
    sess.close()
    steps_done = st["giant_steps"]               # counted on the device (khb_collect, count_walked)
    psum = sampler.summary(work_units=steps_done, seconds=dt)
    lanes = khbsgs.default_lanes(local)
    waves = lanes // (torch.cuda.get_device_properties(local).multi_processor_count * 4 * 64)
    per_launch_steps = args.chunks * tables.cycles * 1024
    kernel_ms = 1e3 * st["kernel_s"] / max(1, st["launches"])
    event_ms = 1e3 * st["event_s"] / max(1, st["launches"])     # dispatch to end, as rocprofv3's trace
    # device-busy time per step: the union of this rank's launch intervals (HIP events on each launch's
    # stream, khb_stats.launch_begin_ms/end_ms) over the timed region, per step
    busy_ms = 1e3 * st["busy_s"] / args.steps
    bad_count = 0.0 if steps_done == args.steps * per_launch_steps and st["rescans"] == 0 else 1.0
    tot_steps, tmax, kmax, bmax, bad = steps_done, dt, kernel_ms, busy_ms, bad_count
    if world > 1:
        v = torch.tensor([float(steps_done), dt, kernel_ms, busy_ms, bad_count, event_ms], dtype=torch.float64)
        s = v.clone()
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        m = v.clone()
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        tot_steps, tmax, kmax, bmax, bad = s[0].item(), m[1].item(), m[2].item(), m[3].item(), m[4].item()
        event_ms = m[5].item()
    if bad or tot_steps != world * args.steps * per_launch_steps:
        # a line over an incomplete or repeated count is never printed (every rank exits non-zero)
        print(f"[bench] ERROR: the device counted {tot_steps:.0f} giant steps over the ranks, "
              f"{world * args.steps * per_launch_steps} submitted (or a launch was rescanned)", file=sys.stderr, flush=True)
        if world > 1:
            dist.destroy_process_group()
        raise SystemExit(3)

    ranges = [(start, end)]
    if world > 1:
        ranges = [None] * world
        dist.all_gather_object(ranges, (start, end))
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    if not all(lo <= s0 < e0 <= hi for s0, e0 in ranges):
        print(f"[bench] ERROR: a rank's block leaves [{hex(lo)}, {hex(hi)})", file=sys.stderr, flush=True)
        raise SystemExit(3)
    gsps = tot_steps / tmax
    wall_ms = 1e3 * tmax / args.steps
    if bmax > wall_ms * 1.0005:
        print(f"[bench] ERROR: device-busy {bmax:.3f} ms per step exceeds the wall time {wall_ms:.3f} ms",
              file=sys.stderr, flush=True)
        raise SystemExit(3)
    time_basis = ("kernel_busy_ms_per_step: union of the k_giant_scan launch intervals over the timed steps / steps "
                  "(each launch's execution span on the device's 100 MHz clock, ending at its end event on the "
                  "launch's stream); <= ms_per_step")
    if bmax <= 0:    # no launch interval was timed (events unavailable): fall back to the wall time
        bmax = wall_ms
        time_basis = "ms_per_step (the launches' event intervals were unavailable)"
    achieved = OPS_PER_STEP * per_launch_steps / (bmax * 1e-3) / 1e12
    achieved_launch = OPS_PER_STEP * per_launch_steps / (max(kmax, 1e-9) * 1e-3) / 1e12
    exec_ops = exec_ops_per_step(lib_rec["build"])
    executed = exec_ops * per_launch_steps / (bmax * 1e-3) / 1e12
    mhz = st["shader_mhz"]
    peak_at_clock = PEAK_LANES_PER_CLK_CU * CUS * mhz * 1e6 / 1e12 if mhz > 0 else None
    roofline = {"bound": "valu", "unit": "Tops/s", "achieved": round(achieved, 3), "peak": PEAK_MULOPS_T,
                "frac": round(achieved / PEAK_MULOPS_T, 4), "traffic": None,
                "ops": "32-bit multiply-class lane ops of the reference algorithm (v_mad_u64_u32 / v_mul_lo_u32)",
                "ops_per_giant_step": round(OPS_PER_STEP, 2), "kernel": "k_giant_scan",
                "per": "one GPU (the slowest rank's busy time when n_gpus > 1)",
                "time_basis": time_basis,
                "kernel_busy_ms_per_step": round(bmax, 3),
                "shader_mhz_avg": round(mhz, 1),
                "kernel_ms_avg": round(kmax, 3),
                "kernel_event_ms_avg": round(event_ms, 3),
                "kernel_ms_basis": "kernel_ms_avg: a launch's execution span (its first workgroup's start to its "
                                   "last wave's exit); kernel_event_ms_avg: its HIP events, dispatch to end, the "
                                   "duration rocprofv3 --kernel-trace reports, which with two launches in flight "
                                   "includes the wait behind the other slot's launch (DESIGN.md §5)",
                "achieved_per_launch": round(achieved_launch, 3),
                "frac_per_launch": round(achieved_launch / PEAK_MULOPS_T, 4),
                "peak_basis": "v_mad_u64_u32 %.1f lane-ops/clk/CU (profiles/r01_intops2.txt) x %d CUs at the %.1f GHz "
                              "peak engine clock (MI355X_MICROARCH.md)" % (PEAK_LANES_PER_CLK_CU, CUS, PEAK_CLK_GHZ),
                "peak_at_2p16ghz": PEAK_MULOPS_T_2P16,
                "frac_at_2p16ghz": round(achieved / PEAK_MULOPS_T_2P16, 4),
                "peak_at_shader_clock": round(peak_at_clock, 3) if peak_at_clock else None,
                "frac_at_shader_clock": round(achieved / peak_at_clock, 4) if peak_at_clock else None}
    executed_info = {"ops_per_giant_step": round(exec_ops, 2),
                     "note": "multiply-class work the kernel performs: the reference's field work without the "
                             "3 of 4 inversions the 8-group batch saves and without the two XXH64 the level-0 "
                             "gate skips for 99.96 % of x, plus the half prefix stream's 255 products per group",
                     "achieved": round(executed, 3), "frac": round(executed / PEAK_MULOPS_T, 4),
                     "frac_at_2p16ghz": round(executed / PEAK_MULOPS_T_2P16, 4)}
    # the PMC record of this run's k: profiles/pmc_latest.json (k = 1, configs B and D) or pmc_latest_k4.json (C)
    pmc_path = os.path.join(REPO, "profiles", "pmc_latest.json" if args.k == 1 else "pmc_latest_k%d.json" % args.k)
    if not os.path.exists(pmc_path):
        roofline["traffic_note"] = "no PMC record for k = %d (%s)" % (args.k, os.path.relpath(pmc_path, REPO))
    else:
        try:
            with open(pmc_path) as f:
                pmc = json.load(f)
            # the PMC record applies only to the kernel it was measured on
            build = lib_rec["build"]
            note = pmc_mismatch(pmc, {"k": args.k, "level0_gate": not args.no_gate, "lanes": lanes,
                                      "waves_per_simd": waves,
                                      "kernel_build": {k: build.get(k) for k in ("variant", "half_stream", "batch",
                                                                                 "waves_per_simd", "gate1", "gate0")}})
            if note:
                roofline["traffic_note"] = note
            else:
                roofline.update(pmc_traffic(pmc, args.chunks, per_launch_steps))
                roofline["traffic_source"] = os.path.relpath(pmc_path, REPO)
                if pmc.get("valu_instr_per_giant_step"):
                    vi = pmc["valu_instr_per_giant_step"]
                    executed_info.update({
                        "valu_lane_instr_per_giant_step": vi,
                        "valu_busy_pct": pmc.get("valu_util_pct"),
                        "valu_busy_basis": pmc.get("valu_util_basis"),
                        "valu_busy_4cycle_model_pct": pmc.get("valu_busy_pct"),
                        "valu_lane_instr_T_per_s": round(vi * per_launch_steps / (bmax * 1e-3) / 1e12, 2),
                        "vop3_issue_ceiling": "58-61 lane-instr/clk/CU = %.1f-%.1f T at 2.4 GHz (intops2)"
                                              % (58 * CUS * 2.4e-3, 61 * CUS * 2.4e-3),
                        "pmc_source": pmc.get("valu_source")})
        except (OSError, ValueError):
            pass
    roofline["executed"] = executed_info
    roofline["power"] = psum
    # Two launches overlap (the context's two submission slots): a launch's event time
    # includes the tail it shares with its neighbour (kernel_ms_avg > ms_per_step), so `achieved` /
    # `frac` use the device-busy time per step; the per-launch and wall figures are beside them.
    roofline["achieved_wall"] = round(OPS_PER_STEP * per_launch_steps / (wall_ms * 1e-3) / 1e12, 3)
    roofline["frac_wall"] = round(roofline["achieved_wall"] / PEAK_MULOPS_T, 4)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        c_threads, hinfo = host_cores()
        from oracle import ora                     # the checker-side restatement, timed only here
        cpu_pt = ora.pubkey(PUZZLE66_KEY) if args.workload == "p66" else ora.parse_pubkey(line)[0]
        vs = [cpu_baseline(args.cpu_seconds, c_threads, cpu_pt, cpu_base + w * (1 << 56))
              for w in range(max(1, args.cpu_windows))]
        v = sum(vs) / len(vs)
        cpu = {"value": round(v / 1e6, 4), "unit": "Mkeys/s", "cores": c_threads, "kind": "port",
               "sample": f"oracle thread_process_bsgs restatement (k=1, default -n), same target, chunks from "
                         f"{hex(cpu_base)}, {len(vs)} x {args.cpu_seconds:.0f} s window(s) on {c_threads} threads "
                         f"(every core this job may use: host below) after the table build",
               "window_s": args.cpu_seconds, "windows_mkeys": [round(x / 1e6, 3) for x in vs],
               "spread_pct": round(100.0 * (max(vs) - min(vs)) / v, 2) if len(vs) > 1 else None,
               "host": hinfo,
               "reference_published": {"value": BSGSD_CPU_MKEYS, "unit": "M giant-steps/s",
                                       "source": "BSGSD.md:52-58 (bsgsd -k 4096 -t 8, unnamed 64 GB server)"}}
    out = {
        "metric": "Mkeys/s (BSGS giant-steps/s) on puzzle #66 at 1/2/4/8 MI355X",
        "value": round(gsps / 1e6, 2),
        "unit": "Mkeys/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * tmax / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": data,
        "config": {"workload": workload,
                   "n": hex(tables.n_low), "bsgs_m": tables.m, "groups_per_chunk": tables.cycles,
                   "chunks_per_step": args.chunks, "giant_steps_per_step": per_launch_steps,
                   "parallelism": "range-partition x%d" % world, "table_build_s": round(t_build, 2),
                   **gpu_info,
                   "rank0_range": [hex(start), hex(end)],
                   "rank_ranges": [[hex(a), hex(b)] for a, b in ranges],
                   "timed_ranges": [[hex(a + args.warmup * args.chunks * two_n),
                                     hex(a + (args.warmup + args.steps) * args.chunks * two_n)] for a, _ in ranges],
                   "launcher": ("bench.py child ranks" if os.environ.get("KHB_BENCH_CHILD") else
                                "external (WORLD_SIZE set)") if world > 1 else "none",
                   "batch_note": chunks_note,
                   "ref_keys_per_s": "%.3e" % (gsps * 2 * tables.m),
                   "candidates": st["candidates"], "found": [hex(r) if r else None for r in res],
                   "level0_gate": not args.no_gate, "check": args.check,
                   "device_checked": st["device_checked"], "device_check_s": round(st["device_check_s"], 4),
                   **lib_rec},
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    if args.variant:
        out["variant"] = args.variant
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()



# -m address (configs[4]).  Executed VALU lane-instructions per key at -l both: PMC SQ_INSTS_VALU x 64 / keys
# of one 8-chunk launch (tools/addr_floor.py under rocprofv3; profiles/r04b/addr_libkhbsgs: 4.9695e12 x 64 /
# 2^35 = 9,256.1; round 2's profiles/r02w/addr_valu_counter_collection.csv read 9,253.4).  The
# issue ceiling is that of the kernel's own instruction mix: the hash blocks are 43 % full-rate VALU
# (v_add_u32, v_bitop3_b32, shifts: ~2.6 SIMD cycles per wave-instruction at 4 waves/SIMD) and 57 %
# half-rate (v_alignbit_b32, v_add3_u32, v_mad_u64_u32: ~4.6), profiles/r03_valu_cost.txt and
# tools/debug/bb_path.py over tools/microbench/hash_isa.hip = 3.73 cycles per wave-instruction.
ADDR_EXEC_VALU_PER_KEY = {2: 9256.1}
# With -e (-l both): SQ_INSTS_VALU x 64 / keys of a two-chunk launch of k_giant_scan<kAddrBE> (tools/addr_floor.py with
# SEARCH=6 under rocprofv3, profiles/r06h/addr_s6: 4.9495e12 x 64 / 2^33 = 36,877.0 per key; the plain kernel's
# count in the same call, 9,259.8, reproduces the value above).  Twelve hashes per key instead of three.
ADDR_EXEC_VALU_PER_KEY_ENDO = {2: 36877.0}
# The VALU floor per key of -l both, in the same unit: the hash blocks as compiled alone
# (tools/microbench/hash_isa.hip -> profiles/r02_hash_isa_counts.txt: the 02/03 compressed hash160 pair
# 4,401, the uncompressed hash160 3,616, XXH64 of three 20-byte hashes 3 x 137 / 2) plus the x/y walk,
# measured as PMC SQ_INSTS_VALU of the hash-less build of the same kernel (tools/experiments/addrwalk_patch.py;
# profiles/r04b/addr_libkhbsgs_addrwalk: 5.308e11 x 64 / 2^35 = 988.7 per key).
ADDR_FLOOR_TERMS = {2: {"hash160_compressed_pair": 4401, "hash160_uncompressed": 3616, "xxh64_x3": 205.5,
                        "xy_walk": 988.7}}
ADDR_MIX_CYCLES_PER_INSTR = 3.73
ADDR_ALG_OPS = {0: 2 * 2032 + 1440 + 680, 1: 2 * (2032 + 1440) + 530, 2: 4 * 2032 + 3 * 1440 + 680}


def addr_cpu_baseline(text: str, seconds: float, threads: int, search: int):
    """Oracle restatement of thread_process's group loop (ora_addr.c) on `threads` host threads."""
    import threading
    from oracle import ora
    A = ora.AddrTable(text)
    done = [0] * threads
    stop = time.perf_counter() + seconds

    def work(t):
        g = ora.AddrGen(1)
        key = (1 << 70) + t * (1 << 40)
        while time.perf_counter() < stop:
            g.group(A, key, search)
            key += 1024
            done[t] += 1024
        g.close()
    t0 = time.perf_counter()
    th = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    el = time.perf_counter() - t0
    A.close()
    return sum(done) / el


def bench_address(args, world, rank, dist, torch, lib_rec):
    from keyhuntm1cpu_amd import khhost
    from keyhuntm1cpu_amd.partition import rank_range
    n_seq, chunks = 1 << 32, args.chunks or 8
    with open(os.path.join(REPO, "tests", "golden", "address", "unsolvedpuzzles.rmd")) as f:
        text = f.read()
    t0 = time.time()
    A = khhost.Addr(text, n_seq=n_seq, threads=min(16, os.cpu_count() or 1))
    t_build = time.time() - t0
    lo, hi = 1 << 70, 1 << 71
    start, end = rank_range(lo, hi, n_seq, rank, world)
    per_rank = (args.warmup + args.steps) * chunks
    if start + per_rank * n_seq > end:
        raise SystemExit("[bench] -b 71 block too small for the requested steps")
    search = args.search | (4 if args.endo else 0)          # KHB_SEARCH_ENDOMORPHISM
    if args.warmup:
        A.search(start, start + args.warmup * chunks * n_seq, search=search)
    tstart = start + args.warmup * chunks * n_seq
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    found, st = A.search(tstart, tstart + args.steps * chunks * n_seq, search=search)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    keys = st["keys"]
    bad = 0.0 if keys == args.steps * chunks * n_seq else 1.0
    tot, tmax, mhz = float(keys), dt, st["shader_mhz"]
    if world > 1:
        v = torch.tensor([float(keys), dt, bad, mhz], dtype=torch.float64)
        s, m = v.clone(), v.clone()
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        tot, tmax, bad, mhz = s[0].item(), m[1].item(), m[2].item(), s[3].item() / world
    if bad:
        print(f"[bench] ERROR: the device counted {tot:.0f} keys, {world * args.steps * chunks * n_seq} submitted",
              file=sys.stderr, flush=True)
        if world > 1:
            dist.destroy_process_group()
        raise SystemExit(3)
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    rate = tot / tmax
    per_gpu = rate / world
    roofline = {"bound": "valu", "unit": "T lane-instr/s", "kernel": "k_giant_scan<address>",
                "time_basis": "wall time of the timed steps (two launches in flight, as the CLI runs them)",
                "shader_mhz_avg": round(mhz, 1)}
    e = (ADDR_EXEC_VALU_PER_KEY_ENDO if args.endo else ADDR_EXEC_VALU_PER_KEY).get(args.search)
    if e and mhz > 0:
        peak = CUS * 4 * 64 / ADDR_MIX_CYCLES_PER_INSTR * mhz * 1e6 / 1e12
        ach = e * per_gpu / 1e12
        roofline.update({"achieved": round(ach, 3), "peak": round(peak, 3), "frac": round(ach / peak, 4),
                         "valu_lane_instr_per_key": e,
                         "peak_basis": "the hash mix's issue ceiling, %.2f SIMD cycles per wave-instruction (43 %% "
                                       "full-rate / 57 %% half-rate VALU, profiles/r03_valu_cost.txt) x 1024 SIMDs at "
                                       "the launches' measured shader clock" % ADDR_MIX_CYCLES_PER_INSTR,
                         "executed_source": ("profiles/r06h/addr_s6" if args.endo else "profiles/r04b/addr_libkhbsgs")
                                            + " (PMC SQ_INSTS_VALU, tools/addr_floor.py)"})
        fl = None if args.endo else ADDR_FLOOR_TERMS.get(args.search)
        if fl:
            floor = sum(fl.values())
            roofline.update({"floor_valu_lane_instr_per_key": round(floor, 1), "floor_terms": fl,
                             "executed_over_floor": round(e / floor, 4),
                             "floor_basis": "hash blocks compiled alone (profiles/r02_hash_isa_counts.txt) + the x/y "
                                            "walk's PMC count in the hash-less build (profiles/r04b)"})
    if not args.endo:
        roofline["algorithmic_ops_per_key"] = ADDR_ALG_OPS[args.search]
    elif e is None:
        roofline["note"] = "-e: no PMC instruction count measured for this -l mode's endomorphism kernel; frac not computed"
    roofline["traffic"] = None
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        c_threads, hinfo = host_cores()
        v = addr_cpu_baseline(text, args.cpu_seconds, c_threads, search)
        cpu = {"value": round(v / 1e6, 4), "unit": "Mkeys/s", "cores": c_threads, "kind": "port",
               "sample": f"oracle ora_addr_group (thread_process group loop restatement, -l "
                         f"{['uncompress', 'compress', 'both'][args.search]}{' -e' if args.endo else ''}), keys from 2^70, "
                         f"{args.cpu_seconds:.0f} s "
                         f"on {c_threads} threads", "host": hinfo}
    out = {
        "metric": "Mkeys/s (-m address: keys hashed and bloom-probed per second) on 1/2/4/8 MI355X",
        "value": round(rate / 1e6, 2), "unit": "Mkeys/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1e3 * tmax / args.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "real target file tests/unsolvedpuzzles.rmd (the reference's, committed as a fixture), -b 71 range "
                "[2^70, 2^71) split into static rank blocks, sequential 2^32-key chunks",
        "config": {"workload": "-m address -f tests/unsolvedpuzzles.rmd -l %s%s -b 71 (BASELINE configs[4]%s)"
                               % (["uncompress", "compress", "both"][args.search], " -e" if args.endo else "",
                                  " with -e" if args.endo else ""),
                   "endomorphism": args.endo,
                   "reference_stat_keys_per_s": round(rate * (6 if args.endo else (2 if args.search == 1 else 1))),
                   "targets": len(A.table()), "n_seq": hex(n_seq), "chunks_per_step": chunks,
                   "keys_per_step": chunks * n_seq, "parallelism": "range-partition x%d" % world,
                   "table_build_s": round(t_build, 2), "bloom_hits": st["hits"], "found": len(found),
                   "launches": st["launches"], **lib_rec},
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    if args.variant:
        out["variant"] = args.variant
    print(json.dumps(out), flush=True)
    A.close()
    if world > 1:
        dist.destroy_process_group()

if __name__ == "__main__":
    main()
