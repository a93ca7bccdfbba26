"""bench.py --gpus N launches N ranks by itself: the launch decision, the spawned
world (gloo on CPU, no GPU touched: --launch-check) and the failure paths."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

from keyhuntm1cpu_amd import launch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _clean_env(**kw):
    e = {k: v for k, v in os.environ.items()
         if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "KHB_BENCH_CHILD")}
    e.update(kw)
    return e


def test_plan():
    assert launch.plan(1, {}) == "single"
    assert launch.plan(8, {}) == "spawn"                       # bare --gpus 8: N children
    assert launch.plan(8, {"WORLD_SIZE": ""}) == "spawn"
    assert launch.plan(8, {"WORLD_SIZE": "8"}) == "rank"       # under torch.distributed.run
    assert launch.plan(1, {"WORLD_SIZE": "1"}) == "single"
    for gpus, ws in ((2, "8"), (8, "1"), (1, "2")):
        with pytest.raises(SystemExit) as e:
            launch.plan(gpus, {"WORLD_SIZE": ws})
        assert e.value.code == 2
    with pytest.raises(SystemExit):
        launch.plan(0, {})
    with pytest.raises(SystemExit):
        launch.plan(2, {"WORLD_SIZE": "two"})


def test_rank_env():
    e = launch.rank_env({"X": "1"}, 3, 8, 12345)
    assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["MASTER_ADDR"], e["MASTER_PORT"], e["X"]) == \
        ("3", "3", "8", "127.0.0.1", "12345", "1")


def _bench(args, env, timeout=180):
    return subprocess.run([sys.executable, BENCH, *args], env=env, capture_output=True, text=True, timeout=timeout,
                          cwd="/tmp")


@pytest.mark.parametrize("n", [2, 3])
def test_bare_gpus_n_spawns_n_ranks(n):
    r = _bench(["--gpus", str(n), "--launch-check"], _clean_env())
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1                                     # exactly rank 0's line on stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n
    assert [v["rank"] for v in d["ranks"]] == list(range(n))
    assert [v["local_rank"] for v in d["ranks"]] == list(range(n))
    assert len({v["pid"] for v in d["ranks"]}) == n            # n distinct processes


def test_single_gpu_runs_in_process():
    r = _bench(["--gpus", "1", "--launch-check"], _clean_env())
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout)["n_gpus"] == 1
    assert "starting" not in r.stderr


def test_world_size_mismatch_refused():
    r = _bench(["--gpus", "4", "--launch-check"], _clean_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2
    assert r.stdout.strip() == ""
    assert "differs from --gpus 4" in r.stderr


def test_failing_rank_fails_the_launch():
    r = _bench(["--gpus", "3", "--launch-check", "--launch-check-fail", "2"], _clean_env())
    assert r.returncode == 3
    assert r.stdout.strip() == ""                              # no line when a rank failed
    assert "rank 2 exited with status 3" in r.stderr


def test_straggler_rank_is_stopped():
    """A rank that hangs after another rank exited cleanly is stopped after straggler_s:
    the launch returns 124 instead of polling forever."""
    code = ("import os, time, sys\n"
            "time.sleep(3600 if os.environ['RANK'] == '1' else 0)\n")
    import time
    t0 = time.time()
    rc = launch.spawn_ranks(2, [sys.executable, "-c", code], env=_clean_env(), grace_s=1.0, straggler_s=2.0)
    assert rc == 124
    assert time.time() - t0 < 30


def test_overall_timeout_stops_ranks():
    code = "import time\ntime.sleep(3600)\n"
    rc = launch.spawn_ranks(2, [sys.executable, "-c", code], env=_clean_env(), grace_s=1.0, timeout_s=2.0)
    assert rc == 124


def test_rank0_may_outlive_the_others():
    """bench.py's rank 0 runs the CPU baseline alone after the other ranks returned: a rank 0 that
    outlives them by more than straggler_s is not stopped; the launch returns its status and its stdout."""
    code = ("import os, time, sys\n"
            "if os.environ['RANK'] == '0':\n"
            "    time.sleep(4.0)\n"
            "    print('rank0-line', flush=True)\n")
    rc = launch.spawn_ranks(2, [sys.executable, "-c", code], env=_clean_env(), grace_s=1.0, straggler_s=1.0)
    assert rc == 0


def test_bench_gpus_8_launch_check():
    """bench.py --gpus 8 --launch-check: eight gloo ranks spawned by bench.py itself (no GPU touched), the
    world the driver's N=8 scaling run starts."""
    r = _bench(["--gpus", "8", "--launch-check"], _clean_env(), timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8
    assert [v["rank"] for v in d["ranks"]] == list(range(8))
    assert len({v["pid"] for v in d["ranks"]}) == 8


def test_bench_refuses_unnamed_library_dir(tmp_path):
    """KHB_LIB_DIR pointing away from the in-tree build is refused before any rank starts unless
    --variant names the build (whose line is then marked); the in-tree directory itself is accepted."""
    r = _bench(["--gpus", "1", "--launch-check"], _clean_env(KHB_LIB_DIR=str(tmp_path)))
    assert r.returncode != 0 and r.stdout.strip() == ""
    assert "--variant" in r.stderr and str(tmp_path) in r.stderr
    r = _bench(["--gpus", "1", "--launch-check", "--variant", "x"], _clean_env(KHB_LIB_DIR=str(tmp_path)))
    assert r.returncode == 0, r.stderr
    r = _bench(["--gpus", "1", "--launch-check"], _clean_env(KHB_LIB_DIR=os.path.join(REPO, "keyhuntm1cpu_amd", "lib")))
    assert r.returncode == 0, r.stderr


def test_bench_records_the_loaded_library():
    """bench.lib_record: the line's config names the loaded libkhbsgs.so (path, sha256 prefix, khb_build_info) and
    refuses a build that says it is not the product when no --variant is given."""
    import argparse
    import hashlib
    sys.path.insert(0, REPO)
    import bench
    rec = bench.lib_record(argparse.Namespace(variant=None))
    with open(os.path.join(REPO, "keyhuntm1cpu_amd", "lib", "libkhbsgs.so"), "rb") as f:
        assert rec["lib_sha16"] == hashlib.sha256(f.read()).hexdigest()[:16]
    assert rec["lib_path"] == "keyhuntm1cpu_amd/lib/libkhbsgs.so"
    assert rec["build"]["variant"] == "product" and rec["build"]["abi"] == "7"
    with pytest.raises(SystemExit):
        bench.lib_record(argparse.Namespace(variant="half"))     # the product build is not variant "half"


def test_rank0_stuck_after_the_others_is_stopped():
    """The other side of ADVICE r5: a rank 0 that hangs after every other rank exited cleanly is stopped after
    rank0_grace_s (bench.py passes its CPU-baseline budget + 300 s), so a hung rank 0 cannot poll forever."""
    import time
    code = ("import os, time\n"
            "time.sleep(3600 if os.environ['RANK'] == '0' else 0)\n")
    t0 = time.time()
    rc = launch.spawn_ranks(2, [sys.executable, "-c", code], env=_clean_env(), grace_s=1.0, straggler_s=1.0,
                            rank0_grace_s=2.0)
    assert rc == 124
    assert time.time() - t0 < 30
