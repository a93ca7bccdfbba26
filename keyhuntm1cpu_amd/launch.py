"""One process per GPU for bench.py, without an external launcher.

`python bench.py --gpus N` must time N ranks whether the driver wraps it in torch.distributed.run
(WORLD_SIZE set by the launcher) or runs it bare.  Bare with N > 1, bench.py starts N rank processes
itself as children — before anything touches the GPU, and never by exec — with the environment
torch.distributed.run would give them, forwards rank 0's single JSON line, and exits non-zero if any
rank fails.  The ranks share nothing on the data path (chunks are independent,
keyhunt.cpp:3824-3844); gloo only joins their barriers and max-reduces their times.

No torch import here: the parent never initialises HIP."""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import Mapping, Sequence


class LaunchError(SystemExit):
    """A launch the bench refuses: its message goes to stderr and the exit status is 2."""

    def __init__(self, msg: str):
        print(f"[bench] {msg}", file=sys.stderr, flush=True)
        super().__init__(2)


def plan(gpus: int, env: Mapping[str, str]) -> str:
    """'single' (one rank, no launcher), 'spawn' (start `gpus` ranks here) or 'rank' (this process is one
    rank of a launcher's world, WORLD_SIZE == gpus).  A WORLD_SIZE that differs from --gpus is refused:
    a line would otherwise claim a GPU count other than the one that ran."""
    if gpus < 1:
        raise LaunchError(f"--gpus {gpus}: at least one GPU")
    ws = env.get("WORLD_SIZE")
    if ws is None or ws == "":
        return "single" if gpus == 1 else "spawn"
    try:
        world = int(ws)
    except ValueError:
        raise LaunchError(f"WORLD_SIZE={ws!r} is not an integer")
    if world != gpus:
        raise LaunchError(f"WORLD_SIZE={world} (set by the launcher) differs from --gpus {gpus}")
    return "rank" if world > 1 else "single"


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(base: Mapping[str, str], rank: int, world: int, port: int) -> dict:
    """The variables torch.distributed.run sets for a one-node world (rendezvous on 127.0.0.1)."""
    e = dict(base)
    e.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
             GROUP_RANK="0", ROLE_RANK=str(rank), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
             KHB_BENCH_CHILD="1")
    return e


def _pump(src, dst):
    for line in iter(src.readline, b""):
        dst.write(line)
        dst.flush()
    src.close()


def _kill_group(p: subprocess.Popen, sig: int):
    try:
        os.killpg(p.pid, sig)
    except (ProcessLookupError, PermissionError):
        pass


def spawn_ranks(world: int, cmd: Sequence[str], env: Mapping[str, str] | None = None, grace_s: float = 15.0,
                straggler_s: float = 300.0, timeout_s: float | None = None, rank0_grace_s: float | None = None) -> int:
    """Run `cmd` as `world` rank processes; rank 0's stdout is forwarded to ours, the other ranks' stdout
    goes to our stderr (stdout keeps exactly rank 0's JSON line).  When a rank fails, the others are
    terminated (SIGTERM, then SIGKILL after grace_s) and its exit status is returned; 0 when all succeed.
    Once rank 0 has exited cleanly, the others have straggler_s to follow (rank 0 is the last to need them:
    bench.py's other ranks return after the final all_gather and rank 0 alone goes on to the CPU baseline, so
    only a rank still running after rank 0 is stuck); with timeout_s the whole run has that long.
    Rank 0 itself, once every other rank has exited cleanly, has rank0_grace_s (bench.py: its CPU-baseline budget
    plus straggler_s) before it is taken to be stuck.  Either limit stops the remaining ranks the same way and
    returns 124, as timeout(1) does."""
    base = dict(os.environ if env is None else env)
    port = free_port()
    procs: list[subprocess.Popen] = []
    pumps = []
    out = sys.stdout.buffer
    err = sys.stderr.buffer
    rc = 0

    def _stop(signum, frame):                 # the caller's timeout reaches the ranks too (finally below)
        raise SystemExit(128 + signum)
    prev = {sig: signal.signal(sig, _stop) for sig in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP)}
    try:
        for r in range(world):
            p = subprocess.Popen(list(cmd), env=rank_env(base, r, world, port), stdout=subprocess.PIPE,
                                 start_new_session=True)      # own process group: a failure ends the whole rank
            procs.append(p)
            t = threading.Thread(target=_pump, args=(p.stdout, out if r == 0 else err), daemon=True)
            t.start()
            pumps.append(t)
        live = set(range(world))
        t_start = time.time()
        first_exit = None                          # when rank 0 exited cleanly
        others_done = None                         # when every rank but 0 had exited cleanly

        def stop_live():
            for q in live:
                _kill_group(procs[q], signal.SIGTERM)
            deadline = time.time() + grace_s
            for q in list(live):
                try:
                    procs[q].wait(timeout=max(0.1, deadline - time.time()))
                except subprocess.TimeoutExpired:
                    _kill_group(procs[q], signal.SIGKILL)
                    procs[q].wait()
            live.clear()

        while live:
            for r in sorted(live):
                c = procs[r].poll()
                if c is None:
                    continue
                live.discard(r)
                if first_exit is None and r == 0 and c == 0:
                    first_exit = time.time()      # the straggler clock: rank 0 done, the others should be too
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c          # a signal -s reads as 128 + s, like a shell
                    print(f"[bench] rank {r} exited with status {c}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    stop_live()
                    break
            if not live:
                break
            now = time.time()
            if others_done is None and live == {0} and rc == 0:
                others_done = now
            late = first_exit is not None and now - first_exit > straggler_s
            late0 = rank0_grace_s is not None and others_done is not None and now - others_done > rank0_grace_s
            if late or late0 or (timeout_s is not None and now - t_start > timeout_s):
                why = (f"{straggler_s:.0f} s after rank 0 exited" if late else
                       f"{rank0_grace_s:.0f} s after the other ranks exited" if late0 else f"after {timeout_s:.0f} s")
                print(f"[bench] ranks {sorted(live)} still running {why}; stopping them", file=sys.stderr, flush=True)
                stop_live()
                rc = rc or 124
                break
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                _kill_group(p, signal.SIGKILL)
                p.wait()
        for t in pumps:
            t.join(timeout=5)
        for sig, h in prev.items():
            signal.signal(sig, h)
    return rc


def main_or_spawn(gpus: int, argv: Sequence[str], script: str, rank0_extra_s: float = 0.0) -> str:
    """bench.py's entry decision.  Returns the plan for this process; for 'spawn' it runs the ranks and
    exits with their status (the parent does no GPU work).  rank0_extra_s: the work rank 0 does alone after the
    other ranks return (bench.py's CPU baseline)."""
    p = plan(gpus, os.environ)
    if p == "spawn":
        print(f"[bench] WORLD_SIZE unset and --gpus {gpus}: starting {gpus} rank processes "
              f"(one per GPU, rendezvous on 127.0.0.1)", file=sys.stderr, flush=True)
        raise SystemExit(spawn_ranks(gpus, [sys.executable, "-u", script, *argv],
                                     rank0_grace_s=300.0 + rank0_extra_s))
    return p
