"""bsgsd_amd (bsgsd.cpp / BSGSD.md): tables resident on the GPU, one line per TCP connection,
replies exactly as the reference daemon: the key in hex, "404 Not Found" or "400 Bad Request"."""
from __future__ import annotations

import os
import socket
import subprocess
import time

import pytest

from keyhuntm1cpu_amd import BIN_DIR

pytestmark = pytest.mark.gpu
P63 = "0365ec2994b8cc0a20d40dd69edfe55ca32a54bcbbaa6b0ddcff36049301a54579"
P125 = "0233709eb11e0d4439a729f21c2c443dedb727528229713f0065721ba8fa46f00e"


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ask(port: int, line: bytes) -> str:
    with socket.create_connection(("127.0.0.1", port), timeout=120) as s:
        s.sendall(line)
        data = b""
        while True:
            chunk = s.recv(4096)
            if not chunk:
                break
            data += chunk
    return data.decode()


@pytest.fixture(scope="module", params=["host", "gpu"])
def daemon(tmp_path_factory, request):
    """The daemon with its candidates confirmed on the host pool, then on the GPU (--check gpu, khb_check)."""
    cwd = tmp_path_factory.mktemp("bsgsd")
    port = _free_port()
    log = open(cwd / "bsgsd.log", "w")
    p = subprocess.Popen([os.path.join(BIN_DIR, "bsgsd_amd"), "-k", "1", "-t", "8", "-p", str(port), "--check",
                          request.param], cwd=cwd, stdout=log, stderr=subprocess.STDOUT)
    t0 = time.time()
    while time.time() - t0 < 180:
        if p.poll() is not None:
            break
        if "[+] Listening in 127.0.0.1:%d" % port in (cwd / "bsgsd.log").read_text():
            break
        time.sleep(0.2)
    assert p.poll() is None, (cwd / "bsgsd.log").read_text()
    yield port, cwd
    p.terminate()
    try:
        p.wait(timeout=20)
    except subprocess.TimeoutExpired:
        p.kill()
        p.wait()
    log.close()


def test_bsgsd_known_answer(daemon):
    port, cwd = daemon
    assert _ask(port, f"{P63} 7cce500000000000:7cce600000000000\n".encode()) == "7cce5efdaccf6808"
    # the -S files were written at start-up (bsgsd reads / writes them like keyhunt -S)
    assert (cwd / "keyhunt_bsgs_4_4194304.blm").exists()


def test_bsgsd_not_found(daemon):
    port, _ = daemon
    assert _ask(port, f"{P125} 4000000000000000:4000800000000000\n".encode()) == "404 Not Found"


@pytest.mark.parametrize("line", [b"hello\n", P63.encode() + b" 10\n",
                                  b"02" + b"0" * 64 + b" 1:2\n",            # x = 0 is not on the curve
                                  P63.encode() + b" 12zz:34\n"])
def test_bsgsd_bad_request(daemon, line):
    port, _ = daemon
    assert _ask(port, line) == "400 Bad Request"


def test_bsgsd_serves_sequential_clients(daemon):
    port, cwd = daemon
    for _ in range(2):
        assert _ask(port, f"{P63} 7cce5e0000000000:7cce600000000000\n".encode()) == "7cce5efdaccf6808"
    log = (cwd / "bsgsd.log").read_text()
    assert "[+] Accepting incoming conection from 127.0.0.1:" in log
    assert "[+] Closing conection from 127.0.0.1:" in log
