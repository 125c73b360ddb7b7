"""Native worker-failure detection (dca-pidwatch server/client)."""
import os
import subprocess
import sys
import time

import pytest

from determined_clone_amd.native import build


@pytest.fixture(scope="module")
def pw():
    return str(build.build_pidwatch())


def _launch(pw, addr, workers):
    clients = " & ".join(f"{pw} client {addr} -- {w}" for w in workers)
    return [pw, "server", "--grace-period", "1", addr, str(len(workers)), "--", "bash", "-c", clients + " & wait"]


def test_all_workers_succeed(pw, tmp_path):
    addr = str(tmp_path / "pid.sock")
    r = subprocess.run(_launch(pw, addr, ["true", "sleep 0.5"]), timeout=60)
    assert r.returncode == 0


def test_worker_failure_tears_down_job(pw, tmp_path):
    addr = str(tmp_path / "pid.sock")
    t0 = time.time()
    r = subprocess.run(_launch(pw, addr, ["sleep 60", "bash -c 'sleep 0.5; exit 3'"]), timeout=60)
    assert r.returncode == 70
    assert time.time() - t0 < 20, "surviving worker was not torn down"


def test_tcp_address_and_python_entrypoints(tmp_path):
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "determined_clone_amd.exec.pid_server", str(port), "1", "--",
           sys.executable, "-m", "determined_clone_amd.exec.pid_client", str(port), "--", "true"]
    env = dict(os.environ, PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert subprocess.run(cmd, timeout=120, env=env).returncode == 0


def test_wrap_rank_prefixes_lines(capfd):
    from determined_clone_amd.launch import wrap_rank

    rc = wrap_rank.main(["3", "--", sys.executable, "-c",
                         "import sys; print('a'); sys.stdout.write('b\\rc\\n'); print('err', file=sys.stderr)"])
    out, err = capfd.readouterr()
    assert rc == 0
    assert out.splitlines() == ["[rank=3] a", "[rank=3] b", "[rank=3] c"]
    assert err.strip() == "[rank=3] err"
