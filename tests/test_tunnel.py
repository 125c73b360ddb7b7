"""TCP tunnels through the master (reference: `harness/determined/cli/tunnel.py`, `cli/proxy.py`):
``/tunnel/{task}`` upgrade on the master, ``open_tunnel`` / ``listeners`` on the client, and the
stdio mode used as an ssh ProxyCommand."""
import os
import socket
import socketserver
import subprocess
import sys
import threading

import pytest

from determined_clone_amd.cli import tunnel
from determined_clone_amd.master.core import Allocation, Master
from determined_clone_amd.master.server import MasterServer

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Echo(socketserver.BaseRequestHandler):
    def handle(self):
        while True:
            data = self.request.recv(65536)
            if not data:
                break
            self.request.sendall(data.upper())


@pytest.fixture()
def cluster(tmp_path):
    echo = socketserver.ThreadingTCPServer(("127.0.0.1", 0), _Echo)
    echo.daemon_threads = True
    threading.Thread(target=echo.serve_forever, daemon=True).start()
    m = Master(str(tmp_path / "m.db"))
    srv = MasterServer(m, port=0).start()
    a = Allocation("t1.a", "t1", "SHELL")
    a.proxy_address = f"http://127.0.0.1:{echo.server_address[1]}"
    m.allocations[a.id] = a
    admin_tok, _ = m.login("admin", "")
    yield m, f"http://127.0.0.1:{srv.port}", admin_tok, echo.server_address[1]
    srv.stop()
    echo.shutdown()
    echo.server_close()


def _roundtrip(sock, payload=b"hello tunnel"):
    sock.sendall(payload)
    got = b""
    while len(got) < len(payload):
        got += sock.recv(65536)
    return got


def test_open_tunnel_default_and_explicit_port(cluster):
    m, url, tok, echo_port = cluster
    s, rest = tunnel.open_tunnel(url, tok, "t1")
    with s:
        assert rest == b"" and _roundtrip(s) == b"HELLO TUNNEL"
        big = os.urandom(1 << 20).hex().encode()[: 1 << 20]  # 1 MiB both ways
        assert _roundtrip(s, big) == big.upper()
    s, _ = tunnel.open_tunnel(url, tok, "t1", port=echo_port)
    with s:
        assert _roundtrip(s, b"x") == b"X"


def test_tunnel_refusals(cluster):
    m, url, tok, _ = cluster
    with pytest.raises(ConnectionError, match="401"):
        tunnel.open_tunnel(url, None, "t1")
    with pytest.raises(ConnectionError, match="404"):
        tunnel.open_tunnel(url, tok, "nope")
    with pytest.raises(ConnectionError, match="502"):
        tunnel.open_tunnel(url, tok, "t1", port=1)
    # another (non-admin) user may not tunnel into someone else's task
    from determined_clone_amd.master.core import hash_password

    m.db.insert("users", {"username": "eve", "admin": 0, "active": 1, "password_hash": hash_password(""),
                          "created": 0})
    m.task_owner = lambda task_id: 1  # owned by admin
    eve_tok, _ = m.login("eve", "")
    with pytest.raises(ConnectionError, match="403"):
        tunnel.open_tunnel(url, eve_tok, "t1")
    # a plain GET without the upgrade header is rejected
    import requests

    r = requests.get(url + "/tunnel/t1", headers={"Authorization": f"Bearer {tok}"})
    assert r.status_code == 400


def test_listeners_port_map(cluster):
    m, url, tok, echo_port = cluster
    with tunnel.listeners(url, tok, "t1", {0: echo_port}) as ports:
        for p in ports:
            with socket.create_connection(("127.0.0.1", p)) as c:
                assert _roundtrip(c, b"abc") == b"ABC"
    assert tunnel.parse_port_map(["8080:80", "6006"]) == {8080: 80, 6006: 6006}


def test_stdio_mode_as_proxy_command(cluster):
    m, url, tok, _ = cluster
    p = subprocess.run([sys.executable, "-m", "determined_clone_amd.cli.tunnel", url, "t1", "--token", tok],
                       input=b"ssh-2.0 banner\n", capture_output=True, timeout=60, cwd=REPO)
    assert p.stdout == b"SSH-2.0 BANNER\n", p.stderr
