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
    # only the service port and declared proxy_ports are reachable, even for an admin
    with pytest.raises(ConnectionError, match="403"):
        tunnel.open_tunnel(url, tok, "t1", port=1)
    # another (non-admin) user may not tunnel into someone else's task
    from determined_clone_amd.master.core import hash_password

    m.db.insert("users", {"username": "eve", "admin": 0, "active": 1, "password_hash": hash_password(""),
                          "created": 0})
    eve_tok, eve = m.login("eve", "")
    with pytest.raises(ConnectionError, match="403"):  # a task nobody owns is not public
        tunnel.open_tunnel(url, eve_tok, "t1")
    m.task_owner = lambda task_id: 1  # owned by admin
    with pytest.raises(ConnectionError, match="403"):
        tunnel.open_tunnel(url, eve_tok, "t1")
    m.task_owner = lambda task_id: eve["id"]
    s, _ = tunnel.open_tunnel(url, eve_tok, "t1")
    s.close()
    # a plain GET without the upgrade header is rejected
    import requests

    r = requests.get(url + "/tunnel/t1", headers={"Authorization": f"Bearer {tok}"})
    assert r.status_code == 400


def test_trial_tunnel_needs_experiment_rights(cluster):
    """A trial task has no NTSC owner: the tunnel checks the experiment (owner / admin / RBAC
    UPDATE_EXPERIMENT) and reaches only the ports the experiment declares in proxy_ports."""
    from determined_clone_amd.master.core import hash_password

    m, url, tok, echo_port = cluster
    a = Allocation("9.1.0", "9.1", "TRIAL")
    a.placements = [{"agent_id": "agent-x"}]
    m.allocations[a.id] = a

    class _Agent:
        addresses = ["127.0.0.1"]

    m.rm.agents["agent-x"] = _Agent()
    for name in ("alice", "bob"):
        m.db.insert("users", {"username": name, "admin": 0, "active": 1, "password_hash": hash_password(""),
                              "created": 0})
    alice_tok, alice = m.login("alice", "")
    bob_tok, _ = m.login("bob", "")
    exp = {"id": 9, "owner_id": alice["id"], "project_id": None,
           "config": {"environment": {"proxy_ports": [{"proxy_port": echo_port, "proxy_tcp": True}]}}}
    m.task_experiment = lambda task_id: exp if task_id == "9.1" else None
    with pytest.raises(ConnectionError, match="403"):
        tunnel.open_tunnel(url, bob_tok, "9.1", port=echo_port)
    with pytest.raises(ConnectionError, match="403"):  # not a declared port
        tunnel.open_tunnel(url, alice_tok, "9.1", port=echo_port + 1)
    for t in (alice_tok, tok):
        s, _ = tunnel.open_tunnel(url, t, "9.1", port=echo_port)
        with s:
            assert _roundtrip(s, b"ok") == b"OK"
    # with RBAC, an editor role in the experiment's workspace grants access too
    m.authz.mode = "rbac"
    with pytest.raises(ConnectionError, match="403"):
        tunnel.open_tunnel(url, bob_tok, "9.1", port=echo_port)
    m.authz.permitted = lambda user, perm, ws=None: perm == "UPDATE_EXPERIMENT"
    s, _ = tunnel.open_tunnel(url, bob_tok, "9.1", port=echo_port)
    s.close()


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


def test_ports_example_published_through_master(tmp_path):
    """examples/features/ports on an in-process cluster: the trial's dashboard port is reached
    from this machine through `/tunnel/{task}` (what `det e create ports.yaml . -p 8265` does)."""
    import base64
    import json
    import time
    import urllib.request

    import yaml

    from determined_clone_amd.agent import Agent
    from determined_clone_amd.common.api import Session
    from determined_clone_amd.util import tar_directory

    ex = os.path.join(REPO, "examples", "features", "ports")
    m = Master(str(tmp_path / "m.db"), checkpoint_storage={"type": "shared_fs", "host_path": str(tmp_path / "ck")})
    srv = MasterServer(m, port=0).start()
    agent = Agent(m.master_url, "agent-0", artificial_slots=1).start_background()
    try:
        s = Session(m.master_url)
        s.token = s.post("/api/v1/auth/login", {"username": "admin", "password": ""})["token"]
        with socket.socket() as probe:
            probe.bind(("127.0.0.1", 0))
            port = probe.getsockname()[1]
        cfg = yaml.safe_load(open(os.path.join(ex, "ports.yaml")))
        cfg["hyperparameters"] = {"steps": 30, "linger_s": 60}
        cfg["environment"]["environment_variables"] = [f"DASHBOARD_PORT={port}"]
        cfg["environment"]["proxy_ports"] = [{"proxy_port": port, "proxy_tcp": True}]
        body = {"config": cfg, "model_definition": base64.b64encode(tar_directory(ex)).decode()}
        eid = s.post("/api/v1/experiments", body)["experiment"]["id"]
        task_id, state, deadline = None, None, time.time() + 120
        while time.time() < deadline:
            ts = s.get(f"/api/v1/experiments/{eid}/trials")["trials"]
            task_id = next((t["task_id"] for t in ts if t.get("task_id")), None)
            if task_id:
                try:
                    with tunnel.listeners(m.master_url, s.token, task_id, {0: port}) as (local,):
                        with urllib.request.urlopen(f"http://127.0.0.1:{local}/", timeout=10) as r:
                            state = json.loads(r.read())
                    if state.get("step", 0) >= 30:
                        break
                except (OSError, ValueError):
                    pass
            time.sleep(0.5)
        assert state is not None and state["step"] == 30 and state["task"] == task_id, state
        s.post(f"/api/v1/experiments/{eid}/kill")
    finally:
        agent.stop()
        srv.stop()
