"""Shell task: an interactive bash session in the task's container, reachable through the master's
``/proxy/<task_id>/`` route.

Reference: SHELL tasks (`master/internal/api_shell.go`) run ``sshd`` in the container and
``det shell open`` connects with ``ssh`` through ``det tunnel`` (a TCP-over-websocket proxy via the
master). There is no sshd in this image, so the session is served over HTTP instead: a bash
process on a pseudo-terminal, output kept in a byte log that clients read by offset.

* ``POST /input {"data"}``     -- bytes to the terminal (keystrokes / lines);
* ``GET  /output?since=N&wait=S`` -- output from byte offset N, long-polling up to S seconds for
  new bytes -> ``{"data", "next", "closed"}``;
* ``POST /run {"cmd", "timeout"}`` -- one non-interactive command in a fresh ``bash -lc`` in the
  same environment -> ``{"exit_code", "output"}`` (``det shell run``).

The task ends when the bash session exits or after ``--idle-timeout`` seconds without requests.
"""
import argparse
import json
import os
import pty
import select
import subprocess
import sys
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, List, Optional
from urllib.parse import parse_qs, urlparse

from determined_clone_amd.util import proxy_secret_ok, routable_address


class ShellSession:
    def __init__(self, cwd: str, shell: str = "/bin/bash") -> None:
        self.master_fd, slave = pty.openpty()
        env = dict(os.environ, TERM=os.environ.get("TERM", "xterm"), PS1="det-shell$ ")
        self.proc = subprocess.Popen([shell, "--norc", "-i"], stdin=slave, stdout=slave, stderr=slave,
                                     cwd=cwd, env=env, start_new_session=True)
        os.close(slave)
        self.log = bytearray()
        self.cv = threading.Condition()
        self.closed = False
        threading.Thread(target=self._read, daemon=True).start()

    def _read(self) -> None:
        while True:
            try:
                r, _, _ = select.select([self.master_fd], [], [], 0.5)
                if not r:
                    if self.proc.poll() is not None:
                        break
                    continue
                chunk = os.read(self.master_fd, 65536)
            except OSError:
                break
            if not chunk:
                break
            with self.cv:
                self.log.extend(chunk)
                self.cv.notify_all()
        with self.cv:
            self.closed = True
            self.cv.notify_all()

    def write(self, data: str) -> None:
        os.write(self.master_fd, data.encode())

    def read(self, since: int, wait: float) -> dict:
        deadline = time.time() + wait
        with self.cv:
            while len(self.log) <= since and not self.closed and time.time() < deadline:
                self.cv.wait(max(0.0, deadline - time.time()))
            data = bytes(self.log[since:])
            return {"data": data.decode(errors="replace"), "next": since + len(data), "closed": self.closed}

    def close(self) -> None:
        if self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(5)
            except subprocess.TimeoutExpired:
                self.proc.kill()


def make_server(session: ShellSession, cwd: str, host: Optional[str] = None, port: int = 0) -> ThreadingHTTPServer:
    """The shell's HTTP service, bound to ``host`` (default: the routable address registered with
    the master). On a cluster every request must carry the task's proxy secret
    (``util.proxy_secret_ok``), which only the master's owner-checked ``/proxy/`` route attaches."""
    class H(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"
        disable_nagle_algorithm = True  # headers + body writes: no delayed-ACK stall
        last = [time.time()]

        def log_message(self, *a: Any) -> None:
            pass

        def _send(self, code: int, obj: Any) -> None:
            data = json.dumps(obj).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

        def _body(self) -> Any:
            n = int(self.headers.get("Content-Length") or 0)
            return json.loads(self.rfile.read(n)) if n else {}

        def _authorized(self) -> bool:
            if proxy_secret_ok(self.headers):
                return True
            self._send(403, {"error": "requests must come through the master's /proxy/ route"})
            return False

        def do_GET(self) -> None:
            if not self._authorized():
                return
            H.last[0] = time.time()
            u = urlparse(self.path)
            q = parse_qs(u.query)
            if u.path == "/output":
                self._send(200, session.read(int(q.get("since", ["0"])[0]), min(30.0, float(q.get("wait", ["0"])[0]))))
            else:
                self._send(200, {"service": "shell", "closed": session.closed})

        def do_POST(self) -> None:
            if not self._authorized():
                return
            H.last[0] = time.time()
            u = urlparse(self.path)
            b = self._body()
            if u.path == "/input":
                session.write(str(b.get("data", "")))
                self._send(200, {})
            elif u.path == "/run":
                try:
                    p = subprocess.run(["bash", "-lc", str(b["cmd"])], cwd=cwd, capture_output=True,
                                       text=True, timeout=float(b.get("timeout", 600)))
                    self._send(200, {"exit_code": p.returncode, "output": p.stdout + p.stderr})
                except subprocess.TimeoutExpired as e:
                    self._send(200, {"exit_code": 124, "output": f"timed out after {e.timeout}s"})
            else:
                self._send(404, {"error": "no route"})

    srv = ThreadingHTTPServer((routable_address() if host is None else host, port), H)
    srv.daemon_threads = True
    srv.last_activity = H.last  # type: ignore[attr-defined]
    return srv


def main(argv: Optional[List[str]] = None) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--port", type=int, default=0)
    p.add_argument("--idle-timeout", type=float, default=float(os.environ.get("DET_SHELL_IDLE_TIMEOUT", "0")))
    a = p.parse_args(argv)
    cwd = os.environ.get("DET_CONTEXT_DIR") or os.getcwd()
    session = ShellSession(cwd)
    srv = make_server(session, cwd, port=a.port)
    addr = f"http://{srv.server_address[0]}:{srv.server_address[1]}"
    print(f"shell service at {addr}", flush=True)
    from determined_clone_amd import _info

    info = _info.get_cluster_info()
    if info is not None:
        from determined_clone_amd.common.api import Session

        try:
            Session(info.master_url, token=info.session_token).post(
                f"/api/v1/allocations/{info.allocation_id}/proxy_address", {"proxy_address": addr})
        except Exception as e:  # pragma: no cover - proxy registration is best effort
            print(f"could not register proxy address: {e}", file=sys.stderr)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        while not session.closed:
            time.sleep(0.5)
            if a.idle_timeout and time.time() - srv.last_activity[0] > a.idle_timeout:
                print("shell idle: shutting down", flush=True)
                break
    finally:
        session.close()
        srv.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
