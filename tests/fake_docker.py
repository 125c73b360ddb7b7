"""A fake Docker Engine daemon on a unix socket for the CPU test tier.

Implements the Engine API subset ``agent/containers.py`` uses (ping, image inspect / pull with
``X-Registry-Auth``, container create / start / logs (multiplexed stream) / wait / kill / remove /
inspect / list by label). A "container" really runs its ``Cmd`` as a local process group: every
bind-mount target in the command, environment and working directory is rewritten to its host
source and ``python3`` to this interpreter -- so a task started through the agent's container
runtime executes for real -- while every create request body is recorded for assertions
(devices, groups, security options, mounts, shm size, labels).
"""
import base64
import json
import os
import signal
import socketserver
import subprocess
import sys
import threading
import time
import urllib.parse
import uuid
from http.server import BaseHTTPRequestHandler
from typing import Any, Dict, List


class _Container:
    def __init__(self, cid: str, name: str, config: Dict[str, Any]) -> None:
        self.id, self.name, self.config = cid, name, config
        self.proc: Any = None
        self.out: List[bytes] = []  # (lines)
        self.cv = threading.Condition()
        self.exit_code: Any = None
        self.started = 0.0


class FakeDocker:
    def __init__(self, sock_path: str) -> None:
        self.sock_path = sock_path
        self.images = set()
        self.pulls: List[Dict[str, Any]] = []
        self.pull_gate = threading.Event()  # cleared: image pulls block until it is set
        self.pull_gate.set()
        self.creates: List[Dict[str, Any]] = []
        self.containers: Dict[str, _Container] = {}
        self.lock = threading.Lock()
        fake = self

        class Handler(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.0"  # streamed responses end at connection close

            def log_message(self, *a: Any) -> None:
                pass

            def do_GET(self) -> None:
                fake._dispatch(self, "GET")

            def do_POST(self) -> None:
                fake._dispatch(self, "POST")

            def do_DELETE(self) -> None:
                fake._dispatch(self, "DELETE")

        class Server(socketserver.ThreadingMixIn, socketserver.UnixStreamServer):
            daemon_threads = True

            def get_request(self):  # BaseHTTPRequestHandler wants a (host, port) client address
                conn, _ = super().get_request()
                return conn, ("local", 0)

        if os.path.exists(sock_path):
            os.unlink(sock_path)
        self.server = Server(sock_path, Handler)
        threading.Thread(target=self.server.serve_forever, daemon=True).start()

    # ------------------------------------------------------------------ plumbing
    def _send(self, h: BaseHTTPRequestHandler, code: int, obj: Any = None) -> None:
        data = b"" if obj is None else (obj if isinstance(obj, bytes) else json.dumps(obj).encode())
        h.send_response(code)
        h.send_header("Content-Type", "application/json")
        h.send_header("Content-Length", str(len(data)))
        h.end_headers()
        h.wfile.write(data)

    def _dispatch(self, h: BaseHTTPRequestHandler, method: str) -> None:
        u = urllib.parse.urlsplit(h.path)
        path = u.path
        if path.startswith("/v1."):
            path = "/" + path.split("/", 2)[2]
        q = dict(urllib.parse.parse_qsl(u.query))
        n = int(h.headers.get("Content-Length") or 0)
        body = json.loads(h.rfile.read(n)) if n else None
        parts = path.strip("/").split("/")
        try:
            if path == "/_ping":
                h.send_response(200)
                h.send_header("Content-Length", "2")
                h.end_headers()
                h.wfile.write(b"OK")
            elif parts[0] == "images" and parts[-1] == "json":
                name = urllib.parse.unquote("/".join(parts[1:-1]))
                self._send(h, 200 if name in self.images else 404,
                           {"Id": name} if name in self.images else {"message": "No such image"})
            elif path == "/images/create":
                auth = h.headers.get("X-Registry-Auth")
                dec = json.loads(base64.urlsafe_b64decode(auth + "===")) if auth else None
                ref = q["fromImage"] + (f":{q['tag']}" if q.get("tag") else "")
                self.pulls.append({"image": ref, "auth": dec})
                self.pull_gate.wait(60)  # a slow registry
                self.images.add(ref)
                self._send(h, 200, b'{"status":"Pulling from fake"}\n{"status":"Download complete"}\n')
            elif path == "/containers/create":
                cid = uuid.uuid4().hex
                with self.lock:
                    self.containers[cid] = _Container(cid, q.get("name", cid), body)
                    self.creates.append(body)
                self._send(h, 201, {"Id": cid, "Warnings": []})
            elif path == "/containers/json":
                want = json.loads(q.get("filters", "{}")).get("label", [])
                out = []
                for c in list(self.containers.values()):
                    labels = c.config.get("Labels") or {}
                    if all(labels.get(w.split("=", 1)[0]) == w.split("=", 1)[1] for w in want):
                        running = c.exit_code is None and c.proc is not None
                        if q.get("all") in ("1", "true") or running:
                            out.append({"Id": c.id, "Labels": labels, "State": "running" if running else "exited"})
                self._send(h, 200, out)
            elif parts[0] == "containers" and len(parts) >= 2:
                c = self.containers.get(parts[1])
                if c is None:
                    self._send(h, 404, {"message": "No such container"})
                    return
                op = parts[2] if len(parts) > 2 else ""
                if method == "DELETE":
                    self._stop(c, signal.SIGKILL)
                    with self.lock:
                        self.containers.pop(c.id, None)
                    self._send(h, 204)
                elif op == "start":
                    self._start(c)
                    self._send(h, 204)
                elif op == "wait":
                    with c.cv:
                        c.cv.wait_for(lambda: c.exit_code is not None)
                    self._send(h, 200, {"StatusCode": c.exit_code})
                elif op == "kill":
                    sig = getattr(signal, q.get("signal", "SIGKILL"))
                    if c.exit_code is not None or c.proc is None:
                        self._send(h, 409, {"message": "not running"})
                    else:
                        self._stop(c, sig)
                        self._send(h, 204)
                elif op == "json":
                    self._send(h, 200, {"Id": c.id, "State": {"Running": c.exit_code is None and c.proc is not None,
                                                             "ExitCode": c.exit_code or 0}})
                elif op == "logs":
                    self._stream_logs(h, c, float(q["since"]) if q.get("since") else None)
                else:
                    self._send(h, 404, {"message": f"unsupported {path}"})
            else:
                self._send(h, 404, {"message": f"unsupported {path}"})
        except BrokenPipeError:
            pass

    # ------------------------------------------------------------------ "containers"
    def _host_path(self, c: _Container, s: str) -> str:
        mounts = sorted((c.config.get("HostConfig") or {}).get("Mounts") or [], key=lambda m: -len(m["Target"]))
        for m in mounts:
            s = s.replace(m["Target"], m["Source"])
        return s

    def _start(self, c: _Container) -> None:
        cfg = c.config
        env = {k: self._host_path(c, v) for k, v in (e.split("=", 1) for e in cfg.get("Env") or [])}
        env["PATH"] = os.environ.get("PATH", "/usr/bin:/bin")
        env.setdefault("HOME", os.environ.get("HOME", "/tmp"))
        cmd = [sys.executable if a == "python3" else self._host_path(c, a) for a in cfg["Cmd"]]
        cwd = self._host_path(c, cfg.get("WorkingDir") or "/")
        c.proc = subprocess.Popen(cmd, cwd=cwd, env=env, stdout=subprocess.PIPE,
                                  stderr=subprocess.STDOUT, start_new_session=True)
        c.started = time.time()

        def pump() -> None:
            for line in iter(c.proc.stdout.readline, b""):
                with c.cv:
                    c.out.append((time.time(), line))
                    c.cv.notify_all()
            code = c.proc.wait()
            with c.cv:
                c.exit_code = code if code >= 0 else 128 - code
                c.cv.notify_all()

        threading.Thread(target=pump, daemon=True).start()

    def _stop(self, c: _Container, sig: int) -> None:
        if c.proc is not None and c.exit_code is None:
            try:
                os.killpg(c.proc.pid, sig)
            except ProcessLookupError:
                pass

    def _stream_logs(self, h: BaseHTTPRequestHandler, c: _Container, since: Any) -> None:
        h.send_response(200)
        h.send_header("Content-Type", "application/vnd.docker.raw-stream")
        h.end_headers()
        i = 0
        while True:
            with c.cv:
                c.cv.wait_for(lambda: len(c.out) > i or c.exit_code is not None, timeout=1.0)
                batch = c.out[i:]
                i = len(c.out)
                done = c.exit_code is not None and i == len(c.out)
            for ts, line in batch:
                if since is not None and ts < since:
                    continue
                h.wfile.write(bytes([1, 0, 0, 0]) + len(line).to_bytes(4, "big") + line)
            h.wfile.flush()
            if done:
                return

    def close(self) -> None:
        for c in list(self.containers.values()):
            self._stop(c, signal.SIGKILL)
        self.server.shutdown()
        self.server.server_close()
