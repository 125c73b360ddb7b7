"""TCP tunnels to task ports through the master (reference: `harness/determined/cli/tunnel.py`
and `cli/proxy.py`: ``http_connect_tunnel`` for ssh ``ProxyCommand`` and
``http_tunnel_listener`` / ``--publish`` port maps).

The master upgrades ``GET /tunnel/{task_id}?port=N`` (``Upgrade: det-tcp``) to a raw byte pipe
to port N on the task's host, so no WebSocket framing is needed on either side.

* ``python -m determined_clone_amd.cli.tunnel MASTER TASK_ID [--port N]`` splices stdin/stdout
  (``ssh -o ProxyCommand="python -m determined_clone_amd.cli.tunnel $MASTER <task>" ...``);
* ``... --listener LOCAL_PORT`` / ``det task tunnel TASK_ID -p LOCAL:REMOTE`` serve local ports,
  one tunnel per accepted connection."""
import argparse
import os
import socket
import ssl
import socketserver
import sys
import threading
import urllib.parse
from typing import Dict, Iterator, List, Optional, Tuple
import contextlib


def open_tunnel(master_url: str, token: Optional[str], task_id: str,
                port: Optional[int] = None, timeout: float = 30.0) -> Tuple[socket.socket, bytes]:
    """Connect to the master and upgrade to a tunnel; returns the socket and any bytes the
    master's side already sent after the 101 response."""
    u = urllib.parse.urlsplit(master_url if "://" in master_url else "http://" + master_url)
    if u.scheme not in ("http", "https"):
        raise ValueError(f"unsupported master URL scheme {u.scheme!r}")
    sock = socket.create_connection((u.hostname or "127.0.0.1", u.port or 8080), timeout=timeout)
    if u.scheme == "https":  # verified like the REST session (DET_MASTER_CERT_FILE / _NAME)
        from determined_clone_amd.common.api import Cert

        cert = Cert.from_env()
        ctx = ssl.create_default_context(cafile=cert.bundle or None)
        if cert.bundle is False:
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE
        sock = ctx.wrap_socket(sock, server_hostname=cert.name or u.hostname)
    path = f"/tunnel/{urllib.parse.quote(task_id)}" + (f"?port={int(port)}" if port else "")
    req = (f"GET {path} HTTP/1.1\r\nHost: {u.netloc}\r\nConnection: Upgrade\r\nUpgrade: det-tcp\r\n"
           + (f"Authorization: Bearer {token}\r\n" if token else "") + "\r\n")
    sock.sendall(req.encode())
    buf = b""
    while b"\r\n\r\n" not in buf:
        chunk = sock.recv(4096)
        if not chunk:
            raise ConnectionError("master closed the connection during the tunnel handshake")
        buf += chunk
    head, rest = buf.split(b"\r\n\r\n", 1)
    status = head.split(b"\r\n", 1)[0].decode(errors="replace")
    if " 101 " not in status + " ":
        body = rest.decode(errors="replace")[:300]
        sock.close()
        raise ConnectionError(f"tunnel refused: {status} {body}")
    sock.settimeout(None)
    return sock, rest


def _pump(src: socket.socket, dst: socket.socket) -> None:
    try:
        while True:
            data = src.recv(65536)
            if not data:
                break
            dst.sendall(data)
    except OSError:
        pass
    finally:
        with contextlib.suppress(OSError):
            if isinstance(dst, ssl.SSLSocket):
                dst.close()  # TLS has no half-close
            else:
                dst.shutdown(socket.SHUT_WR)


def splice(a: socket.socket, b: socket.socket, a_pending: bytes = b"") -> None:
    """Copy both directions until both sides close (``a_pending`` goes to ``b`` first)."""
    if a_pending:
        b.sendall(a_pending)
    t = threading.Thread(target=_pump, args=(b, a), daemon=True)
    t.start()
    _pump(a, b)
    t.join()


def stdio_tunnel(master_url: str, token: Optional[str], task_id: str, port: Optional[int]) -> None:
    sock, rest = open_tunnel(master_url, token, task_id, port)
    out = sys.stdout.buffer
    if rest:
        out.write(rest)
        out.flush()

    def down() -> None:
        while True:
            data = sock.recv(65536)
            if not data:
                break
            out.write(data)
            out.flush()
        os._exit(0)

    threading.Thread(target=down, daemon=True).start()
    inp = sys.stdin.buffer
    while True:
        data = inp.read1(65536) if hasattr(inp, "read1") else inp.read(65536)
        if not data:
            with contextlib.suppress(OSError):
                sock.shutdown(socket.SHUT_WR)
            break
        sock.sendall(data)
    threading.Event().wait()


class _Server(socketserver.ThreadingTCPServer):
    allow_reuse_address = True
    daemon_threads = True


@contextlib.contextmanager
def listeners(master_url: str, token: Optional[str], task_id: str,
              port_map: Dict[int, int], host: str = "127.0.0.1") -> Iterator[List[int]]:
    """Serve ``local -> remote`` port maps (local 0 = any free port); yields the bound local ports."""
    servers = []
    for local, remote in port_map.items():
        class H(socketserver.BaseRequestHandler):
            remote_port = remote

            def handle(self) -> None:
                try:
                    up, rest = open_tunnel(master_url, token, task_id, self.remote_port)
                except (OSError, ConnectionError) as e:
                    print(f"tunnel to {task_id}:{self.remote_port} failed: {e}", file=sys.stderr)
                    return
                with up:
                    if rest:
                        self.request.sendall(rest)
                    splice(self.request, up)

        srv = _Server((host, local), H)
        threading.Thread(target=srv.serve_forever, daemon=True).start()
        servers.append(srv)
    try:
        yield [s.server_address[1] for s in servers]
    finally:
        for s in servers:
            s.shutdown()
            s.server_close()


def parse_port_map(specs: List[str]) -> Dict[int, int]:
    """``["8080:80", "6006"]`` -> ``{8080: 80, 6006: 6006}``."""
    out: Dict[int, int] = {}
    for spec in specs:
        local, _, remote = spec.partition(":")
        out[int(local)] = int(remote or local)
    return out


def main(argv: Optional[List[str]] = None) -> None:
    ap = argparse.ArgumentParser(description="Tunnel a TCP connection to a task through the master")
    ap.add_argument("master_url")
    ap.add_argument("task_id")
    ap.add_argument("--port", type=int, default=None, help="task port (default: its service port)")
    ap.add_argument("--listener", type=int, default=None, help="serve this local port instead of stdio")
    ap.add_argument("--token", default=os.environ.get("DET_SESSION_TOKEN"))
    a = ap.parse_args(argv)
    if a.listener is not None:
        with listeners(a.master_url, a.token, a.task_id, {a.listener: a.port or 0}):
            threading.Event().wait()
    else:
        stdio_tunnel(a.master_url, a.token, a.task_id, a.port)


if __name__ == "__main__":
    main()
