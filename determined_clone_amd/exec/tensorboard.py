"""TensorBoard task (reference: `harness/determined/exec/tensorboard.py`, which fetches trial event
files from checkpoint storage and starts the TensorBoard server).

TensorBoard is not part of this image, so the task serves the scalars itself: it resolves each
experiment's synced event-file directory (``<storage>/tensorboard/<cluster>/experiment/<id>``),
parses the TF event files natively (:func:`determined_clone_amd.tensorboard.read_scalars`) and serves
``/`` (HTML index), ``/data/runs`` and ``/data/scalars?run=...&tag=...`` (JSON, TensorBoard's scalar
route shape: ``[[wall_time, step, value], ...]``). Its address is registered as the task's proxy.

Usage: ``python -m determined_clone_amd.exec.tensorboard EXP_ID... [--logdir DIR] [--port N]``.
"""
import argparse
import html
import json
import os
import sys
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Dict, List, Optional
from urllib.parse import parse_qs, urlparse

from determined_clone_amd import _info
from determined_clone_amd.tensorboard import read_scalars
from determined_clone_amd.util import proxy_secret_ok, routable_address


def collect(logdirs: Dict[str, str]) -> Dict[str, Dict[str, list]]:
    runs: Dict[str, Dict[str, list]] = {}
    for name, d in logdirs.items():
        for run, tags in read_scalars(d).items():
            runs[f"{name}/{run}" if run != "." else name] = tags
    return runs


def make_server(logdirs: Dict[str, str], host: Optional[str] = None, port: int = 0) -> ThreadingHTTPServer:
    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):  # quiet
            pass

        def _send(self, code: int, body: bytes, ctype: str) -> None:
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def do_GET(self) -> None:
            if not proxy_secret_ok(self.headers):
                return self._send(403, b'{"error": "requests must come through the master proxy"}',
                                  "application/json")
            u = urlparse(self.path)
            q = {k: v[0] for k, v in parse_qs(u.query).items()}
            runs = collect(logdirs)
            if u.path.endswith("/data/runs"):
                return self._send(200, json.dumps({r: sorted(t) for r, t in runs.items()}).encode(), "application/json")
            if u.path.endswith("/data/scalars"):
                series = runs.get(q.get("run", ""), {}).get(q.get("tag", ""))
                if series is None:
                    return self._send(404, b'{"error": "no such run/tag"}', "application/json")
                return self._send(200, json.dumps([[w, s, v] for s, w, v in series]).encode(), "application/json")
            rows = []
            for r, tags in sorted(runs.items()):
                for t, series in sorted(tags.items()):
                    last = series[-1]
                    rows.append(f"<tr><td>{html.escape(r)}</td><td>{html.escape(t)}</td><td>{len(series)}</td>"
                                f"<td>{last[0]}</td><td>{last[2]:.6g}</td></tr>")
            page = ("<html><head><title>determined_clone_amd tensorboard</title></head><body>"
                    "<h2>Scalars</h2><table border=1><tr><th>run</th><th>tag</th><th>points</th>"
                    "<th>last step</th><th>last value</th></tr>" + "".join(rows) + "</table></body></html>")
            return self._send(200, page.encode(), "text/html")

    return ThreadingHTTPServer((routable_address() if host is None else host, port), H)


def _experiment_logdirs(exp_ids: List[str]) -> Dict[str, str]:
    from determined_clone_amd.common.api import Session

    info = _info.get_cluster_info()
    master = info.master_url if info else os.environ.get("DET_MASTER", "http://127.0.0.1:8080")
    s = Session(master)
    if info is not None:
        s.token = info.session_token
    cluster_id = s.get("/api/v1/master").get("cluster_id", "")
    out = {}
    for eid in exp_ids:
        cfg = s.get(f"/api/v1/experiments/{eid}")["config"]
        cs = cfg.get("checkpoint_storage") or {}
        root = cs.get("host_path") or cs.get("container_path") or ""
        if cs.get("storage_path"):
            root = os.path.join(root, cs["storage_path"])
        out[f"exp{eid}"] = os.path.join(root, "tensorboard", cluster_id, "experiment", str(eid))
    return out


def main(argv: Optional[List[str]] = None) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("experiment_ids", nargs="*")
    p.add_argument("--logdir", action="append", default=[])
    p.add_argument("--port", type=int, default=0)
    a = p.parse_args(argv)
    logdirs = {f"dir{i}": d for i, d in enumerate(a.logdir)}
    if a.experiment_ids:
        logdirs.update(_experiment_logdirs(a.experiment_ids))
    srv = make_server(logdirs, port=a.port)
    addr = f"http://{srv.server_address[0]}:{srv.server_address[1]}"
    print(f"serving tensorboard scalars at {addr}", flush=True)
    info = _info.get_cluster_info()
    if info is not None:
        try:
            from determined_clone_amd.common.api import Session

            s = Session(info.master_url, token=info.session_token)
            s.post(f"/api/v1/allocations/{info.allocation_id}/proxy_address", {"proxy_address": addr})
        except Exception as e:  # pragma: no cover - proxy registration is best effort
            print(f"could not register proxy address: {e}", file=sys.stderr)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    t.join()
    return 0


if __name__ == "__main__":
    sys.exit(main())
