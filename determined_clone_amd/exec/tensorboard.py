"""TensorBoard task (reference: `harness/determined/exec/tensorboard.py`, which fetches trial event
files from checkpoint storage and starts the TensorBoard server).

TensorBoard is not part of this image, so the task serves the event data itself. Each
experiment's event files (``tensorboard/<cluster>/experiment/<id>`` in its checkpoint storage --
shared_fs, directory, s3, gcs or azure) are synced into a local directory by the fetchers of
:mod:`determined_clone_amd.tensorboard.fetchers` (once before serving, then every few seconds in
a background thread, like the reference's fetch threads), parsed natively
(:func:`~determined_clone_amd.tensorboard.read_scalars` / ``read_images``) and served as
``/`` (HTML index with scalar tables and the latest image of each image tag), ``/data/runs``,
``/data/scalars?run=...&tag=...`` (TensorBoard's scalar route shape:
``[[wall_time, step, value], ...]``), ``/data/images?run=...&tag=...`` (``[{step, wall_time,
height, width, index}]``) and ``/data/image?run=...&tag=...&index=N`` (the PNG). Its address is
registered as the task's proxy.

Usage: ``python -m determined_clone_amd.exec.tensorboard EXP_ID... [--logdir DIR] [--port N]``.
"""
import argparse
import html
import json
import os
import sys
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional
from urllib.parse import parse_qs, quote, urlparse

from determined_clone_amd import _info
from determined_clone_amd.tensorboard import fetchers, read_images, read_scalars
from determined_clone_amd.util import proxy_secret_ok, routable_address


def collect(logdirs: Dict[str, str], reader=read_scalars) -> Dict[str, Dict[str, list]]:
    runs: Dict[str, Dict[str, list]] = {}
    for name, d in logdirs.items():
        for run, tags in reader(d).items():
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
            images = collect(logdirs, read_images)
            if u.path.endswith("/data/images") or u.path.endswith("/data/image"):
                series = images.get(q.get("run", ""), {}).get(q.get("tag", ""))
                if series is None:
                    return self._send(404, b'{"error": "no such run/tag"}', "application/json")
                if u.path.endswith("/data/images"):
                    meta = [{"step": st, "wall_time": w, "height": im["height"], "width": im["width"],
                             "index": i} for i, (st, w, im) in enumerate(series)]
                    return self._send(200, json.dumps(meta).encode(), "application/json")
                try:
                    return self._send(200, series[int(q.get("index", "-1"))][2]["png"], "image/png")
                except (ValueError, IndexError):
                    return self._send(404, b'{"error": "no such image"}', "application/json")
            rows = []
            for r, tags in sorted(runs.items()):
                for t, series in sorted(tags.items()):
                    last = series[-1]
                    rows.append(f"<tr><td>{html.escape(r)}</td><td>{html.escape(t)}</td><td>{len(series)}</td>"
                                f"<td>{last[0]}</td><td>{last[2]:.6g}</td></tr>")
            imgs = []
            for r, tags in sorted(images.items()):
                for t, series in sorted(tags.items()):
                    st = series[-1][0]
                    src = f"data/image?run={quote(r)}&tag={quote(t)}&index={len(series) - 1}"
                    imgs.append(f"<figure><img src=\"{html.escape(src)}\"><figcaption>{html.escape(r)} "
                                f"{html.escape(t)} step {st}</figcaption></figure>")
            page = ("<html><head><title>determined_clone_amd tensorboard</title></head><body>"
                    "<h2>Scalars</h2><table border=1><tr><th>run</th><th>tag</th><th>points</th>"
                    "<th>last step</th><th>last value</th></tr>" + "".join(rows) + "</table>"
                    + ("<h2>Images</h2>" + "".join(imgs) if imgs else "") + "</body></html>")
            return self._send(200, page.encode(), "text/html")

    return ThreadingHTTPServer((routable_address() if host is None else host, port), H)


def _experiment_sources(exp_ids: List[str]) -> List[Dict[str, Any]]:
    """Per experiment: its checkpoint storage config and the event-file path inside it."""
    from determined_clone_amd.common.api import Session

    info = _info.get_cluster_info()
    master = info.master_url if info else os.environ.get("DET_MASTER", "http://127.0.0.1:8080")
    s = Session(master)
    if info is not None:
        s.token = info.session_token
    cluster_id = s.get("/api/v1/master").get("cluster_id", "")
    out = []
    for eid in exp_ids:
        cfg = s.get(f"/api/v1/experiments/{eid}")["config"]
        out.append({"name": f"exp{eid}", "storage": cfg.get("checkpoint_storage") or {},
                    "path": f"tensorboard/{cluster_id}/experiment/{eid}"})
    return out


class SyncedLogdirs:
    """Fetchers for every (storage, path) source into one local directory, refreshed by a
    background thread every ``interval`` seconds (reference: TBFetchIterationThread)."""

    def __init__(self, sources: List[Dict[str, Any]], local_dir: str, interval: float = 5.0) -> None:
        self.local_dir = local_dir
        self.interval = interval
        self.logdirs: Dict[str, str] = {}
        self._fetchers: List[fetchers.Fetcher] = []
        by_storage: Dict[str, Dict[str, Any]] = {}
        for src in sources:
            key = json.dumps(src["storage"], sort_keys=True)
            ent = by_storage.setdefault(key, {"storage": src["storage"], "paths": []})
            ent["paths"].append(src["path"])
            self.logdirs[src["name"]] = os.path.join(local_dir, src["path"])
        for ent in by_storage.values():
            self._fetchers.append(fetchers.build(ent["storage"], ent["paths"], local_dir))
        self._stop = threading.Event()
        self.fetched = 0

    def fetch_once(self) -> int:
        n = 0
        for f in self._fetchers:
            try:
                n += f.fetch_new()
            except Exception as e:  # noqa: BLE001 - a storage hiccup must not kill the task
                print(f"tensorboard fetch failed: {e}", file=sys.stderr, flush=True)
        self.fetched += n
        return n

    def start(self) -> None:
        def loop() -> None:
            while not self._stop.wait(self.interval):
                self.fetch_once()
        threading.Thread(target=loop, daemon=True, name="tb-fetch").start()

    def stop(self) -> None:
        self._stop.set()


def main(argv: Optional[List[str]] = None) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("experiment_ids", nargs="*")
    p.add_argument("--logdir", action="append", default=[])
    p.add_argument("--port", type=int, default=0)
    a = p.parse_args(argv)
    logdirs = {f"dir{i}": d for i, d in enumerate(a.logdir)}
    if a.experiment_ids:
        import tempfile

        synced = SyncedLogdirs(_experiment_sources(a.experiment_ids), tempfile.mkdtemp(prefix="det-tb-"))
        n = synced.fetch_once()
        print(f"fetched {n} tensorboard file(s)", flush=True)
        synced.start()
        logdirs.update(synced.logdirs)
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
