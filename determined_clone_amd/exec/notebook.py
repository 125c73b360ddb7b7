"""Notebook task: a self-contained notebook server (Jupyter is not part of this image).

Reference: the master's NOTEBOOK tasks (`master/internal/api_notebook.go`, `command/`), which run
JupyterLab in the task container behind the master's proxy, with ``idle_timeout`` shutdown
(``notebook_idle_type``). This server keeps that contract -- launched as the NOTEBOOK task's
entrypoint, registers its address for ``/proxy/<task_id>/``, exits after ``--idle-timeout``
seconds without requests -- and speaks a Jupyter-shaped REST subset:

* ``GET  /api/contents`` / ``GET|PUT|DELETE /api/contents/<name>.ipynb`` -- nbformat-4 notebooks in
  the working directory (the task's context directory);
* ``POST /api/kernels`` -> ``{"id"}``; ``GET /api/kernels``; ``DELETE /api/kernels/<id>``;
  ``POST /api/kernels/<id>/interrupt`` (SIGINT);
* ``POST /api/kernels/<id>/execute {"code"}`` -> ``{"execution_count", "outputs": [...]}`` with
  nbformat output dicts (``stream``, ``execute_result`` text/plain, ``error`` with traceback);
* ``GET /`` -- a minimal browser UI (cells, run, save) over the same API.

A kernel is a child Python process (``--kernel`` mode) executing cells in one persistent
namespace; like IPython, a trailing expression's value becomes the cell's ``execute_result``.
The task's environment (``DET_*``, GPUs) is the kernel's, so ``determined_clone_amd`` Core API /
client SDK calls work from cells.
"""
import argparse
import ast
import io
import json
import os
import signal
import subprocess
import sys
import threading
import time
import traceback
import uuid
from contextlib import redirect_stderr, redirect_stdout
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional

from determined_clone_amd.util import proxy_secret_ok, routable_address

PAGE = """<!doctype html><html><head><meta charset="utf-8"><title>notebook</title>
<style>body{font-family:monospace;margin:2em}textarea{width:100%;height:6em}pre{background:#f4f4f4;padding:.5em}</style>
</head><body><h3>determined-clone-amd notebook</h3>
<div>notebook: <input id="nb" value="Untitled.ipynb"> <button onclick="load()">open</button>
<button onclick="save()">save</button> <button onclick="add()">+ cell</button></div><div id="cells"></div>
<script>
const base = location.pathname.replace(/\\/$/, '');
let kernel = null;
async function api(m, p, b) { const r = await fetch(base + p, {method: m, headers: {'Content-Type': 'application/json'},
  body: b ? JSON.stringify(b) : undefined}); return r.json(); }
function add(src) { const d = document.createElement('div');
  d.innerHTML = '<textarea></textarea><button>run</button><pre></pre>';
  d.querySelector('textarea').value = src || '';
  d.querySelector('button').onclick = () => run(d); document.getElementById('cells').appendChild(d); }
async function run(d) { if (!kernel) kernel = (await api('POST', '/api/kernels')).id;
  const r = await api('POST', '/api/kernels/' + kernel + '/execute', {code: d.querySelector('textarea').value});
  d.querySelector('pre').textContent = r.outputs.map(o => o.text || (o.data && o.data['text/plain']) ||
    (o.traceback || []).join('\\n')).join(''); }
async function load() { const nb = await api('GET', '/api/contents/' + document.getElementById('nb').value);
  document.getElementById('cells').innerHTML = ''; (nb.content.cells || []).forEach(c => add([].concat(c.source).join(''))); }
async function save() { const cells = [...document.querySelectorAll('#cells textarea')].map(t => ({cell_type: 'code',
  source: t.value, metadata: {}, outputs: [], execution_count: null}));
  await api('PUT', '/api/contents/' + document.getElementById('nb').value, {content: {nbformat: 4, nbformat_minor: 5,
  metadata: {}, cells: cells}}); }
add();
</script></body></html>"""


# ----------------------------------------------------------------------------- kernel process
def _run_cell(code: str, ns: Dict[str, Any]) -> List[Dict[str, Any]]:
    out, err = io.StringIO(), io.StringIO()
    outputs: List[Dict[str, Any]] = []
    result = None
    try:
        tree = ast.parse(code, mode="exec")
        last = tree.body[-1] if tree.body and isinstance(tree.body[-1], ast.Expr) else None
        if last is not None:
            tree.body = tree.body[:-1]
        with redirect_stdout(out), redirect_stderr(err):
            exec(compile(tree, "<cell>", "exec"), ns)
            if last is not None:
                result = eval(compile(ast.Expression(last.value), "<cell>", "eval"), ns)
    except KeyboardInterrupt:
        outputs.append({"output_type": "error", "ename": "KeyboardInterrupt", "evalue": "",
                        "traceback": ["KeyboardInterrupt"]})
    except BaseException as e:  # noqa: BLE001 - a cell may raise anything
        outputs.append({"output_type": "error", "ename": type(e).__name__, "evalue": str(e),
                        "traceback": traceback.format_exception(type(e), e, e.__traceback__)})
    if out.getvalue():
        outputs.insert(0, {"output_type": "stream", "name": "stdout", "text": out.getvalue()})
    if err.getvalue():
        outputs.insert(1 if out.getvalue() else 0, {"output_type": "stream", "name": "stderr", "text": err.getvalue()})
    if result is not None:
        outputs.append({"output_type": "execute_result", "data": {"text/plain": repr(result)}, "metadata": {}})
    return outputs


def kernel_main() -> int:
    """JSON-lines REPL on stdin/stdout: {"code"} -> {"outputs"}."""
    ns: Dict[str, Any] = {"__name__": "__main__"}
    signal.signal(signal.SIGINT, signal.default_int_handler)
    real_out = sys.stdout
    for line in sys.stdin:
        try:
            req = json.loads(line)
        except ValueError:
            continue
        outs = _run_cell(req.get("code", ""), ns)
        real_out.write(json.dumps({"outputs": outs}) + "\n")
        real_out.flush()
    return 0


class Kernel:
    def __init__(self, cwd: str) -> None:
        self.id = str(uuid.uuid4())
        self.proc = subprocess.Popen([sys.executable, "-u", "-m", "determined_clone_amd.exec.notebook", "--kernel"],
                                     stdin=subprocess.PIPE, stdout=subprocess.PIPE, cwd=cwd, text=True)
        self.count = 0
        self.lock = threading.Lock()

    def execute(self, code: str) -> Dict[str, Any]:
        with self.lock:
            self.count += 1
            self.proc.stdin.write(json.dumps({"code": code}) + "\n")
            self.proc.stdin.flush()
            line = self.proc.stdout.readline()
            if not line:
                return {"execution_count": self.count, "status": "dead",
                        "outputs": [{"output_type": "error", "ename": "KernelDied", "evalue": "",
                                     "traceback": ["the kernel process exited"]}]}
            return {"execution_count": self.count, "status": "ok", **json.loads(line)}

    def interrupt(self) -> None:
        if self.proc.poll() is None:
            self.proc.send_signal(signal.SIGINT)

    def shutdown(self) -> None:
        if self.proc.poll() is None:
            self.proc.kill()
            self.proc.wait()


# ----------------------------------------------------------------------------- server
class NotebookServer:
    def __init__(self, root: str, host: Optional[str] = None, port: int = 0) -> None:
        self.root = os.path.abspath(root)
        self.kernels: Dict[str, Kernel] = {}
        self.last_activity = time.time()
        srv = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"
            disable_nagle_algorithm = True  # headers + body writes: no delayed-ACK stall

            def log_message(self, *a: Any) -> None:
                pass

            def _send(self, code: int, obj: Any, ctype: str = "application/json") -> None:
                data = obj.encode() if isinstance(obj, str) else json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def _body(self) -> Any:
                n = int(self.headers.get("Content-Length") or 0)
                return json.loads(self.rfile.read(n)) if n else {}

            def _go(self, method: str) -> None:
                # kernels run arbitrary code: on a cluster only the master's owner-checked
                # /proxy/ route (which attaches the task's secret) may reach them
                if not proxy_secret_ok(self.headers):
                    self._body()
                    return self._send(403, {"message": "requests must come through the master's /proxy/ route"})
                srv.last_activity = time.time()
                try:
                    code, obj, *ct = srv.handle(method, self.path.split("?")[0], self._body())
                except (KeyError, FileNotFoundError) as e:
                    code, obj, ct = 404, {"message": f"not found: {e}"}, []
                except ValueError as e:
                    code, obj, ct = 400, {"message": str(e)}, []
                self._send(code, obj, *ct)

            def do_GET(self) -> None:
                self._go("GET")

            def do_POST(self) -> None:
                self._go("POST")

            def do_PUT(self) -> None:
                self._go("PUT")

            def do_DELETE(self) -> None:
                self._go("DELETE")

        self.httpd = ThreadingHTTPServer((routable_address() if host is None else host, port), H)
        self.httpd.daemon_threads = True

    def _nb_path(self, name: str) -> str:
        p = os.path.abspath(os.path.join(self.root, name))
        if not p.startswith(self.root + os.sep) or not p.endswith(".ipynb"):
            raise ValueError(f"bad notebook path {name!r}")
        return p

    def handle(self, method: str, path: str, body: Any):
        if path in ("/", "/lab", "/tree") and method == "GET":
            return 200, PAGE, "text/html; charset=utf-8"
        if path == "/api/status":
            return 200, {"kernels": len(self.kernels), "last_activity": self.last_activity}
        if path == "/api/contents" and method == "GET":
            items = [{"name": f, "path": f, "type": "notebook"} for f in sorted(os.listdir(self.root))
                     if f.endswith(".ipynb")]
            return 200, {"type": "directory", "content": items}
        if path.startswith("/api/contents/"):
            name = path[len("/api/contents/"):]
            p = self._nb_path(name)
            if method == "GET":
                with open(p) as f:
                    return 200, {"name": name, "type": "notebook", "content": json.load(f)}
            if method == "PUT":
                nb = body.get("content") or {}
                if nb.get("nbformat") != 4 or not isinstance(nb.get("cells"), list):
                    raise ValueError("content must be an nbformat-4 notebook")
                with open(p, "w") as f:
                    json.dump(nb, f, indent=1)
                return 200, {"name": name, "type": "notebook"}
            if method == "DELETE":
                os.remove(p)
                return 204, {}
        if path == "/api/kernels":
            if method == "POST":
                k = Kernel(self.root)
                self.kernels[k.id] = k
                return 201, {"id": k.id, "name": "python3"}
            return 200, [{"id": k, "name": "python3"} for k in self.kernels]
        if path.startswith("/api/kernels/"):
            parts = path.split("/")
            k = self.kernels[parts[3]]
            action = parts[4] if len(parts) > 4 else ""
            if method == "DELETE" and not action:
                k.shutdown()
                self.kernels.pop(k.id, None)
                return 204, {}
            if action == "execute" and method == "POST":
                return 200, k.execute(str(body.get("code", "")))
            if action == "interrupt" and method == "POST":
                k.interrupt()
                return 204, {}
        return 404, {"message": f"no route {method} {path}"}

    def serve(self, idle_timeout: float = 0.0) -> None:
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()
        try:
            while True:
                time.sleep(1.0)
                if idle_timeout and time.time() - self.last_activity > idle_timeout:
                    print(f"notebook idle for {idle_timeout:.0f}s: shutting down", flush=True)
                    return
        finally:
            for k in list(self.kernels.values()):
                k.shutdown()
            self.httpd.shutdown()


def main(argv: Optional[List[str]] = None) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--kernel", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--port", type=int, default=0)
    p.add_argument("--root", default=os.environ.get("DET_CONTEXT_DIR") or os.getcwd())
    p.add_argument("--idle-timeout", type=float, default=float(os.environ.get("DET_NOTEBOOK_IDLE_TIMEOUT", "0")))
    a = p.parse_args(argv)
    if a.kernel:
        return kernel_main()
    srv = NotebookServer(a.root, port=a.port)
    addr = f"http://{srv.httpd.server_address[0]}:{srv.httpd.server_address[1]}"
    print(f"notebook server at {addr} (root {a.root})", flush=True)
    from determined_clone_amd import _info

    info = _info.get_cluster_info()
    if info is not None:
        from determined_clone_amd.common.api import Session

        try:
            Session(info.master_url, token=info.session_token).post(
                f"/api/v1/allocations/{info.allocation_id}/proxy_address", {"proxy_address": addr})
        except Exception as e:  # pragma: no cover - proxy registration is best effort
            print(f"could not register proxy address: {e}", file=sys.stderr)
    srv.serve(a.idle_timeout)
    return 0


if __name__ == "__main__":
    sys.exit(main())
