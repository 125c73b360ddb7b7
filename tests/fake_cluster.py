"""In-process fakes of external cluster managers for the CPU test tier:

* :class:`FakeKubeAPI` -- a Kubernetes API server subset (nodes, pods CRUD with label selectors,
  bearer-token auth) plus a "kubelet" that really runs each pod's container command as a local
  process (downward-API env resolved), moving the pod Pending -> Running -> Succeeded/Failed;
* :func:`install_fake_slurm` / :func:`install_fake_pbs` -- ``sbatch``/``squeue``/``sacct``/
  ``scancel``/``sinfo``/``srun`` and ``qsub``/``qstat``/``qdel`` scripts that run the batch script
  locally as a 1-node job;
* :class:`FakeEC2` / :class:`FakeGCE` -- EC2 Query API (SigV4 header checked) and Compute Engine
  REST subsets keeping an instance table.
"""
import json
import os
import signal
import stat
import subprocess
import sys
import threading
import time
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional


class _Server:
    def __init__(self, handler_cls: type) -> None:
        self.httpd = ThreadingHTTPServer(("127.0.0.1", 0), handler_cls)
        self.httpd.daemon_threads = True
        self.url = f"http://127.0.0.1:{self.httpd.server_address[1]}"
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()


def _json_handler(fake: Any) -> type:
    class H(BaseHTTPRequestHandler):
        def log_message(self, *a: Any) -> None:
            pass

        def _body(self) -> bytes:
            n = int(self.headers.get("Content-Length") or 0)
            return self.rfile.read(n) if n else b""

        def _send(self, code: int, obj: Any, ctype: str = "application/json") -> None:
            data = obj if isinstance(obj, bytes) else json.dumps(obj).encode()
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

        def _go(self, method: str) -> None:
            u = urllib.parse.urlsplit(self.path)
            q = dict(urllib.parse.parse_qsl(u.query))
            code, obj, *ct = fake.handle(method, u.path, q, self._body(), self.headers)
            self._send(code, obj, *ct)

        def do_GET(self) -> None:
            self._go("GET")

        def do_POST(self) -> None:
            self._go("POST")

        def do_DELETE(self) -> None:
            self._go("DELETE")

    return H


# ============================================================================ Kubernetes
class FakeKubeAPI:
    def __init__(self, nodes: List[Dict[str, Any]], token: str = "secret-token",
                 env: Optional[Dict[str, str]] = None) -> None:
        self.nodes = nodes
        self.token = token
        self.pods: Dict[str, Dict[str, Any]] = {}
        self.procs: Dict[str, subprocess.Popen] = {}
        self.created: List[Dict[str, Any]] = []
        self.deleted: List[str] = []
        self.env = env or {}
        self.lock = threading.Lock()
        self.server = _Server(_json_handler(self))
        self.url = self.server.url

    @staticmethod
    def node(name: str, gpus: int = 8, cpu: str = "64", ready: bool = True,
             labels: Optional[Dict[str, str]] = None, unschedulable: bool = False) -> Dict[str, Any]:
        return {"metadata": {"name": name, "labels": labels or {}},
                "spec": {"unschedulable": unschedulable},
                "status": {"allocatable": {"cpu": cpu, "amd.com/gpu": str(gpus), "memory": "2Ti"},
                           "conditions": [{"type": "Ready", "status": "True" if ready else "False"}],
                           "addresses": [{"type": "InternalIP", "address": "127.0.0.1"}]}}

    def handle(self, method: str, path: str, q: Dict[str, str], body: bytes, headers: Any):
        if headers.get("Authorization") != f"Bearer {self.token}":
            return 401, {"kind": "Status", "message": "Unauthorized"}
        parts = path.strip("/").split("/")
        if path == "/api/v1/nodes" and method == "GET":
            return 200, {"kind": "NodeList", "items": self.nodes}
        if len(parts) >= 5 and parts[:2] == ["api", "v1"] and parts[2] == "namespaces" and parts[4] == "pods":
            ns = parts[3]
            if len(parts) == 5 and method == "GET":
                sel = dict(kv.split("=", 1) for kv in q.get("labelSelector", "").split(",") if "=" in kv)
                with self.lock:
                    items = [p for p in self.pods.values() if p["metadata"]["namespace"] == ns and
                             all(p["metadata"].get("labels", {}).get(k) == v for k, v in sel.items())]
                return 200, {"kind": "PodList", "items": json.loads(json.dumps(items))}
            if len(parts) == 5 and method == "POST":
                pod = json.loads(body)
                name = pod["metadata"]["name"]
                with self.lock:
                    if name in self.pods:
                        return 409, {"kind": "Status", "message": "AlreadyExists"}
                    pod["metadata"]["namespace"] = ns
                    pod["status"] = {"phase": "Pending"}
                    self.pods[name] = pod
                    self.created.append(json.loads(json.dumps(pod)))
                threading.Thread(target=self._kubelet, args=(name,), daemon=True).start()
                return 201, pod
            if len(parts) == 6 and method == "DELETE":
                name = parts[5]
                with self.lock:
                    pod = self.pods.pop(name, None)
                    proc = self.procs.pop(name, None)
                    self.deleted.append(name)
                if pod is None:
                    return 404, {"kind": "Status", "message": "NotFound"}
                if proc is not None and proc.poll() is None:
                    try:
                        os.killpg(proc.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
                return 200, {"kind": "Status", "status": "Success"}
        return 404, {"kind": "Status", "message": f"no route {method} {path}"}

    def _kubelet(self, name: str) -> None:
        with self.lock:
            pod = self.pods.get(name)
        if pod is None:
            return
        c = pod["spec"]["containers"][0]
        env = dict(os.environ)
        env.update(self.env)
        for e in c.get("env", []):
            if "value" in e:
                env[e["name"]] = e["value"]
            else:
                f = e["valueFrom"]["fieldRef"]["fieldPath"]
                env[e["name"]] = pod["spec"].get("nodeName", "") if f == "spec.nodeName" else "127.0.0.1"
        cmd = list(c["command"])
        if cmd[0] in ("python", "python3"):
            cmd[0] = sys.executable
        proc = subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                                start_new_session=True)
        with self.lock:
            if name not in self.pods:
                os.killpg(proc.pid, signal.SIGKILL)
                return
            self.procs[name] = proc
            self.pods[name]["status"] = {"phase": "Running", "podIP": "127.0.0.1"}
        code = proc.wait()
        with self.lock:
            p = self.pods.get(name)
            if p is not None:
                p["status"] = {"phase": "Succeeded" if code == 0 else "Failed", "containerStatuses": [
                    {"name": c["name"], "state": {"terminated": {"exitCode": code}}}]}

    def stop(self) -> None:
        with self.lock:
            procs = list(self.procs.values())
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
        self.server.stop()


# ============================================================================ Slurm / PBS
_SLURM = r'''#!{py}
import json, os, subprocess, sys, time
D = os.environ["FAKE_HPC_DIR"]
tool = os.path.basename(sys.argv[0])
def jobs():
    out = {{}}
    for f in os.listdir(D):
        if f.endswith(".json"):
            with open(os.path.join(D, f)) as fh:
                out[f[:-5]] = json.load(fh)
    return out
def save(jid, j):
    tmp = os.path.join(D, jid + ".tmp")
    with open(tmp, "w") as fh:
        json.dump(j, fh)
    os.replace(tmp, os.path.join(D, jid + ".json"))
if len(sys.argv) > 3 and sys.argv[1] == "--reap":
    # detached reaper: run the job script in its own process group and record its exit code
    jid, script = sys.argv[2], sys.argv[3]
    env = dict(os.environ, SLURM_JOB_ID=jid, SLURM_NODEID="0", SLURM_JOB_NUM_NODES="1",
               PBS_JOBID=jid)
    p = subprocess.Popen(["bash", script], env=env, stdout=open(os.path.join(D, jid + ".out"), "w"),
                         stderr=subprocess.STDOUT, start_new_session=True)
    if jobs().get(jid, {{}}).get("state") == "CANCELLED":
        os.killpg(p.pid, 9)
    save(jid, {{"state": "RUNNING", "pid": p.pid, "code": None}})
    code = p.wait()
    if jobs().get(jid, {{}}).get("state") != "CANCELLED":
        save(jid, {{"state": "COMPLETED" if code == 0 else "FAILED", "pid": p.pid, "code": code}})
elif tool in ("sbatch", "qsub"):
    script = sys.argv[-1]
    jid = str(1000 + len([f for f in os.listdir(D) if f.endswith(".json")]))
    with open(os.path.join(D, "submitted.log"), "a") as fh:
        fh.write(jid + " " + script + "\n")
    save(jid, {{"state": "PENDING", "pid": None, "code": None}})
    subprocess.Popen([sys.executable, sys.argv[0], "--reap", jid, script], start_new_session=True,
                     stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    print(jid + (";cluster" if tool == "sbatch" else ".fakepbs"))
elif tool == "squeue":
    ids = sys.argv[sys.argv.index("-j") + 1].split(",")
    for jid, j in jobs().items():
        if jid in ids and j["state"] in ("PENDING", "RUNNING"):
            print(jid + "|" + j["state"])
elif tool == "sacct":
    ids = sys.argv[sys.argv.index("-j") + 1].split(",")
    for jid, j in jobs().items():
        if jid in ids:
            print(jid + "|" + j["state"] + "|" + str(j["code"] if j["code"] is not None else 0) + ":0")
elif tool in ("scancel", "qdel"):
    jid = sys.argv[-1].split(".")[0]
    j = jobs()[jid]
    try:
        if j["pid"]:
            os.killpg(j["pid"], 15)
    except ProcessLookupError:
        pass
    save(jid, {{"state": "CANCELLED", "pid": j["pid"], "code": 143}})
elif tool == "sinfo":
    print("mi355x|2|gpu:mi355x:8")
    print("debug|1|(null)")
elif tool == "qstat":
    if "-Q" in sys.argv:
        print("Queue Max Tot"); print("----- --- ---"); print("workq 0 0")
    else:
        out = {{}}
        for jid, j in jobs().items():
            st = {{"RUNNING": "R", "PENDING": "Q"}}.get(j["state"], "F")
            d = {{"job_state": st}}
            if st == "F":
                d["Exit_status"] = j["code"] if j["code"] is not None else 0
            out[jid + ".fakepbs"] = d
        print(json.dumps({{"Jobs": out}}))
elif tool == "srun":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    sys.exit(subprocess.call(args))
'''


def install_fake_hpc(bindir: str, statedir: str) -> Dict[str, str]:
    """Write the fake Slurm + PBS CLI into ``bindir``; returns env additions (PATH, state dir)."""
    os.makedirs(bindir, exist_ok=True)
    os.makedirs(statedir, exist_ok=True)
    src = _SLURM.format(py=sys.executable)
    for tool in ("sbatch", "squeue", "sacct", "scancel", "sinfo", "srun", "qsub", "qstat", "qdel"):
        p = os.path.join(bindir, tool)
        with open(p, "w") as f:
            f.write(src)
        os.chmod(p, os.stat(p).st_mode | stat.S_IEXEC | stat.S_IXGRP | stat.S_IXOTH)
    return {"PATH": bindir + os.pathsep + os.environ.get("PATH", ""), "FAKE_HPC_DIR": statedir}


# ============================================================================ EC2 / GCE
class FakeEC2:
    def __init__(self, access_key: str = "AKIDEXAMPLE") -> None:
        self.access_key = access_key
        self.instances: Dict[str, Dict[str, Any]] = {}
        self.calls: List[Dict[str, str]] = []
        self.server = _Server(_json_handler(self))
        self.url = self.server.url + "/"
        self._n = 0

    def handle(self, method: str, path: str, q: Dict[str, str], body: bytes, headers: Any):
        auth = headers.get("Authorization") or ""
        if not auth.startswith(f"AWS4-HMAC-SHA256 Credential={self.access_key}/") or "/ec2/aws4_request" not in auth:
            return 403, b"<Response><Errors><Error><Code>AuthFailure</Code></Error></Errors></Response>", "text/xml"
        p = dict(urllib.parse.parse_qsl(body.decode()))
        self.calls.append(p)
        a = p.get("Action")
        if a == "DescribeInstances":
            want_pool = p.get("Filter.2.Value.1")
            items = "".join(
                f"<item><instanceId>{i}</instanceId><instanceState><code>16</code><name>{d['state']}</name>"
                f"</instanceState><launchTime>{d['launch']}</launchTime></item>"
                for i, d in self.instances.items() if d["pool"] == want_pool and d["state"] != "terminated")
            xml = (f'<DescribeInstancesResponse xmlns="http://ec2.amazonaws.com/doc/2016-11-15/">'
                   f"<reservationSet><item><instancesSet>{items}</instancesSet></item></reservationSet>"
                   f"</DescribeInstancesResponse>")
            return 200, xml.encode(), "text/xml"
        if a == "RunInstances":
            tags = {p[k]: p[k[:-3] + "Value"] for k in p if k.startswith("TagSpecification.1.Tag.") and k.endswith(".Key")}
            for _ in range(int(p["MaxCount"])):
                self._n += 1
                iid = f"i-{self._n:08x}"
                self.instances[iid] = {"state": "pending", "pool": tags.get("determined-resource-pool"),
                                       "tags": tags, "user_data": p.get("UserData"),
                                       "launch": time.strftime("%Y-%m-%dT%H:%M:%S.000Z", time.gmtime())}
            return 200, b'<RunInstancesResponse xmlns="http://ec2.amazonaws.com/doc/2016-11-15/"/>', "text/xml"
        if a == "TerminateInstances":
            for k, v in p.items():
                if k.startswith("InstanceId.") and v in self.instances:
                    self.instances[v]["state"] = "terminated"
            return 200, b'<TerminateInstancesResponse xmlns="http://ec2.amazonaws.com/doc/2016-11-15/"/>', "text/xml"
        return 400, b"<Response/>", "text/xml"

    def stop(self) -> None:
        self.server.stop()


class FakeGCE:
    def __init__(self, token: str = "gce-token") -> None:
        self.token = token
        self.instances: Dict[str, Dict[str, Any]] = {}
        self.bodies: List[Any] = []
        self.server = _Server(_json_handler(self))
        self.url = self.server.url
        self._n = 0

    def handle(self, method: str, path: str, q: Dict[str, str], body: bytes, headers: Any):
        if headers.get("Authorization") != f"Bearer {self.token}":
            return 401, {"error": "unauthorized"}
        if path.endswith("/instances") and method == "GET":
            return 200, {"items": [dict(name=n, **{k: v for k, v in d.items() if k != "labels"})
                                   for n, d in self.instances.items() if d["status"] != "DELETED"
                                   and all(f"labels.{k} = {v}" in q.get("filter", "")
                                           for k, v in d["labels"].items() if k.startswith("determined-"))]}
        if path.endswith("/instances/bulkInsert") and method == "POST":
            b = json.loads(body)
            self.bodies.append(b)
            for _ in range(int(b["count"])):
                self._n += 1
                name = b["namePattern"].replace("#" * 8, f"{self._n:08d}")
                self.instances[name] = {"status": "PROVISIONING",
                                        "labels": b["instanceProperties"]["labels"],
                                        "creationTimestamp": "2026-10-16T00:00:00.000-07:00"}
            return 200, {"kind": "compute#operation", "status": "RUNNING"}
        if "/instances/" in path and method == "DELETE":
            name = path.rsplit("/", 1)[1]
            if name in self.instances:
                self.instances[name]["status"] = "DELETED"
                return 200, {"kind": "compute#operation"}
            return 404, {"error": "not found"}
        return 404, {"error": "no route"}

    def stop(self) -> None:
        self.server.stop()
